"""The ctypes mirrors of include/pnp.h's structs (pnp_amd/_lib.py: PnpState, PnpEnvParams,
PnpEnvState, PnpEnvOut, PnpTqcDesc, PnpTqcBatch, PnpTqcReplay) against the C compiler's layout:
gcc compiles a probe that prints every field's offsetof and the struct's sizeof, and each must
equal the ctypes field's offset and the ctypes sizeof (pnp_model_desc has its own runtime check,
pnp_model_desc_size).  CPU only."""
import ctypes as C
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_struct_layouts_match_c(tmp_path):
    from pnp_amd import _lib
    structs = {"pnp_state": _lib.PnpState, "pnp_env_params": _lib.PnpEnvParams, "pnp_env_state": _lib.PnpEnvState,
               "pnp_env_out": _lib.PnpEnvOut, "pnp_tqc_desc": _lib.PnpTqcDesc, "pnp_tqc_batch": _lib.PnpTqcBatch,
               "pnp_tqc_replay": _lib.PnpTqcReplay}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pnp.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            s, f, v = ln.split()
            got[(s, f)] = int(v)
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)
