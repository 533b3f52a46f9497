"""Diagnostic: per geom-pair contact lists, GPU fp64 forward_debug vs oracle, on the mesh-contact
fixture of tests/test_step_gpu.py."""
import os
import sys
from collections import Counter

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
from test_step_gpu import _dev, mesh_states  # noqa: E402

D = _lib.DBG
eng = get_engine()
m = eng.model
st = mesh_states(m)
dbg = eng.forward_debug(_dev(st, torch.float64)).cpu().numpy()
name = lambda g: str(m.names_geom[g]) or str(g)
for b in range(st["qpos"].shape[0]):
    f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["contact", "ncon"])
    n = int(f["ncon"][0])
    c = f["contact"].reshape(n, 30)
    ng = int(dbg[b][D["COUNTS"]])
    gq = [dbg[b][D["CON"] + 16 * i:D["CON"] + 16 * (i + 1)] for i in range(ng)]
    ref = Counter((int(r[27]), int(r[28])) for r in c)
    gpu = Counter((int(q[13]), int(q[14])) for q in gq)
    if ref == gpu:
        for i, (r, q) in enumerate(zip(c, gq)):
            if abs(r[12] - q[12]) > 1e-9 or np.abs(r[:3] - q[:3]).max() > 1e-9:
                print(f"env {b} con {i} {name(int(r[27]))}/{name(int(r[28]))} types {m.geom_type[int(r[27])]}/{m.geom_type[int(r[28])]}"
                      f" ref d {r[12]:.6e} n {np.round(r[3:6], 4)} p {np.round(r[:3], 4)} | gpu d {q[12]:.6e} n {np.round(q[3:6], 4)} p {np.round(q[:3], 4)}")
        continue
    print(f"env {b}: gpu {ng} ref {n}")
    for k in sorted(set(ref) | set(gpu)):
        if ref[k] != gpu[k]:
            print("  ", name(k[0]), name(k[1]), m.geom_type[k[0]], m.geom_type[k[1]], "gpu", gpu[k], "ref", ref[k])
            for r in c:
                if (int(r[27]), int(r[28])) == k:
                    print("      ref", np.round(r[:3], 5), f"{r[12]:.3e}", np.round(r[3:6], 3))
            for q in gq:
                if (int(q[13]), int(q[14])) == k:
                    print("      gpu", np.round(q[:3], 5), f"{q[12]:.3e}", np.round(q[3:6], 3))
