"""Knife-edge account per contact pair (GPU): for every env of the fp32
parity fixtures whose fp32 kernel's contact count differs from the oracle's on the same
(fp32-rounded) state, the geom pairs whose contact counts differ, with each side's contact depths
in that pair, and the oracle's counts for that pair on the one-ulp candidates of
tests/test_step_gpu.py::_backward_errors -- which pair flips, how close its contacts sit to the
margin, and whether a perturbed oracle lands on the kernel's count.
usage: python tools/knife_edge_pairs.py [fixture ...]   (mesh_scene pressed pads pile; default all)"""
import collections
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402
import box_states as BS  # noqa: E402
import physics_states as PS  # noqa: E402
import test_step_gpu as T  # noqa: E402

D = _lib.DBG


def fixtures(m, names):
    out = {}
    if "mesh_scene" in names:
        out["mesh_scene"] = T.mesh_states(m)
    if "pressed" in names or "pile" in names:
        n = 12
        st = PS.reset_states(n, seed=11, model=m)
        st["qpos"][:, 7:9] = -np.linspace(0.001, 0.004, n)[:, None]
        st["ctrl"][:, -2:] = 0.0
        st["qvel"] += np.random.default_rng(5).normal(size=st["qvel"].shape) * 0.02
        if "pressed" in names:
            out["pressed"] = st
        if "pile" in names:
            p = PS.copy_state(st)
            PS.cube_pile(p["qpos"], m)
            out["pile"] = p
    if "pads" in names:
        idx, st = BS.box_states(m)
        out["pads"] = {k: v[[idx["pads"]]] for k, v in st.items()}
    return out


def pairs(con, gcols):
    c = collections.defaultdict(list)
    for row in con:
        c[(int(row[gcols[0]]), int(row[gcols[1]]))].append(float(row[12]))
    return c


def main():
    names = sys.argv[1:] or ["mesh_scene", "pressed", "pads", "pile"]
    m = load_model()
    eng = get_engine()
    gname = lambda g: str(m.names_geom[g]) or f"geom{g}"
    for label, st0 in fixtures(m, names).items():
        st = T._round32(st0)
        B = st["qpos"].shape[0]
        dbg = eng.forward_debug(T._dev(st, torch.float32)).cpu().numpy()
        cands = T._perturbed_states(st, 8)
        print(f"== {label}: {B} envs", flush=True)
        for b in range(B):
            kn = int(dbg[b, D["COUNTS"]])
            kc = dbg[b, D["CON"]:D["CON"] + 16 * kn].reshape(kn, 16)
            orc = []
            for p in cands:
                f = O.forward_fields({k: p[k][b] for k in O.STATE_KEYS}, ["ncon", "contact"], model=m)
                n = int(f["ncon"][0])
                orc.append(pairs(f["contact"].reshape(n, 30), (27, 28)))
            on = [sum(len(v) for v in o.values()) for o in orc]
            if on[0] == kn and all(x == kn for x in on):
                continue
            kp = pairs(kc, (13, 14))
            print(f"env {b}: kernel {kn} contacts; oracle candidates {on}", flush=True)
            for pr in sorted(set(kp) | set().union(*[set(o) for o in orc])):
                counts = [len(o.get(pr, [])) for o in orc]
                if len(kp.get(pr, [])) == counts[0] and all(c == counts[0] for c in counts):
                    continue
                kd = np.round(np.array(kp.get(pr, [])) * 1e3, 4)
                od = np.round(np.array(orc[0].get(pr, [])) * 1e3, 4)
                print(f"   pair {gname(pr[0])} / {gname(pr[1])} ({m.geom_type[pr[0]]}, {m.geom_type[pr[1]]}): kernel "
                      f"{len(kp.get(pr, []))} depths(mm) {kd.tolist()}; oracle {counts[0]} depths(mm) {od.tolist()}; "
                      f"counts over candidates {counts}", flush=True)


if __name__ == "__main__":
    main()
