"""Diagnostic: find the first sub-step where the fp64 step kernel and the oracle diverge (> 1e-10)
from the env's post-reset state, and dump both sides' contacts / solver info there."""
import os
import sys
from collections import Counter

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402

D = _lib.DBG
B = 4
g = BatchedFrankaShelfPNPEnv(B, dtype=torch.float64, autoreset=False)
g.reset()
a = np.random.default_rng(10).uniform(-1, 1, size=(B, 7))
a[:, 6] = 1.0
g.step(torch.as_tensor(a))          # sets ctrl / mocap; now step sub-step by sub-step
m = g.model
st = {k: v.cpu().numpy().astype(np.uint32 if k == "warn" else np.float64) for k, v in g.state.items()}
gs = {k: v.clone() for k, v in g.state.items()}
for n in range(1, 251):
    prev_ref = {k: v.copy() for k, v in st.items()}
    prev_g = {k: v.clone() for k, v in gs.items()}
    O.step(st, nsub=1, nthreads=8)
    g.engine.step(gs, 1)
    dv = np.abs(gs["qvel"].cpu().numpy() - st["qvel"]).max(1)
    if dv.max() > 1e-9:
        b = int(dv.argmax())
        k = int(np.abs(gs["qvel"].cpu().numpy()[b] - st["qvel"][b]).argmax())
        print(f"diverged at sub-step {n}, env {b}, dof {k} ({m.names_jnt[m.dof_jntid[k]]}): dqvel {dv[b]:.2e}")
        row = {kk: prev_ref[kk][b] for kk in O.STATE_KEYS}
        f = O.forward_fields(row, ["ncon", "nefc", "contact", "solver_iter", "efc_force"])
        dbg = g.engine.forward_debug({kk: v[b:b + 1].contiguous() for kk, v in prev_g.items()}).cpu().numpy()[0]
        nc = int(f["ncon"][0])
        c = f["contact"].reshape(nc, 30)
        print(" oracle ncon", nc, "nefc", int(f["nefc"][0]), "iters", int(f["solver_iter"][0]))
        print(" gpu    ncon", int(dbg[D["COUNTS"]]), "nefc", int(dbg[D["COUNTS"] + 1]), "iters", int(dbg[D["COUNTS"] + 2]))
        for i in range(max(nc, int(dbg[D["COUNTS"]]))):
            q = dbg[D["CON"] + 16 * i:D["CON"] + 16 * (i + 1)]
            r = c[i] if i < nc else None
            print(f"  {i:2d} ref", (m.names_geom[int(r[27])], m.names_geom[int(r[28])], np.round(r[:3], 5), f"{r[12]:.3e}", np.round(r[3:6], 3)) if r is not None else None)
            print(f"     gpu", (m.names_geom[int(q[13])], m.names_geom[int(q[14])], np.round(q[:3], 5), f"{q[12]:.3e}", np.round(q[3:6], 3)))
        break
else:
    print("no divergence")
