"""Diagnostic: fp32 qacc_smooth error per dof vs the oracle, against what an fp32 Cholesky of the
oracle's own M / qfrc_smooth gives.  usage: python tools/smooth_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd import _lib  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
import physics_states as PS  # noqa: E402
from test_step_gpu import _dev  # noqa: E402

D = _lib.DBG


def main():
    eng = get_engine()
    m = eng.model
    nv = m.nv
    st = PS.settled_states(24, seed=0, nsettle=60)
    PS.random_ctrl(st)
    st["qvel"] += np.random.default_rng(3).normal(size=st["qvel"].shape) * 0.05
    dbg = eng.forward_debug(_dev(st, torch.float32)).cpu().numpy()
    worst = (0, None)
    for b in range(24):
        f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["qM", "qacc_smooth", "qfrc_smooth", "qfrc_passive", "qfrc_bias", "qfrc_actuator"])
        M = f["qM"].reshape(nv, nv)
        g = dbg[b][D["QACC_SMOOTH"]:D["QACC_SMOOTH"] + nv]
        gb = dbg[b][D["BIAS"]:D["BIAS"] + nv]
        ga = dbg[b][D["ACT"]:D["ACT"] + nv]
        scale = max(1.0, np.abs(M @ f["qacc_smooth"]).max())
        e = np.abs(M @ (g - f["qacc_smooth"])) / scale
        M32 = M.astype(np.float32)
        x32 = np.linalg.solve(M32, f["qfrc_smooth"].astype(np.float32)).astype(np.float64)
        e32 = np.abs(M @ (x32 - f["qacc_smooth"])) / scale
        k = int(e.argmax())
        if e[k] > worst[0]:
            worst = (e[k], b)
        print(f"env {b}: frc err {e.max():.2e} at dof {k} ({m.names_jnt[m.dof_jntid[k]]}); numpy fp32 solve {e32.max():.2e}; "
              f"qacc_smooth gpu {g[k]:.6g} ref {f['qacc_smooth'][k]:.6g}; bias err {np.abs(gb - f['qfrc_bias']).max():.2e} "
              f"act err {np.abs(ga - f['qfrc_actuator']).max():.2e} passive[k] {f['qfrc_passive'][k]:.4g} scale {scale:.3g}")
    print("worst", worst)


if __name__ == "__main__":
    main()
