"""Closed-finger (`pressed`) fixture diagnosis (GPU): per env, the oracle's Newton iterations and
noslip sweeps against the fp32 kernel's (stage-profile counts over the compact -> full -> wide
tiers) and the fp64 kernel's one-step state (full -> fp64 wide tier) against the oracle.
usage: python tools/pressed_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402
import physics_states as PS  # noqa: E402
import test_step_gpu as T  # noqa: E402


def pressed(m, n=12):
    st = PS.reset_states(n, seed=11, model=m)
    st["qpos"][:, 7:9] = -np.linspace(0.001, 0.004, n)[:, None]
    st["ctrl"][:, -2:] = 0.0
    st["qvel"] += np.random.default_rng(5).normal(size=st["qvel"].shape) * 0.02
    return st


def main():
    m = load_model()
    eng = get_engine()
    st = T._round32(pressed(m))
    B = st["qpos"].shape[0]
    prof = eng.step_profile(T._dev(st, torch.float32), 1).cpu().numpy()
    S = list(eng.STAGES)
    ref = PS.copy_state(st)
    O.step(ref, nsub=1, nthreads=8, model=m)
    g64 = T._host(eng.step(T._dev(st, torch.float64), 1))
    g32 = T._host(eng.step(T._dev(st, torch.float32), 1))
    ev32, _ = T._tree_metrics(m, st, ref, g32, per_env=True)
    ev64, _ = T._tree_metrics(m, st, ref, g64, per_env=True)
    for b in range(B):
        f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS},
                             ["ncon", "nefc", "solver_iter", "noslip_iter", "noslip_improvement"], model=m)
        print(f"env {b}: ncon {int(f['ncon'][0])} nefc {int(f['nefc'][0])}; oracle newton {int(f['solver_iter'][0])} "
              f"noslip {int(f['noslip_iter'][0])} {np.array2string(f['noslip_improvement'][:3], precision=2)}; "
              f"fp32 kernel newton {prof[b, S.index('n_newton_iter')]} noslip {prof[b, S.index('n_noslip_iter')]} "
              f"dense {prof[b, S.index('n_ns_dense')]} con {prof[b, S.index('n_con')]}; "
              f"dqvel arm fp32 {ev32[b, 0]:.2e} fp64 {ev64[b, 0]:.2e}; warn64 {int(g64['warn'][b])}", flush=True)
    print("fp64 |dqpos| max", np.abs(g64["qpos"] - ref["qpos"]).max(), "|dqvel| max", np.abs(g64["qvel"] - ref["qvel"]).max())


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def variants():
    """env 6 / 8: fp32 arm error with multiccd on / off on both sides, and the per-dof velocity
    change difference against the oracle; the contacts per pair of those envs."""
    from pnp_amd.engine import Engine
    from pnp_amd.model import PandaModel
    m = load_model()
    st = T._round32(pressed(m))
    m0 = PandaModel()
    m0.opt_multiccd = 0
    m0._desc = None
    e0 = Engine(model=m0, device=get_engine().device)
    for tag, mm, eng in (("multiccd on", m, get_engine()), ("multiccd off", m0, e0)):
        ref = PS.copy_state(st)
        O.step(ref, nsub=1, nthreads=8, model=mm)
        g32 = T._host(eng.step(T._dev(st, torch.float32), 1))
        ev32, _ = T._tree_metrics(mm, st, ref, g32, per_env=True)
        print(tag, "arm dqvel errors", np.array2string(ev32[:, 0], precision=2), flush=True)
        for b in (6, 8):
            d = (g32["qvel"][b] - ref["qvel"][b])
            print(f"  env {b} dqvel diff per dof (arm 0-8) {np.array2string(d[:9], precision=2)}", flush=True)
            import collections
            f = O.forward_fields({k: st[k][b] for k in O.STATE_KEYS}, ["contact", "ncon"], model=mm)
            c = f["contact"].reshape(int(f["ncon"][0]), 30)
            print("   pairs", dict(collections.Counter((int(x), int(y)) for x, y in c[:, 27:29])), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "variants":
    variants()
