"""Why the gym workload routes envs to the wide tier: after a few random-action gym steps (4096
envs), the envs whose next step starts in the wide tier against the others -- contacts, rows and
live convex pairs per sub-step over 25 profiled sub-steps from their current state (pnp_step
stage counts), and the row / slot estimate of tier_need's thresholds.  usage:
python tools/gym_wide_why.py [B] [gym_steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.engine import Engine, get_engine  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = get_engine()
    g = BatchedFrankaShelfPNPEnv(B, engine=eng, autoreset=True)
    g.reset()
    gen = torch.Generator(device="cuda").manual_seed(20250808)
    for _ in range(n):
        g.step(torch.rand(B, 7, device="cuda", generator=gen) * 2 - 1)
    torch.cuda.synchronize()
    tier = (g.env["tier"].to(torch.int64) & 3).cpu().numpy()
    st = {k: v.clone() for k, v in g.state.items()}
    st["warn"].zero_()
    nsub = 25
    prof = eng.step_profile(st, nsub).cpu().numpy().astype(np.float64) / nsub
    S = list(Engine.STAGES)
    for t in range(3):
        sel = tier == t
        if not sel.any():
            continue
        line = []
        for k in ("n_con", "n_efc", "n_convex", "n_island", "n_newton_iter", "n_noslip_sweep", "n_live"):
            v = prof[sel, S.index(k)]
            line.append(f"{k} p50 {np.percentile(v, 50):.1f} p90 {np.percentile(v, 90):.1f} max {v.max():.1f}")
        print(f"tier {t}: {int(sel.sum())} envs; " + "; ".join(line), flush=True)
    qp = g.state["qpos"].cpu().numpy()
    print("fingers (qpos 7, 8) of wide envs, p10/p50/p90:",
          np.percentile(qp[tier == 2, 7], [10, 50, 90]), np.percentile(qp[tier == 2, 8], [10, 50, 90]))
    print("fingers of compact envs, p10/p50/p90:", np.percentile(qp[tier == 0, 7], [10, 50, 90]))


if __name__ == "__main__":
    main()
