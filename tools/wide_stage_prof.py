"""Wide-tier stage profile (GPU): the wide kernel alone (PNP_STEP_COMPACT=3) on contact-rich
states -- the closed-finger `pressed` fixture (47-63 contacts per env) tiled to B envs -- per-stage
shader cycles per env-sub-step and the kernel's wall time.  The gym leg's critical path is the
heaviest envs' 250-sub-step chains in this tier (profiles/r04/gym_trace_summary.txt).
usage: python tools/wide_stage_prof.py [B] [nsub]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
os.environ["PNP_STEP_COMPACT"] = "3"
from pnp_amd.engine import get_engine  # noqa: E402
import pressed_diag as P  # noqa: E402
import test_step_gpu as T  # noqa: E402


def main(B=256, nsub=5):
    eng = get_engine()
    st = T._round32(P.pressed(eng.model, 16))
    big = {k: torch.cat([v] * (B // 16)) for k, v in T._dev(st, torch.float32).items()}
    keep = {k: v.clone() for k, v in big.items()}
    prof = eng.step_profile(big, nsub).cpu().numpy().astype(np.float64)
    tot = prof[:, :16].sum(1).mean()
    for rep in range(3):
        s2 = {k: v.clone() for k, v in keep.items()}
        torch.cuda.synchronize()
        t = time.time()
        eng.step(s2, nsub)
        torch.cuda.synchronize()
        t = time.time() - t
        print(f"wide kernel alone B={B} nsub={nsub}: {t * 1e3:.2f} ms ({t * 1e6 / nsub:.0f} us per sub-step; "
              f"warn max {int(s2['warn'].max())})", flush=True)
    print(f"per env per sub-step: {tot / nsub:.0f} cycles")
    for k, name in enumerate(eng.STAGES):
        if k < eng.N_STAGE_CYCLES or name.startswith("aux"):
            if name.startswith("aux") and not prof[:, k].any():
                continue
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.0f} cycles  {100 * prof[:, k].mean() / tot:5.1f}%")
        else:
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.2f} per env-sub-step (max {prof[:, k].max() / nsub:.2f})")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
