"""Stage-cycle profile of the steady-state gym workload's heavy envs (GPU): the state
tools/gym_steady_census.py dumped after a long run, split by contact count into the classes the
tiers hold (<= 20: compact, 21-64: full, > 64: wide), each class tiled to B envs and stepped by the
tier that holds it alone (PNP_STEP_COMPACT=1 with the hand-overs, or 0 / 3: the full / the wide
kernel from sub-step 0) -- per-stage shader cycles per env-sub-step and the launch's wall time.
usage: python tools/steady_stage_prof.py states.npz [B] [nsub]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.engine import get_engine  # noqa: E402

KEYS = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time", "warn")


def main():
    z = np.load(sys.argv[1])
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    nsub = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    eng = get_engine()
    nc = z["ncon"]
    print(f"{len(nc)} envs: contacts p50/90/99/max {np.percentile(nc, [50, 90, 99, 100]).astype(int).tolist()}")
    for label, sel, mode in (("compact (<= 20)", nc <= 20, "1"), ("full (21-64)", (nc > 20) & (nc <= 64), "0"),
                             ("wide (> 64)", nc > 64, "3")):
        idx = np.nonzero(sel)[0]
        if len(idx) == 0:
            continue
        rep = idx[np.arange(B) % len(idx)]
        st = {k: torch.as_tensor(z[k][rep], device="cuda").contiguous() for k in KEYS}
        st["warn"] = st["warn"].to(torch.int32)
        os.environ["PNP_STEP_COMPACT"] = mode
        keep = {k: v.clone() for k, v in st.items()}
        prof = eng.step_profile(st, nsub).cpu().numpy().astype(np.float64)
        s2 = {k: v.clone() for k, v in keep.items()}
        torch.cuda.synchronize()
        t = time.time()
        eng.step(s2, nsub)
        torch.cuda.synchronize()
        t = time.time() - t
        tot = prof[:, :eng.N_STAGE_CYCLES].sum(1)
        print(f"== {label}: {len(idx)} envs, tiled to {B}; {t * 1e3:.2f} ms for {nsub} sub-steps "
              f"({t * 1e6 / nsub:.0f} us per sub-step); cycles per env-sub-step mean {tot.mean() / nsub:.0f}, "
              f"max {tot.max() / nsub:.0f}", flush=True)
        for k, name in enumerate(eng.STAGES):
            if k < eng.N_STAGE_CYCLES:
                print(f"  {name:18s} {prof[:, k].mean() / nsub:10.0f} cycles  {100 * prof[:, k].mean() / tot.mean():5.1f}%"
                      f"  (slowest env {prof[int(tot.argmax()), k] / nsub:.0f})")
            elif prof[:, k].any():
                print(f"  {name:18s} {prof[:, k].mean() / nsub:10.2f} per env-sub-step (max {prof[:, k].max() / nsub:.2f})")
    os.environ.pop("PNP_STEP_COMPACT", None)


if __name__ == "__main__":
    main()
