"""Stage-cycle profile of the full tier on the gym's closed-gripper states: the states the compact
tier handed over (tools/gym_handover_census.py ... states.npz: stored before the overflowing
sub-step), tiled to B envs, stepped by the full kernel alone (PNP_STEP_COMPACT=0, PNP_STEP_WIDE=0:
sub-steps past 48 contacts truncate instead of handing over -- a profile, not a result).
usage: python tools/full_tier_profile.py states.npz [B] [nsub]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
os.environ["PNP_STEP_COMPACT"] = "0"
os.environ["PNP_STEP_WIDE"] = "0"
from pnp_amd.engine import get_engine  # noqa: E402

KEYS = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time", "warn")


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    nsub = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    d = np.load(path)
    n = len(d["env"])
    idx = np.arange(B) % n
    eng = get_engine()
    st = {}
    for k in KEYS:
        v = d[k][idx]
        if k == "warn":
            st[k] = torch.as_tensor((v.astype(np.int64) & 0xFFFF).astype(np.int32), device="cuda")
        else:
            st[k] = torch.as_tensor(v, dtype=torch.float32, device="cuda").contiguous()
    keep = {k: v.clone() for k, v in st.items()}
    prof = eng.step_profile(st, nsub).cpu().numpy().astype(np.float64)
    tot = prof[:, :16].sum(1).mean()
    for _ in range(3):
        s2 = {k: v.clone() for k, v in keep.items()}
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        eng.step(s2, nsub)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1])
        print(f"full kernel alone B={B} nsub={nsub}: {ms:.2f} ms ({ms / nsub * 1e3:.0f} us per sub-step)")
    print(f"{n} closed-gripper states tiled to {B}; per env per sub-step: {tot / nsub:.0f} cycles")
    nc = eng.N_STAGE_CYCLES
    for k, name in enumerate(eng.STAGES):
        if k < nc or name.startswith("aux"):
            if name.startswith("aux") and not prof[:, k].any():
                continue
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.0f} cycles  {100 * prof[:, k].mean() / tot:5.1f}%")
        else:
            print(f"  {name:18s} {prof[:, k].mean() / nsub:10.2f} per env-sub-step (max {prof[:, k].max() / nsub:.2f})")


if __name__ == "__main__":
    main()
