"""Tier census of the fp32 gym workload (bench's gym leg shape: 4096 envs, uniform random actions):
per gym step, how many envs start in the compact / full / wide tier (env_state.tier after the
previous step) and the step's wall time.  usage: python tools/gym_tier_census.py [B] [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    g = BatchedFrankaShelfPNPEnv(B, autoreset=True)
    g.reset()
    gen = torch.Generator(device="cuda").manual_seed(20250808)
    for k in range(n):
        t = g.env["tier"].to(torch.int64) & 3
        cnt = [int((t == i).sum()) for i in range(3)]
        a = torch.rand(B, 7, device="cuda", generator=gen) * 2 - 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.step(a)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        print(f"step {k}: starts compact {cnt[0]} full {cnt[1]} wide {cnt[2]}; {dt:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
