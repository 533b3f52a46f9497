"""Per gym step of the bench's gym workload (4096 envs from reset, random actions, the bench's
action cycle): the step's wall time, the hand-over queue's counts (full tier -> wide tier hand-overs
published and consumed) and the tiers the envs start the next step in.
usage: python tools/gym_queue_census.py [envs] [steps]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd import _lib  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    env = BatchedFrankaShelfPNPEnv(B, autoreset=False)
    env.reset()
    acts = torch.as_tensor(np.random.default_rng(7).uniform(-1, 1, size=(4, B, 7)), dtype=torch.float32,
                           device=env.device)
    for k in range(n):
        start = (env.env["tier"].to(torch.int64) & 3).cpu().numpy()
        torch.cuda.synchronize()
        t = time.perf_counter()
        env.step(acts[k % 4])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        q = _lib.env_queue_status()
        nxt = (env.env["tier"].to(torch.int64) & 3).cpu().numpy()
        print(f"step {k}: {ms:6.1f} ms  started compact/full/wide {[(start == i).sum() for i in range(3)]}  "
              f"queue {q}  next {[(nxt == i).sum() for i in range(3)]}", flush=True)


if __name__ == "__main__":
    main()
