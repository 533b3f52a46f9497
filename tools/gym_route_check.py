"""Routing check of the fp32 gym step (bench.py's gym workload: 4096 envs, random actions): after
each gym step, the tier every env's NEXT step will start in (env_state.tier, committed) against
the contact count of a forward at the env's new state (forward_debug: the full tier, 48 contacts)
-- do the envs whose grippers stay closed (> 20 contacts) start the next step past the compact
tier, as the routing intends?  usage: python tools/gym_route_check.py [envs] [steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd import _lib  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    env = BatchedFrankaShelfPNPEnv(B, autoreset=False)
    env.reset()
    acts = torch.as_tensor(np.random.default_rng(7).uniform(-1, 1, size=(4, B, 7)), dtype=torch.float32,
                           device=env.device)
    D = _lib.DBG
    edges = [0, 17, 21, 33, 41, 49]
    for k in range(n):
        env.step(acts[k % 4])
        torch.cuda.synchronize()
        tier = (env.env["tier"].to(torch.int64) & 3).cpu().numpy()
        dbg = env.engine.forward_debug({kk: v.clone() for kk, v in env.state.items()})
        ncon = dbg[:, D["COUNTS"]].cpu().numpy().astype(int)
        line = []
        for t, name in enumerate(("compact", "full", "wide")):
            sel = tier == t
            h, _ = np.histogram(ncon[sel], bins=edges + [10 ** 6])
            line.append(f"{name} {int(sel.sum())}: " + " ".join(f"{a}-{b - 1}:{c}" for a, b, c in
                                                                  zip(edges, edges[1:] + [999], h)))
        print(f"after step {k}: next step starts | " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
