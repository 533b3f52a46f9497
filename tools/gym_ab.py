"""A/B of the fp32 gym-step paths on the bench's gym workload (4096 envs, random actions):
full kernel alone vs compact phases with different physics-launch lengths.
usage: python tools/gym_ab.py [B] [steps]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]


def run(B, steps, compact, chunk):
    os.environ["PNP_STEP_COMPACT"] = compact
    os.environ["PNP_GYM_COMPACT"] = compact
    os.environ["PNP_GYM_CHUNK"] = chunk
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    g = BatchedFrankaShelfPNPEnv(B, dtype=torch.float32, autoreset=True)
    g.reset()
    rng = np.random.default_rng(0)
    acts = [torch.as_tensor(rng.uniform(-1, 1, size=(B, 7)), dtype=torch.float32, device=g.device)
            for _ in range(steps + 2)]
    for a in acts[:2]:
        g.step(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts[2:]:
        g.step(a)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"compact={compact} chunk={chunk or 'n_substeps'}: {dt * 1e3:.1f} ms per gym step, "
          f"{B * 250 / dt / 1e6:.2f} M env-steps/s", flush=True)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    for compact, chunk in (("0", ""), ("1", "250"), ("1", "25"), ("1", "5"), ("1", "1")):
        run(B, steps, compact, chunk)


if __name__ == "__main__":
    main()
