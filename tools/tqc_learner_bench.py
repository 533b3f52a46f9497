"""Learner-step timing (C5 at train.py's update ratio is ~all learner): the TQC gradient step on a
64-env short-physics replay, fused HIP step (pnp_tqc_update) vs the PyTorch step, both captured in
a HIP graph; for rocprofv3 --kernel-trace; prints a digest of the trained parameters.  usage: python tools/tqc_learner_bench.py [fused|torch] [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig  # noqa: E402
from pnp_amd.tqc import TQC, TQCConfig  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "fused"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    env = BatchedFrankaShelfPNPEnv(64, config=EnvConfig(n_substeps=2, n_calls=2))
    a = TQC(env, TQCConfig(fused=mode == "fused"))
    a.total_timesteps = 10 ** 6
    a.reset()
    for _ in range(12):
        a.collect_step()
    a.train(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a.train(n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    print(f"{mode}: {dt:.3f} ms per gradient step ({a.logs and {k: float(v) for k, v in a.logs.items()}})")
    # parameter digest (A/B builds of the fused step must agree bit for bit)
    import hashlib
    flat = torch.cat([p.detach().reshape(-1) for p in list(a.actor.parameters()) + list(a.critic.parameters())])
    print("param digest", hashlib.sha256(flat.cpu().numpy().tobytes()).hexdigest()[:16])


if __name__ == "__main__":
    main()
