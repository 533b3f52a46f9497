"""Hand-over census of the fp32 gym step (bench.py's gym workload: 4096 envs, random actions):
after W normal steps, one step with PNP_GYM_COMPACT=2 (the compact pass alone, plus the routed
full / wide passes) leaves every env a pass handed over with its resume bits -- the sub-step it
stopped at (csrc/step.hip PNP_RESUME_*) -- so the counts and sub-step histogram show how much
work each queue would carry.  Diagnostic only: the step is left unfinished.
usage: python tools/gym_handover_census.py [envs] [warm steps] [states.npz]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402

RESUME_FLAG, RESUME_SHIFT, RESUME_MAXSUB, WHY_SHIFT = 0x80000000, 16, 0xFFF, 28


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    env = BatchedFrankaShelfPNPEnv(B, autoreset=False)
    env.reset()
    acts = torch.as_tensor(np.random.default_rng(7).uniform(-1, 1, size=(4, B, 7)), dtype=torch.float32,
                           device=env.device)
    for i in range(warm):
        env.step(acts[i % 4])
    tier = (env.env["tier"] & 3).cpu().numpy()
    os.environ["PNP_GYM_COMPACT"] = "2"
    env.step(acts[warm % 4])
    torch.cuda.synchronize()
    w = env.state["warn"].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    handed = (w & RESUME_FLAG) != 0
    k0 = (w >> RESUME_SHIFT) & RESUME_MAXSUB
    why = (w >> WHY_SHIFT) & 0x7
    if len(sys.argv) > 3:   # the handed-over envs' states (stored before their overflowing sub-step)
        sel = np.nonzero(handed)[0]
        np.savez_compressed(sys.argv[3], env=sel, tier=tier[sel], k0=k0[sel],
                            **{k: v[sel].cpu().numpy() for k, v in env.state.items()})
    nsub = env.cfg.n_substeps * env.cfg.n_calls
    print(f"{B} envs, step {warm} (sub-steps {nsub}); starting tiers: compact {int((tier == 0).sum())}, "
          f"full {int((tier == 1).sum())}, wide {int((tier == 2).sum())}")
    for t, name in ((0, "compact -> full"), (1, "full (routed) -> wide")):
        sel = handed & (tier == t)
        k = k0[sel]
        print(f"  {name}: {int(sel.sum())} envs handed over; reason bits {np.bincount(why[sel], minlength=8).tolist()}")
        if k.size:
            h, e = np.histogram(k, bins=[0, 1, 10, 25, 50, 100, 150, 200, 250])
            print("    stop sub-step histogram:", {f"{int(a)}-{int(b) - 1}": int(c) for a, b, c in zip(e[:-1], e[1:], h)})
            print(f"    remaining sub-steps: sum {int((nsub - k).sum())}, mean {float((nsub - k).mean()):.1f}")


if __name__ == "__main__":
    main()
