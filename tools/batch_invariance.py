"""Batch-composition invariance, bit for bit (diagnostic; the batched behaviour tree relies on it):
every kernel's per-env result must not depend on which other envs share the launch.  Checks, for
fp64 and fp32: pnp_step on a batch vs each env alone (B = 1), pnp_ik_dls batched vs single
solves, pnp_env_step on the full batch vs on a gathered subset, site kinematics.
usage: python tools/batch_invariance.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd"), os.path.join(ROOT, "tests")]
import physics_states as PS  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402
from pnp_amd.envs import BatchedFrankaShelfPNPEnv  # noqa: E402


def dev(st, dt):
    return {k: (torch.as_tensor(v.astype(np.int32), device="cuda") if k == "warn" else
                torch.as_tensor(np.ascontiguousarray(v), dtype=dt, device="cuda").contiguous()) for k, v in st.items()}


def main():
    eng = get_engine()
    m = eng.model
    import test_step_gpu as T
    sc = PS.settled_states(16, seed=0, nsettle=60, model=m)
    PS.random_ctrl(sc, model=m)
    sc["qvel"] += np.random.default_rng(3).normal(size=sc["qvel"].shape) * 0.05
    mesh = T.mesh_states(m)
    st = {k: np.concatenate([sc[k], mesh[k]]) for k in sc}
    B = st["qpos"].shape[0]
    bad = 0
    for dt in (torch.float64, torch.float32):
        for nsub in (1, 5):
            full = eng.step(dev(st, dt), nsub)
            for b in range(B):
                one = eng.step(dev({k: v[b:b + 1] for k, v in st.items()}, dt), nsub)
                for k in full:
                    if not torch.equal(full[k][b:b + 1], one[k]):
                        bad += 1
                        d = (full[k][b:b + 1].double() - one[k].double()).abs().max().item()
                        print(f"pnp_step {dt} nsub={nsub} env {b}: {k} differs (max {d:.3e})")
        # IK
        rng = np.random.default_rng(1)
        q = torch.as_tensor(rng.uniform(-1, 1, size=(37, 7)), dtype=dt, device="cuda")
        tg = torch.as_tensor(rng.uniform(-0.1, 0.1, size=(37, 3)) + [1.2, 0.0, 0.5], dtype=dt, device="cuda")
        outb = eng.ik_dls(q, tg)
        for b in range(37):
            o1 = eng.ik_dls(q[b:b + 1].contiguous(), tg[b:b + 1].contiguous())
            for k in o1:
                if not torch.equal(outb[k][b:b + 1], o1[k]):
                    bad += 1
                    print(f"ik_dls {dt} solve {b}: {k} differs")
        # gym step: full batch vs a gathered subset
        for route in ("0",):
            a = BatchedFrankaShelfPNPEnv(24, dtype=dt, autoreset=False)
            bb = BatchedFrankaShelfPNPEnv(24, dtype=dt, autoreset=False)
            a.reset()
            bb.reset()
            acts = torch.as_tensor(np.random.default_rng(2).uniform(-1, 1, size=(24, 7)), dtype=dt, device="cuda")
            a.step(acts)
            idx = list(range(0, 24, 3))
            bb.step_subset(idx, acts[idx])
            for k in a.state:
                if not torch.equal(a.state[k][idx], bb.state[k][idx]):
                    bad += 1
                    print(f"env_step {dt}: subset state {k} differs")
    print(f"batch invariance: {bad} mismatches")
    return bad


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
