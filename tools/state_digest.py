#!/usr/bin/env python3
"""Bit-level digest of the step / gym kernels' outputs, for refactors that must not change a bit
(LDS layout, lifetimes, register placement).  Run before and after, compare the printed lines.

    python tools/state_digest.py [B]

Steps the bench's C3 envs (reset distribution, settle, random ctrl) through the fp32 compact
kernel with its hand-over (default mode), the fp32 full kernel alone, and the fp64 kernel, plus
fused gym steps with random actions and the fresh-reset settle phase (hand-overs mid-launch);
prints a sha256 of each resulting state.
"""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mujoco-panda-pnp_amd"))

import bench  # noqa: E402
from pnp_amd import workloads  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402


def digest(st, keys=("qpos", "qvel", "qacc_warmstart", "time", "warn")):
    h = hashlib.sha256()
    for k in keys:
        h.update(st[k].contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def run_mode(engine, host, ctrl, mode, dtype, nstep):
    os.environ["PNP_STEP_COMPACT"] = mode
    st = {k: torch.as_tensor(v.astype(np.int32) if k == "warn" else v,
                             dtype=torch.int32 if k == "warn" else dtype, device="cuda").contiguous()
          for k, v in host.items()}
    for i in range(nstep):
        st["ctrl"] = ctrl[i % len(ctrl)].to(dtype).contiguous()
        engine.step(st, bench.NSUB)
    torch.cuda.synchronize()
    return st


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    torch.cuda.set_device(0)
    engine = get_engine()
    model = engine.model
    idx = np.arange(B)
    q = torch.as_tensor(np.tile(model.qpos0, (1, 1)), dtype=torch.float64, device="cuda")
    q[:, :9] = torch.as_tensor(workloads.NEUTRAL, dtype=torch.float64)
    sx, sm = engine.site_kinematics(q.contiguous())
    host = workloads.c3_reset(model, idx, sx[0].cpu().numpy(), sm[0].cpu().numpy())
    host = {k: (v.astype(np.float32).astype(np.float64) if k != "warn" else v) for k, v in host.items()}
    ctrl = torch.as_tensor(np.stack([workloads.c3_ctrl(model, idx, s) for s in range(8)]), device="cuda")
    # settle phase (cubes landing: hand-overs) + random ctrl
    for mode in ("1", "0"):
        st = run_mode(engine, host, ctrl, mode, torch.float32, 14)
        print(f"step f32 mode={mode}: {digest(st)}  max_warn={int(st['warn'].max())}")
    st = run_mode(engine, {k: v[:128] for k, v in host.items()}, ctrl[:, :128], "0", torch.float64, 4)
    print(f"step f64: {digest(st)}")
    # fingers open, servos closing: finger pads meet mid-launch (> 20 contacts)
    h2 = {k: v.copy() for k, v in host.items()}
    h2["qpos"][::2, 7:9] = 0.04
    c2 = ctrl.clone()
    c2[:, ::2, -2:] = 0.0
    for mode in ("1", "0"):
        st = run_mode(engine, h2, c2, mode, torch.float32, 6)
        print(f"step f32 fingers mode={mode}: {digest(st)}")
    os.environ.pop("PNP_STEP_COMPACT", None)
    # fused gym step, random actions
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    env = BatchedFrankaShelfPNPEnv(min(B, 512), engine=engine, autoreset=False)
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(5)
    outs = []
    for _ in range(3):
        a = (torch.rand(env.num_envs, 7, generator=g) * 2 - 1).cuda()
        r = env.step(a)
        outs.append(r)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for k in ("qpos", "qvel", "qacc_warmstart"):
        h.update(env.state[k].cpu().numpy().tobytes())
    obs, rew = outs[-1][0], outs[-1][1]
    for t in (obs["observation"] if isinstance(obs, dict) else obs, rew):
        h.update(t.cpu().numpy().tobytes())
    print(f"gym f32: {h.hexdigest()[:16]}")


if __name__ == "__main__":
    main()
