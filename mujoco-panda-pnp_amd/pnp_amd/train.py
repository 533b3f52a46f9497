"""Drop-in for scripts/train.py (reference scripts/train.py:38-116): TQC on
FrankaShelfPNP{Dense,Sparse}-v0, here over ``--envs`` batched device envs (C5: 8192 on one GPU)
instead of 4 SubprocVecEnv workers.  Same hyper-parameters (pnp_amd.tqc.TQCConfig), checkpoints
(model + replay-free state + VecNormalize statistics) every ``--save-every`` transitions and a
10-episode deterministic evaluation at the same cadence (CheckpointCallback / EvalCallback).

    python -m pnp_amd.train [--sparse] [--gpu 0] [--envs 8192] [--total-steps 2000000]
    torchrun --nproc-per-node N -m pnp_amd.train ...     (data-parallel: one process per GPU)

Like the reference, ``task_sequence = ["cube1"]`` is NOT applied (train.py:58 sets it on the
wrapper, where it has no effect: SURVEY App. B quirk 8); ``--task-sequence cube1`` applies it for
real.

Update-to-data ratio: the reference's sb3 TQC (train_freq 1, gradient_steps 1) over 4
SubprocVecEnv workers makes one gradient step per vector step of 4 envs, i.e. one per 4
transitions (~500k updates over 2M transitions).  ``--gradient-steps`` defaults to the same ratio
here (``envs // 4`` gradient steps per vector step of ``--envs`` envs); ``--gradient-steps 1``
gives one update per vector step (the bench's C5 leg: env-bound, ~2000x fewer updates).
"""
from __future__ import annotations

import argparse
import os
from pathlib import Path

import torch
import torch.distributed as dist

from .envs import BatchedFrankaShelfPNPEnv, EnvConfig
from .tqc import TQC, TQCConfig


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sparse", action="store_true")
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--envs", type=int, default=8192, help="envs per GPU")
    ap.add_argument("--total-steps", type=int, default=2_000_000, help="transitions (all ranks)")
    ap.add_argument("--save-every", type=int, default=200_000)
    ap.add_argument("--ckpt-dir", default="./checkpoints")
    ap.add_argument("--eval-episodes", type=int, default=10)
    ap.add_argument("--task-sequence", default=None, help="comma-separated objects (default: all three)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--gradient-steps", type=int, default=-1,
                    help="gradient steps per vector step (default -1: envs // 4, the reference's "
                         "one update per 4 transitions)")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(args.gpu)))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    env_id = "FrankaShelfPNPSparse-v0" if args.sparse else "FrankaShelfPNPDense-v0"
    cfg = EnvConfig(task_sequence=tuple(args.task_sequence.split(","))) if args.task_sequence else EnvConfig()
    reward_type = "sparse" if args.sparse else "dense"
    env = BatchedFrankaShelfPNPEnv(args.envs, reward_type=reward_type, env_offset=rank * args.envs, config=cfg)
    eval_env = BatchedFrankaShelfPNPEnv(args.eval_episodes, reward_type=reward_type, config=cfg,
                                        env_offset=10 ** 8 + rank * args.eval_episodes)
    gsteps = args.gradient_steps if args.gradient_steps > 0 else max(1, args.envs // 4)
    model = TQC(env, TQCConfig(seed=args.seed, gradient_steps=gsteps))
    if rank == 0:
        print(f"==> Training on {env_id} | device=cuda:{local} | {args.envs} envs x {world} GPU(s) | "
              f"{gsteps} gradient steps per vector step", flush=True)
    ckpt = Path(args.ckpt_dir)
    ckpt.mkdir(exist_ok=True)
    tag = "sparse" if args.sparse else "dense"
    per_rank = args.total_steps // world
    every = max(args.save_every // world, args.envs)
    state = {"next": every}

    def callback(m):
        if m.num_timesteps >= state["next"]:
            state["next"] += every
            model.vecnorm.training = False
            r, s = m.evaluate(eval_env, args.eval_episodes)
            model.vecnorm.training = True
            if rank == 0:
                m.save(ckpt / f"tqc_{tag}_{m.num_timesteps * world}_steps.pt")
                print(f"eval: mean reward {r:.2f}, success rate {s:.2f}", flush=True)
        return True

    model.learn(per_rank, callback=callback, log_every=args.log_every)
    if rank == 0:
        model.save(ckpt / f"tqc_final_{tag}.pt")
        print("training finished & model saved", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
