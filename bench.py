#!/usr/bin/env python3
"""Benchmark of the batched DLS-IK hot path (BASELINE.json configs[1], "C2": 4096 Panda
instances, IK-only, free space, one MI355X per rank).

A "step" = one batched JacobianIKController.solve over the rank's 4096 envs (one launch of
pnp_ik_dls: every solve runs to convergence or max_iters inside the kernel).  Inputs are
synthetic (Philox, seed 20250808, counter = global env index, so rank r owns envs
[r*B, (r+1)*B) and inputs are identical at any GPU count), resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--regime waypoint|ik_test]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one process per GPU)

Rank 0 prints ONE JSON line.  `value` = all ranks' solves / max-over-ranks wall time.
`roofline` prices the ik_dls kernel at its algorithmic 89 B/solve against HBM peak, with the
kernel's average duration from HIP events on the launch stream.  `cpu_baseline` (rank 0, N=1)
times the CPU oracle (fp64 C restatement of the same solve, all allowed host threads) on a
bounded sample of the same inputs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mujoco-panda-pnp_amd"))

from pnp_amd import workloads  # noqa: E402
from pnp_amd.engine import get_engine  # noqa: E402

BASELINE_METRIC = "env-steps/sec @4096 envs/GPU, 1/2/4/8 MI355X; DLS-IK solves/sec"
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
IK_BYTES_PER_SOLVE = 89         # q_init 28 + target 12 in; q 28 + final_pos 12 + err 4 + iters 4 + flags 1 out


def host_threads():
    n = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(n, cap, 16))


def make_inputs(engine, model, rank, B, regime):
    idx = np.arange(rank * B, (rank + 1) * B)
    q, delta = workloads.ik_inputs(model, idx, regime=regime)
    dev = engine.device
    qf = torch.as_tensor(np.tile(model.qpos0, (B, 1)), dtype=torch.float32, device=dev)
    qf[:, :7] = torch.as_tensor(q, dtype=torch.float32, device=dev)
    sx, _ = engine.site_kinematics(qf.contiguous(), want_xmat=False)
    s = model.site_id("ee_center_site")
    target = (sx[:, s] + torch.as_tensor(delta, dtype=torch.float32, device=dev)).contiguous()
    return qf[:, :7].contiguous(), target, q, (sx[:, s].double().cpu().numpy() + delta)


def cpu_baseline(q_host, tgt_host, prm, budget_s=12.0):
    """Oracle (fp64 C restatement) on host threads over a bounded sample of the same inputs."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    nth = host_threads()
    n = min(len(q_host), 4096)
    O.ik_dls(q_host[:64], tgt_host[:64], nthreads=1, **prm)  # load / warm
    done, t0 = 0, time.perf_counter()
    reps = 0
    while True:
        O.ik_dls(q_host[:n], tgt_host[:n], nthreads=nth, **prm)
        done += n
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "solves/s", "cores": nth, "kind": "port",
            "sample": f"{reps} x {n} solves of the same C2 inputs (envs 0..{n - 1}), fp64 oracle "
                      f"oracle/oracle.c, {nth} pthreads, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="envs (IK solves) per GPU")
    ap.add_argument("--regime", default="waypoint", choices=sorted(workloads.IK_REGIMES))
    ap.add_argument("--params", default="default", choices=sorted(workloads.IK_PARAMS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    engine = get_engine()
    model = engine.model
    B = args.batch
    prm = workloads.IK_PARAMS[args.params]
    q0, tgt, q_host, tgt_host = make_inputs(engine, model, rank, B, args.regime)
    dev = engine.device
    out = dict(q=torch.empty(B, 7, device=dev), final_pos=torch.empty(B, 3, device=dev),
               pos_error=torch.empty(B, device=dev), iterations=torch.empty(B, dtype=torch.int32, device=dev),
               flags=torch.empty(B, dtype=torch.uint8, device=dev))

    def step():
        engine.ik_dls_into(q0, tgt, out, **prm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record()
        step()
        ends[i].record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    if dist:
        t = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    iters = out["iterations"].cpu().numpy()
    fl = out["flags"].cpu().numpy()
    total_solves = B * world * args.steps
    value = total_solves / elapsed
    achieved = IK_BYTES_PER_SOLVE * B / (kern_ms * 1e-3) / 1e9
    record = {
        "metric": BASELINE_METRIC,
        "value": value,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox seed 20250808, counter = global env index)",
        "config": {
            "workload": "C2: 4096 Panda instances, IK-only DLS (skills/ik_solver.py) batched per MI355X, free space",
            "envs_per_gpu": B, "global_envs": B * world, "regime": args.regime,
            "ik_params": prm, "parallelism": f"env-shard x{world} (no collective on the data path)",
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "kernel": "ik_dls_kernel<float, true>", "kernel_avg_ms": kern_ms,
                     "algorithmic_bytes_per_launch": IK_BYTES_PER_SOLVE * B},
        "ik_stats": {"mean_iterations": float(iters.mean()), "max_iterations": int(iters.max()),
                     "converged_frac": float((fl & 1).astype(bool).mean()),
                     "dls_iterations_per_s": float(iters.sum()) * world * args.steps / elapsed},
        "host_cores": len(os.sched_getaffinity(0)),
    }
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic_ik.json")
    if os.path.exists(traffic_file):
        with open(traffic_file) as f:
            tr = json.load(f)
        if tr.get("batch") == B:
            record["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
            record["roofline"]["traffic_source"] = tr.get("source")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        record["cpu_baseline"] = cpu_baseline(q_host, tgt_host, prm, args.cpu_budget)
    if rank == 0:
        print(json.dumps(record), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
