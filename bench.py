#!/usr/bin/env python3
"""Benchmark of the batched env-step hot path (BASELINE.json metric "env-steps/sec @4096
envs/GPU, 1/2/4/8 MI355X; DLS-IK solves/sec").

Default workload (--workload step) = BASELINE configs[2] "C3" at N=1 and configs[3] "C4" at N>1:
4096 shelf_pnp envs per GPU, full mj_step (kinematics, CRBA, collision, constraints, RNE,
Newton + noslip, Euler), random ctrl.  A "step" = one launch of pnp_step over the rank's envs
with nsub = 25 fused sub-steps (the reference's mj_step(nstep=n_substeps=25),
envs/panda_env.py:355-358) and a fresh ctrl ~ U(actuator_ctrlrange) per step (a table of 64
Philox draws, cycled, resident in HBM).  value = env-steps (= mj_step's) per second, all ranks.
Inputs: the reference's reset distribution (Philox, seed 20250808, counter = global env index;
rank r owns envs [r*B, (r+1)*B)), settled by 250 untimed sub-steps like _env_setup.

--workload ik = configs[1] "C2": one batched JacobianIKController.solve over 4096 envs per step.
The step workload also times C2 briefly ("ik"), the fused gym step of C5's env side ("gym":
FrankaEnv.step = set_action + 250 sub-steps + obs / reward, one launch) and C5's whole TQC loop
("tqc": 8192 envs per GPU, a gym step + a gradient step per step, pnp_amd/tqc.py).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload step|ik]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one process per GPU)

Rank 0 prints ONE JSON line.  `roofline` prices the dominant kernel at its algorithmic bytes
(state read + written once per launch) against HBM peak, with its average duration from HIP
events on the launch stream.  `cpu_baseline` (rank 0, N=1) times the fp64 CPU oracle (C
restatement of the same algorithms, all allowed host threads) on a bounded sample of the same
inputs.
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
# env-step launch: read qpos 37 + qvel 33 + ctrl 9 + mocap 7 + qacc_warmstart 33 + time 1 + warn 1
# words, write qpos 37 + qvel 33 + qacc_warmstart 33 + time 1 + warn 1 words (fp32 / u32)
STEP_BYTES_PER_ENV = 4 * (37 + 33 + 9 + 3 + 4 + 33 + 1 + 1) + 4 * (37 + 33 + 33 + 1 + 1)
NSUB = 25                       # panda_env.py n_substeps
NSETTLE = 250                   # _env_setup settle sub-steps (panda_env.py:124-141)
NCTRL = 64                      # distinct per-step ctrl draws, cycled
RANK_LEGS = {}                  # leg -> every rank's [wall s, kernel ms] (dist_record)


def host_threads():
    """The cores this process can actually use (the CPU baseline runs over all
    cores): its affinity set, bounded by the cgroup CPU quota when one is set -- the GPU box
    shows 256 cores but grants a 16-CPU quota, and 256 threads on it measured 35 % slower than
    16 (CFS throttling: profiles/r03/bench_step_v16.log, 78 k vs 122 k env-steps/s)."""
    n = max(1, len(os.sched_getaffinity(0)))
    q = cpu_quota()
    return max(1, min(n, int(np.ceil(q)))) if q else n


def cpu_quota():
    """cgroup v2 CPU quota in cores (None: unlimited / unknown) -- reported beside the thread
    count, since a quota below the affinity set caps what those threads can do."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def _oracle():
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    return O


def _timed(fn, steps, warmup, dist, per_call_events=True, ranks_out=None):
    """W untimed + K timed calls bracketed by barrier + synchronize; returns (wall s, avg event ms).
    per_call_events: an event pair around every call (the average launch duration of long
    kernels); off, one pair around the K calls (average = region / K): for kernels of tens of
    microseconds, where event markers between the launches cost ~8 us per call (IK leg).
    ranks_out (a list): receives every rank's own (wall s, kernel ms), gathered, in rank order --
    the job's figures are their max."""
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    n_ev = steps if per_call_events else 1
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if not per_call_events:
        starts[0].record()
    for i in range(steps):
        if per_call_events:
            starts[i].record()
        fn(warmup + i)
        if per_call_events:
            ends[i].record()
    if not per_call_events:
        ends[0].record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    if not per_call_events:
        kern_ms /= steps
    if ranks_out is not None:
        ranks_out[:] = gather_ranks([elapsed, kern_ms]) if dist else [[elapsed, kern_ms]]
    if dist:
        elapsed, kern_ms = reduce_max([elapsed, kern_ms], "cuda")
    return elapsed, kern_ms


def reduce_max(values, device):
    """MAX of each value over all ranks (the slowest rank sets the job's time)."""
    t = torch.tensor(values, device=device, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return [float(v) for v in t]


def gather_ranks(obj):
    """Every rank's `obj`, in rank order (all_gather_object: gloo or RCCL)."""
    out = [None] * torch.distributed.get_world_size()
    torch.distributed.all_gather_object(out, obj)
    return out


def rank_identity(local, device):
    """What this rank ran on: its rank / local rank and, on a GPU, the device index, name and PCI
    bus (one MI355X per rank under RCCL -- the record shows it instead of assuming it)."""
    me = {"rank": int(os.environ.get("RANK", "0")), "local_rank": local,
          "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))}
    if device == "cuda":
        d = torch.cuda.current_device()
        pr = torch.cuda.get_device_properties(d)
        me.update(device=d, device_name=pr.name, arch=getattr(pr, "gcnArchName", None),
                  pci=f"{getattr(pr, 'pci_domain_id', 0):04x}:{getattr(pr, 'pci_bus_id', 0):02x}:"
                      f"{getattr(pr, 'pci_device_id', 0):02x}")
    else:
        me.update(device="cpu")
    return me


def dist_record(expected, world, dist, ident, legs):
    """The job as torch.distributed saw it -- world size and backend from the process group (not
    the launcher's environment), each rank's device and its own timings per leg -- and the check
    that it is the job --gpus asked for (rank 0 raises otherwise: a record that is not N ranks on N
    distinct GPUs is never printed).  ident: every rank's rank_identity; legs: {leg: every rank's
    [wall s, kernel ms]}."""
    ws = torch.distributed.get_world_size() if dist else 1
    backend = str(torch.distributed.get_backend()) if dist else None
    ranks = []
    for r, me in enumerate(ident):
        row = dict(me)
        for leg, vals in legs.items():
            if vals:
                row[f"{leg}_wall_s"], row[f"{leg}_kernel_ms"] = float(vals[r][0]), float(vals[r][1])
        ranks.append(row)
    rec = {"world_size": ws, "backend": backend, "gpus_flag": expected, "ranks": ranks}
    problems = []
    if ws != expected or world != expected:
        problems.append(f"process group world size {ws} (launcher {world}) != --gpus {expected}")
    if [r["rank"] for r in ranks] != list(range(ws)):
        problems.append(f"ranks {[r['rank'] for r in ranks]} are not 0..{ws - 1}")
    if backend == "nccl":
        pcis = [r.get("pci") for r in ranks]
        if len(set(pcis)) != len(pcis):
            problems.append(f"ranks share GPUs: {pcis}")
    if problems:
        raise SystemExit("bench.py: " + "; ".join(problems))
    return rec


def _progress(rank, msg):
    """Progress line on stderr (rank 0): the legs take tens of seconds each."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def total_steps(B, world, steps):
    return B * world * steps * NSUB


def shard_range(rank, B):
    """Global env indices of rank r: [r*B, (r+1)*B) (inputs depend only on the global index)."""
    return np.arange(rank * B, (rank + 1) * B)


def _traffic(name, B):
    f = os.path.join(ROOT, "profiles", name)
    if os.path.exists(f):
        with open(f) as fh:
            tr = json.load(fh)
        if tr.get("batch") == B:
            return tr.get("hbm_bytes_per_launch"), tr.get("source")
    return None, None


def _sq_valu():
    """VALU issue share from the committed SQ-counter pass (profiles/sq_counters_step.json): a
    figure measured by a separate rocprofv3 run, not by this one -- returned with its provenance
    (file, kernel build it was measured on) so a stale value is visible."""
    f = os.path.join(ROOT, "profiles", "sq_counters_step.json")
    if os.path.exists(f):
        with open(f) as fh:
            j = json.load(fh)
        return j.get("valu_issue_frac"), {"file": "profiles/sq_counters_step.json", "measured_in_this_run": False,
                                           "kernel_version": j.get("kernel_version"), "source": j.get("source"),
                                           "valu_pipe_util": j.get("valu_pipe_util")}
    return None, None


# ----------------------------------------------------------------------------- C3 / C4 env-step
def step_inputs(engine, model, rank, B):
    idx = shard_range(rank, B)
    q = torch.as_tensor(np.tile(model.qpos0, (1, 1)), dtype=torch.float64, device=engine.device)
    q[:, :9] = torch.as_tensor(workloads.NEUTRAL, dtype=torch.float64)
    sx, sm = engine.site_kinematics(q.contiguous())
    host = workloads.c3_reset(model, idx, sx[0].cpu().numpy(), sm[0].cpu().numpy())
    st = {}
    for k, v in host.items():
        dt = torch.int32 if k == "warn" else torch.float32
        st[k] = torch.as_tensor(v.astype(np.int32) if k == "warn" else v, dtype=dt, device=engine.device).contiguous()
    for _ in range(NSETTLE // NSUB):    # same launch shape as the timed steps (profiles agree)
        engine.step(st, NSUB)
    ctrl = torch.as_tensor(np.stack([workloads.c3_ctrl(model, idx, s) for s in range(NCTRL)]),
                           dtype=torch.float32, device=engine.device).contiguous()
    return st, ctrl


def step_cpu_baseline(st, ctrl, budget_s):
    """fp64 oracle mj_step x NSUB on host threads, over a bounded sample of the same settled envs."""
    O = _oracle()
    nth = host_threads()
    n = min(st["qpos"].shape[0], max(256, 2 * nth))   # >= 2 envs per thread
    sample = {k: (v[:n].cpu().numpy().astype(np.uint32) if k == "warn" else v[:n].double().cpu().numpy())
              for k, v in st.items()}
    ctab = ctrl[:, :n].double().cpu().numpy()
    O.step({k: v[:8].copy() for k, v in sample.items()}, nsub=1, nthreads=1)   # load / warm
    done, reps, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        sample["ctrl"] = np.ascontiguousarray(ctab[reps % NCTRL])
        O.step(sample, nsub=NSUB, nthreads=nth)
        done += n * NSUB
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "env-steps/s", "cores": nth, "kind": "port", "cpu_quota": cpu_quota(),
            "host_cores": len(os.sched_getaffinity(0)),
            "sample": f"{reps} steps x {n} envs x {NSUB} sub-steps of the same settled C3 envs "
                      f"(envs 0..{n - 1}), fp64 oracle oracle/physics.c, {nth} pthreads, {dt:.1f} s"}


def run_step(args, engine, model, rank, world, dist):
    B = args.batch
    st, ctrl = step_inputs(engine, model, rank, B)
    torch.cuda.synchronize()
    _progress(rank, "inputs settled")

    def fn(i):
        st["ctrl"] = ctrl[i % NCTRL]
        engine.step(st, NSUB)

    elapsed, kern_ms = _timed(fn, args.steps, args.warmup, dist, ranks_out=RANK_LEGS.setdefault("step", []))
    _progress(rank, f"step leg done: {total_steps(B, world, args.steps) / elapsed / 1e6:.2f} M env-steps/s")
    warn = int((st["warn"].to(torch.int64) & 0xFFFFFFFF).max())   # warn is int32: bit 31 reads negative
    finite = bool(torch.isfinite(st["qpos"]).all())
    total = B * world * args.steps * NSUB
    achieved = STEP_BYTES_PER_ENV * B / (kern_ms * 1e-3) / 1e9
    traffic, src = _traffic("pmc_traffic_step.json", B)
    valu, valu_src = _sq_valu()
    rec = {
        "metric": BASELINE_METRIC,
        "value": total / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (reset distribution + random ctrl; Philox seed 20250808, counter = global env index)",
        "config": {
            "workload": ("C3: 4096 shelf_pnp envs full mj_step per MI355X, random ctrl" if world == 1 else
                         f"C4: {B * world} shelf_pnp envs sharded over {world} MI355X, random ctrl"),
            "envs_per_gpu": B, "global_envs": B * world, "sub_steps_per_step": NSUB,
            "parallelism": f"env-shard x{world} (no collective on the data path)",
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": src,
                     "kernel": "pnp_compact::step_kernel<float, false> + pnp_full::step_kernel resume pass (one pnp_step)",
                     "kernel_avg_ms": kern_ms,
                     "algorithmic_bytes_per_launch": STEP_BYTES_PER_ENV * B,
                     # the HBM bound is the metric's definition; the kernel itself is latency-bound
                     # (one or two waves per SIMD, dependent LDS / DPP chains): PMC-measured
                     # bandwidth of the same launch, for scale
                     "pmc_GBps": (traffic / (kern_ms * 1e-3) / 1e9) if traffic else None,
                     # SQ counters of the same kernel (profiles/sq_counters_step.json): the share
                     # of cycles the SIMDs' vector ALUs issue, all resident waves together --
                     # from a separate rocprofv3 pass, provenance alongside
                     "valu_issue_frac": valu, "valu_issue_frac_source": valu_src,
                     "limiter": "latency and instruction issue (resident waves x cycles per env-sub-step), not HBM"},
        "state_ok": {"max_warn": warn, "finite": finite},
        "host_cores": len(os.sched_getaffinity(0)),
    }
    if not args.no_gym:
        rec["gym"] = run_gym(engine, B, rank, world, dist)
        _progress(rank, f"gym leg done: {rec['gym']['gym_steps_per_s']:.0f} gym-steps/s")
        if args.steady_burn > 0:
            rec["gym"]["steady"] = run_gym_steady(engine, B, rank, world, dist, burn=args.steady_burn)
            _progress(rank, f"gym steady leg done: {rec['gym']['steady']['gym_steps_per_s']:.0f} gym-steps/s")
    if not args.no_tqc:
        rec["tqc"] = run_tqc(engine, args.tqc_envs, rank, world, dist, steady_burn=args.steady_burn)
        _progress(rank, f"tqc leg done: {rec['tqc']['gym_steps_per_s']:.0f} transitions/s")
    if not args.no_ik:
        ik = run_ik(args, engine, model, rank, world, dist, steps=500, warmup=20,
                    baseline=not args.no_cpu_baseline, budget=min(args.cpu_budget, 4.0))
        rec["ik"] = {k: ik[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup")}
        rec["ik"].update(roofline_frac=ik["roofline"]["frac"], workload=ik["config"]["workload"])
        if "cpu_baseline" in ik:
            rec["ik"]["cpu_baseline"] = ik["cpu_baseline"]
        _progress(rank, f"ik leg done: {ik['value'] / 1e6:.1f} M solves/s")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        _progress(rank, "cpu baseline ...")
        rec["cpu_baseline"] = step_cpu_baseline(st, ctrl, args.cpu_budget)
    return rec


# ----------------------------------------------------------------------------- fused gym step
class QueueHealth:
    """pnp_env_queue_status summed over the routed gym steps it is sampled after: envs handed to
    the wide tier through the device queue, consumers that gave up waiting, envs the fallback pass
    finished -- a run whose consumers time out prints a normal-looking rate, so the record carries
    these next to it.  (Each sample synchronises: taken outside timed regions only.)"""

    def __init__(self):
        self.n, self.tot = 0, {"published": 0, "timeouts": 0, "fallback": 0}

    def sample(self):
        from pnp_amd import _lib
        q = _lib.env_queue_status()
        self.n += 1
        for k in self.tot:
            self.tot[k] += int(q[k])
        return q

    def record(self, what):
        return dict(self.tot, steps_sampled=self.n, sampled=what)


def run_gym(engine, B, rank, world, dist, steps=3, warmup=1):
    """C5's env side: FrankaShelfPNPDense env.step over B envs per GPU as ONE fused launch
    (set_action + 250 sub-steps + obs / reward / success / sequencing), random actions; gym steps
    1-3 after a reset (see run_gym_steady for a long run)."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    env = BatchedFrankaShelfPNPEnv(B, engine=engine, env_offset=rank * B, autoreset=False)
    env.reset()
    acts = torch.as_tensor(np.random.default_rng(7 + rank).uniform(-1, 1, size=(4, B, 7)), dtype=torch.float32,
                           device=engine.device)
    elapsed, kern_ms = _timed(lambda i: env.step(acts[i % 4]), steps, warmup, dist,
                              ranks_out=RANK_LEGS.setdefault("gym", []))
    qh = QueueHealth()
    qh.sample()
    sub = env.cfg.n_substeps * env.cfg.n_calls
    return {"gym_steps_per_s": B * world * steps / elapsed, "env_steps_per_s": B * world * steps * sub / elapsed,
            "ms_per_gym_step": elapsed / steps * 1e3, "kernel_avg_ms": kern_ms, "sub_steps_per_gym_step": sub,
            "kernel": "env_step_kernel<float>", "workload": f"{B} FrankaShelfPNPDense envs per GPU, random actions, "
                                                            f"gym steps {warmup + 1}-{warmup + steps} after reset",
            "queue": qh.record("the last timed step")}


def run_gym_steady(engine, B, rank, world, dist, burn=50, steps=5):
    """The gym step in steady state: train.py runs 300-step episodes
    under auto-reset (panda_mujoco_gym/__init__.py:15), so later gym steps of a long run -- grippers
    that stay closed and pressed, cubes grasped or knocked over -- dominate, not the first steps
    after a reset.  B envs, random actions, auto-reset, `burn` untimed steps (each env's episode at
    step `burn`), then `steps` timed ones.  The hand-over queue's counters are summed over the
    burn-in (sampled after every step) and the timed steps' last."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    env = BatchedFrankaShelfPNPEnv(B, engine=engine, env_offset=rank * B, autoreset=True)
    env.reset()
    rng = np.random.default_rng(11 + rank)
    acts = torch.as_tensor(rng.uniform(-1, 1, size=(16, B, 7)), dtype=torch.float32, device=engine.device)
    qh = QueueHealth()
    t0 = time.perf_counter()
    for i in range(burn):
        env.step(acts[i % 16])
        qh.sample()
    burn_s = time.perf_counter() - t0
    elapsed, kern_ms = _timed(lambda i: env.step(acts[i % 16]), steps, 0, dist,
                              ranks_out=RANK_LEGS.setdefault("gym_steady", []))
    qh.sample()
    sub = env.cfg.n_substeps * env.cfg.n_calls
    return {"gym_steps_per_s": B * world * steps / elapsed, "env_steps_per_s": B * world * steps * sub / elapsed,
            "ms_per_gym_step": elapsed / steps * 1e3, "kernel_avg_ms": kern_ms,
            "burn_in_steps": burn, "burn_in_ms_per_gym_step": burn_s / max(burn, 1) * 1e3,
            "workload": f"{B} FrankaShelfPNPDense envs per GPU, random actions, auto-reset, gym steps "
                        f"{burn + 1}-{burn + steps} of a run",
            "queue": qh.record(f"after each of the {burn} burn-in steps and the last timed step")}


# ----------------------------------------------------------------------------- C5 TQC training loop
def run_tqc(engine, B, rank, world, dist, steps=3, warmup=2, learner_reps=20, steady_burn=0):
    """C5: scripts/train.py's TQC loop over B batched envs per GPU (pnp_amd.tqc, train.py
    hyper-parameters): one step = one fused gym step of every env (policy actions, auto-reset,
    replay insert, obs statistics) + one gradient step (batch 512; gradients all-reduced over
    ranks when N > 1).  Also times the gradient step alone, train.py's update ratio, and (with
    steady_burn) the loop after `steady_burn` further steps of the same run."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    from pnp_amd.tqc import TQC, TQCConfig
    env = BatchedFrankaShelfPNPEnv(B, engine=engine, env_offset=rank * B)
    agent = TQC(env, TQCConfig())
    agent.total_timesteps = 2_000_000
    agent.reset()

    def fn(i):
        agent.collect_step()
        agent.train()

    elapsed, kern_ms = _timed(fn, steps, warmup, dist, ranks_out=RANK_LEGS.setdefault("tqc", []))
    qh = QueueHealth()
    qh.sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(learner_reps):
        agent.train()
    torch.cuda.synchronize()
    learner_ms = (time.perf_counter() - t0) / learner_reps * 1e3
    sub = env.cfg.n_substeps * env.cfg.n_calls
    step_ms = elapsed / steps * 1e3
    # the reference's update-to-data ratio (train.py: one gradient step per 4 transitions, sb3's
    # defaults over 4 SubprocVecEnv workers), measured: one vector step + B / 4 gradient steps
    utd = max(1, B // 4)

    def fn_utd(i):
        agent.collect_step()
        agent.train(utd)

    utd_elapsed, _ = _timed(fn_utd, 1, 0, dist)
    steady = None
    if steady_burn > 0:
        # the same run further on: steady_burn more vector steps (one gradient step each; the
        # episodes are then at step ~steady_burn + 8 of 300), then timed steps
        qs = QueueHealth()
        t0 = time.perf_counter()
        for _ in range(steady_burn):
            fn(0)
            qs.sample()
        burn_s = time.perf_counter() - t0
        s_el, _ = _timed(fn, steps, 0, dist, ranks_out=RANK_LEGS.setdefault("tqc_steady", []))
        qs.sample()
        steady = {"gym_steps_per_s": B * world * steps / s_el, "ms_per_step": s_el / steps * 1e3,
                  "burn_in_steps": steady_burn, "burn_in_ms_per_step": burn_s / steady_burn * 1e3,
                  "vector_steps_before_timing": warmup + steps + 1 + steady_burn,
                  "queue": qs.record(f"after each of the {steady_burn} burn-in steps and the last timed step")}
    return {"gym_steps_per_s": B * world * steps / elapsed, "env_steps_per_s": B * world * steps * sub / elapsed,
            "ms_per_step": step_ms, "learner_ms_per_update": learner_ms,
            "learner": ((("hand-written fused HIP gradient step (csrc/tqc_fused.hip: "
                          + ("pnp_tqc_sample_draw, the random numbers drawn on the device"
                             if agent.cfg.device_rng else "pnp_tqc_sample") + " + pnp_tqc_update, 7 launches)")
                         if agent._fdesc is not None else "PyTorch gradient step (fused Adam)")
                        + (", captured in a HIP graph and replayed" if agent._graph is not None else ", eager")),
            "transitions_per_s_at_reference_utd": B * world / utd_elapsed,
            "reference_utd": {"gradient_steps_per_vector_step": utd, "ms_per_vector_step": utd_elapsed * 1e3,
                              "measured": True},
            "workload": f"C5: TQC (train.py hyper-parameters) on {B} FrankaShelfPNPDense envs per GPU, "
                        f"one gym step + one gradient step per step",
            "queue": qh.record("the last timed step"), "steady": steady}


# ----------------------------------------------------------------------------- C2 IK
def ik_inputs(engine, model, rank, B, regime):
    idx = shard_range(rank, B)
    q, delta = workloads.ik_inputs(model, idx, regime=regime)
    dev = engine.device
    qf = torch.as_tensor(np.tile(model.qpos0, (B, 1)), dtype=torch.float32, device=dev)
    qf[:, :7] = torch.as_tensor(q, dtype=torch.float32, device=dev)
    sx, _ = engine.site_kinematics(qf.contiguous(), want_xmat=False)
    s = model.site_id("ee_center_site")
    target = (sx[:, s] + torch.as_tensor(delta, dtype=torch.float32, device=dev)).contiguous()
    return qf[:, :7].contiguous(), target, q, (sx[:, s].double().cpu().numpy() + delta)


def ik_cpu_baseline(q_host, tgt_host, prm, budget_s):
    O = _oracle()
    nth = host_threads()
    n = min(len(q_host), 4096)
    O.ik_dls(q_host[:64], tgt_host[:64], nthreads=1, **prm)  # load / warm
    done, reps, t0 = 0, 0, time.perf_counter()
    while True:
        O.ik_dls(q_host[:n], tgt_host[:n], nthreads=nth, **prm)
        done += n
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "solves/s", "cores": nth, "kind": "port", "cpu_quota": cpu_quota(),
            "host_cores": len(os.sched_getaffinity(0)),
            "sample": f"{reps} x {n} solves of the same C2 inputs (envs 0..{n - 1}), fp64 oracle "
                      f"oracle/oracle.c, {nth} pthreads, {dt:.1f} s"}


def run_ik(args, engine, model, rank, world, dist, steps=None, warmup=None, baseline=True, budget=None):
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    B = args.batch
    prm = workloads.IK_PARAMS[args.params]
    q0, tgt, q_host, tgt_host = ik_inputs(engine, model, rank, B, args.regime)
    dev = engine.device
    out = dict(q=torch.empty(B, 7, device=dev), final_pos=torch.empty(B, 3, device=dev),
               pos_error=torch.empty(B, device=dev), iterations=torch.empty(B, dtype=torch.int32, device=dev),
               flags=torch.empty(B, dtype=torch.uint8, device=dev))
    elapsed, kern_ms = _timed(lambda i: engine.ik_dls_into(q0, tgt, out, **prm), steps, warmup, dist,
                              per_call_events=False, ranks_out=RANK_LEGS.setdefault("ik", []))
    iters = out["iterations"].cpu().numpy()
    fl = out["flags"].cpu().numpy()
    achieved = IK_BYTES_PER_SOLVE * B / (kern_ms * 1e-3) / 1e9
    traffic, src = _traffic("pmc_traffic_ik.json", B)
    rec = {
        "metric": BASELINE_METRIC,
        "value": B * world * steps / elapsed,
        "unit": "solves/s",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (Philox seed 20250808, counter = global env index)",
        "config": {
            "workload": "C2: 4096 Panda instances, IK-only DLS (skills/ik_solver.py) batched per MI355X, free space",
            "envs_per_gpu": B, "global_envs": B * world, "regime": args.regime,
            "ik_params": prm, "parallelism": f"env-shard x{world} (no collective on the data path)",
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": src,
                     "kernel": "ik_dls_group_kernel<float>", "kernel_avg_ms": kern_ms,
                     "algorithmic_bytes_per_launch": IK_BYTES_PER_SOLVE * B},
        "ik_stats": {"mean_iterations": float(iters.mean()), "max_iterations": int(iters.max()),
                     "converged_frac": float((fl & 1).astype(bool).mean()),
                     "dls_iterations_per_s": float(iters.sum()) * world * steps / elapsed},
        "host_cores": len(os.sched_getaffinity(0)),
    }
    if baseline and rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = ik_cpu_baseline(q_host, tgt_host, prm, budget or args.cpu_budget)
    return rec


def launch_plan(gpus, environ):
    """How `bench.py --gpus N` runs.  Under a launcher (torchrun sets WORLD_SIZE) this process is
    one rank: ("run", WORLD_SIZE), and --gpus must agree with it.  Without one, N > 1 means
    ("spawn", N): this process starts the N rank processes itself (one per GPU, below); N = 1
    runs here.  --gpus omitted = WORLD_SIZE or 1."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise SystemExit(f"bench.py: --gpus {gpus} disagrees with WORLD_SIZE={ws} set by the launcher")
        return "run", ws
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {n}")
    return ("spawn", n) if n > 1 else ("run", 1)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, poll_s=0.2):
    """One process per GPU, started by this one BEFORE it touches the GPU (no HIP call here:
    `torch.cuda.device_count()` does not initialise the runtime): rank r gets RANK = LOCAL_RANK =
    r, WORLD_SIZE = n and a 127.0.0.1 rendezvous, i.e. exactly what `torch.distributed.run
    --nproc-per-node n` would give it, and selects device r itself.  If a rank fails the others
    are stopped (they would wait at the next barrier).  Returns the job's exit code."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(poll_s)
    return rc


def _launch_selftest(rank, world, expected):
    """--launch-selftest: the rank wiring alone (gloo, no GPU): every rank joins the group and
    the job's view of it is printed by rank 0 (tests/test_dist_cpu.py)."""
    torch.distributed.init_process_group("gloo")
    t = torch.tensor([rank, 1], dtype=torch.int64)
    torch.distributed.all_reduce(t)
    # the N > 1 record's "dist" block, built by the same code as a GPU run's (timings: a stand-in
    # "wall" of 1 + rank s)
    ident = gather_ranks(rank_identity(int(os.environ.get("LOCAL_RANK", "0")), "cpu"))
    legs = {"step": gather_ranks([1.0 + rank, 0.5 + rank])}
    drec = dist_record(expected, world, True, ident, legs)
    if rank == 0:
        print(json.dumps({"world": torch.distributed.get_world_size(), "rank_sum": int(t[0]), "ranks": int(t[1]),
                          "local_ranks": os.environ.get("LOCAL_RANK"), "dist": drec}), flush=True)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of the job; without torchrun, N > 1 starts N rank processes")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--workload", default="step", choices=("step", "ik"))
    ap.add_argument("--regime", default="waypoint", choices=sorted(workloads.IK_REGIMES))
    ap.add_argument("--params", default="default", choices=sorted(workloads.IK_PARAMS))
    ap.add_argument("--no-ik", action="store_true", help="step workload: skip the secondary C2 timing")
    ap.add_argument("--no-gym", action="store_true", help="step workload: skip the secondary fused gym-step timing")
    ap.add_argument("--no-tqc", action="store_true", help="step workload: skip the secondary C5 TQC-loop timing")
    ap.add_argument("--tqc-envs", type=int, default=8192, help="C5 envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (C3 leg)")
    ap.add_argument("--steady-burn", type=int, default=50,
                    help="gym / tqc legs: untimed steps of a long run before the steady-state timing (0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1: nccl (= RCCL over xGMI, one GPU per rank); gloo only to rehearse several "
                         "ranks on one GPU")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    mode, world = launch_plan(args.gpus, os.environ)
    if mode == "spawn":
        if not args.launch_selftest and args.dist_backend == "nccl" and torch.cuda.device_count() < world:
            raise SystemExit(f"bench.py: --gpus {world} with nccl needs {world} visible GPUs, "
                             f"found {torch.cuda.device_count()}")
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_selftest:
        _launch_selftest(rank, world, args.gpus if args.gpus is not None else world)
        return
    dist = world > 1
    if dist:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))   # (gloo rehearsal: ranks may share a GPU)
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    engine = get_engine()
    model = engine.model
    if args.workload == "step":
        rec = run_step(args, engine, model, rank, world, dist)
    else:
        rec = run_ik(args, engine, model, rank, world, dist)
    me = rank_identity(local, "cuda")
    ident = gather_ranks(me) if dist else [me]
    rec["dist"] = dist_record(args.gpus if args.gpus is not None else world, world, dist, ident, RANK_LEGS)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
