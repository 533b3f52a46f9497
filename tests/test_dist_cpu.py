"""Multi-rank path on CPU (gloo, world size 2, 127.0.0.1): the env shards of bench.py /
pnp_amd.envs reproduce the single-process batch bitwise, and the job time is the max over ranks.
(The GPU data path has no collective)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 24


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(rank, sx, sm):
    import bench
    from pnp_amd import workloads
    from pnp_amd.model import load_model
    m = load_model()
    idx = bench.shard_range(rank, B)
    st = workloads.c3_reset(m, idx, sx, sm)
    ctrl = np.stack([workloads.c3_ctrl(m, idx, s) for s in range(3)])
    q, d = workloads.ik_inputs(m, idx)
    return dict(qpos=st["qpos"], mocap=st["mocap_pos"], ctrl=ctrl, q=q, d=d)


def _worker(rank, world, port, sx, sm, out):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    mine = _inputs(rank, sx, sm)
    got = [None] * world
    dist.all_gather_object(got, mine)
    t = bench.reduce_max([1.0 + rank, 10.0 - rank], "cpu")
    if rank == 0:
        out.put((got, t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_match_global_batch(model):
    from oracle import oracle as O
    q = model.qpos0.copy()
    q[:9] = [0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00]
    sx, sm = O.site_kinematics(q[None], model=model)
    sx, sm = sx[0], sm[0]
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sx, sm, out)) for r in range(2)]
    for p in procs:
        p.start()
    got, t = out.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == [2.0, 10.0]                     # max over ranks
    # global batch of 2B envs generated in one process == the two shards concatenated
    import bench
    from pnp_amd import workloads
    idx = np.arange(2 * B)
    st = workloads.c3_reset(model, idx, sx, sm)
    ctrl = np.stack([workloads.c3_ctrl(model, idx, s) for s in range(3)])
    qi, d = workloads.ik_inputs(model, idx)
    cat = lambda k, ax=0: np.concatenate([g[k] for g in got], axis=ax)
    assert np.array_equal(cat("qpos"), st["qpos"])
    assert np.array_equal(cat("mocap"), st["mocap_pos"])
    assert np.array_equal(cat("ctrl", 1), ctrl)
    assert np.array_equal(cat("q"), qi) and np.array_equal(cat("d"), d)
    assert not np.array_equal(got[0]["qpos"], got[1]["qpos"])   # shards differ
    assert bench.shard_range(1, 4096)[0] == 4096


def test_launch_plan():
    """bench.py --gpus N: inside torchrun (WORLD_SIZE set) the flag must agree with the launcher;
    without one N > 1 starts N ranks itself."""
    import bench
    assert bench.launch_plan(None, {}) == ("run", 1)
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(None, {"WORLD_SIZE": "2"}) == ("run", 2)
    with pytest.raises(SystemExit):
        bench.launch_plan(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


@pytest.mark.timeout(300)
def test_bench_spawns_ranks_from_gpus_flag():
    """`python bench.py --gpus 2` with no launcher starts two rank processes that join one
    process group (the rank wiring is exercised with gloo, no GPU); a --gpus / WORLD_SIZE
    disagreement exits non-zero before any rank starts."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    d = rec.pop("dist")
    assert rec == {"world": 2, "rank_sum": 1, "ranks": 2, "local_ranks": "0"}
    # the record's dist block (bench.dist_record, the same code a GPU run prints): the process
    # group's own world size and backend, every rank with its own timings
    assert d["world_size"] == 2 and d["backend"] == "gloo" and d["gpus_flag"] == 2
    assert [x["rank"] for x in d["ranks"]] == [0, 1] and [x["local_rank"] for x in d["ranks"]] == [0, 1]
    assert [x["step_wall_s"] for x in d["ranks"]] == [1.0, 2.0]
    assert [x["step_kernel_ms"] for x in d["ranks"]] == [0.5, 1.5]
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-selftest"],
                         env=dict(env, WORLD_SIZE="2"), capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "disagrees" in bad.stderr


def test_dist_record_rejects_a_job_that_is_not_the_one_asked_for():
    """bench.dist_record raises (rank 0 prints no record) when the process group is not --gpus
    ranks, ranks are missing, or RCCL ranks share a GPU."""
    import bench
    one = [{"rank": 0, "local_rank": 0, "device": "cpu"}]
    rec = bench.dist_record(1, 1, False, one, {"step": [[2.0, 1.0]]})
    assert rec["world_size"] == 1 and rec["backend"] is None
    assert rec["ranks"][0]["step_wall_s"] == 2.0 and rec["ranks"][0]["step_kernel_ms"] == 1.0
    with pytest.raises(SystemExit, match="world size"):
        bench.dist_record(2, 1, False, one, {})
    with pytest.raises(SystemExit, match="not 0"):
        bench.dist_record(1, 1, False, [{"rank": 3, "local_rank": 0}], {})
