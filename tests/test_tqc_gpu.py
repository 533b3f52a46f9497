"""C5 on the device: the TQC learner (pnp_amd/tqc.py, reference scripts/train.py) driving the fused
gym env (libpnp.so pnp_env_step through pnp_amd.envs).

* reward / success parity vs the CPU reference env: the learner's own rollout (its actions, its
  auto-reset handling, its replay rows) is replayed through the env oracle (oracle/env_oracle.py:
  the reference's FrankaEnv logic over the fp64 physics oracle) on the short-physics configuration
  of tests/test_env_gpu.py (inside the scene's divergence horizon): rewards and observations within
  1e-9 (fp64 env), success / termination flags identical, replay rows = the env's outputs.
* the full C5 configuration (fp32, 250 sub-steps per gym step): rollout + gradient steps stay
  finite, and the replay buffer holds exactly what the env returned.
"""
import ctypes as C
import math

import numpy as np
import pytest
import torch

from oracle.env_oracle import EnvConfig as OCfg, EnvOracle

pytestmark = pytest.mark.gpu

SHORT = dict(n_substeps=2, n_calls=2)


def test_learner_rollout_matches_oracle_env(model):
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    from pnp_amd.tqc import TQC, TQCConfig, flat_obs
    B = 4
    env = BatchedFrankaShelfPNPEnv(B, dtype=torch.float64, config=EnvConfig(**SHORT))
    o = EnvOracle(B, cfg=OCfg(**SHORT), model=model)
    agent = TQC(env, TQCConfig(net_arch=(64, 64), batch_size=8, learning_starts=8, buffer_size=B * 16))
    agent.total_timesteps = 10 ** 6
    agent.reset()
    ref = o.reset()
    ref_flat = np.stack([np.concatenate([ref[b]["achieved_goal"], ref[b]["desired_goal"], ref[b]["observation"]])
                         for b in range(B)])
    np.testing.assert_allclose(flat_obs(agent._last_raw).double().cpu().numpy(), ref_flat, atol=1e-6)
    for k in range(8):
        reward, done, info = agent.collect_step()
        act = agent.buffer.actions[k].double().cpu().numpy()      # what the learner sent
        res = o.step(act)
        for b in range(B):
            assert abs(float(reward[b]) - res[b]["reward"]) < 1e-9
            assert float(info["is_success"][b]) == res[b]["is_success"]
            assert bool(done[b]) == (res[b]["terminated"] or res[b]["truncated"])
            want = np.concatenate([res[b]["obs"]["achieved_goal"], res[b]["obs"]["desired_goal"],
                                   res[b]["obs"]["observation"]])
            np.testing.assert_allclose(agent.buffer.next_obs[k, b].double().cpu().numpy(), want, atol=1e-6)
            assert float(agent.buffer.rewards[k, b]) == pytest.approx(res[b]["reward"], abs=1e-6)
            assert float(agent.buffer.dones[k, b]) == float(res[b]["terminated"])
        if agent.num_timesteps > agent.cfg.learning_starts:
            logs = agent.train()
            assert all(math.isfinite(v) for v in logs.values())


def test_c5_full_physics_learner_steps():
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    from pnp_amd.tqc import TQC, TQCConfig, flat_obs
    B = 256
    env = BatchedFrankaShelfPNPEnv(B)
    agent = TQC(env, TQCConfig(learning_starts=0))
    agent.total_timesteps = 10 ** 6
    agent.reset()
    for k in range(3):
        reward, done, info = agent.collect_step()
        assert torch.equal(agent.buffer.rewards[k], reward)
        assert torch.equal(agent.buffer.next_obs[k][~done], flat_obs(env._obs())[~done])
        logs = agent.train()
        assert all(math.isfinite(v) for v in logs.values()), logs
    assert bool(torch.isfinite(agent.buffer.next_obs[:3]).all())
    assert int((env.state["warn"] & 7).max()) == 0          # no bad-state resets
    for p in list(agent.actor.parameters()) + list(agent.critic.parameters()):
        assert bool(torch.isfinite(p).all())


@pytest.mark.timeout(600)
def test_c5_config_8192_envs():
    """BASELINE configs[4] at its own size: TQC (train.py hyper-parameters) over 8192 fused gym
    envs on one GPU, 2 collect + train steps: replay rows = env outputs, finite losses / weights,
    no bad-state reset, no capacity truncation (warn bits 0..4 clear)."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    from pnp_amd.tqc import TQC, TQCConfig, flat_obs
    B = 8192
    env = BatchedFrankaShelfPNPEnv(B)
    agent = TQC(env, TQCConfig(learning_starts=0))
    agent.total_timesteps = 2_000_000
    agent.reset()
    for k in range(2):
        reward, done, info = agent.collect_step()
        assert torch.equal(agent.buffer.rewards[k], reward)
        assert torch.equal(agent.buffer.next_obs[k][~done], flat_obs(env._obs())[~done])
        logs = agent.train()
        assert all(math.isfinite(v) for v in logs.values()), logs
    torch.cuda.synchronize()
    assert bool(torch.isfinite(agent.buffer.next_obs[:2]).all())
    assert bool(torch.isfinite(env.state["qpos"]).all()) and bool(torch.isfinite(env.state["qvel"]).all())
    w = env.state["warn"].to(torch.int64) & 0xFFFFFFFF
    assert int((w & 0x1F).max()) == 0, "bad-state reset or contact / row truncation"
    assert int((w >> 16).max()) == 0, "a tier hand-over bit leaked out of the call"


def test_captured_learner_step_equals_eager():
    """The HIP-graph gradient step of the PyTorch learner (TQC._capture: one captured update
    replayed gradient_steps times; the fused HIP step has its own tests below) gives the eager
    steps' results bit for bit -- same replay samples, same exploration
    noise (the generator is registered with the graph), fused Adam either way -- over 12 updates
    across two train() calls, and its learner step is faster than the eager one."""
    import time
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    from pnp_amd.tqc import TQC, TQCConfig
    B = 64
    agents = []
    for graph in (False, True):
        env = BatchedFrankaShelfPNPEnv(B, config=EnvConfig(**SHORT))
        a = TQC(env, TQCConfig(learning_starts=0, graph=graph, fused=False))
        a.total_timesteps = 10 ** 6
        a.reset()
        for _ in range(3):
            a.collect_step()
        agents.append(a)
    eager, graphed = agents
    for n in (5, 7):
        le, lg = eager.train(n), graphed.train(n)
        for k in ("critic_loss", "actor_loss", "ent_coef_loss", "ent_coef"):
            assert torch.equal(le[k], lg[k]), k
    assert graphed._graph is not None and eager._graph is None
    for name in ("actor", "critic", "critic_target"):
        for (kp, p), (_, q) in zip(getattr(eager, name).state_dict().items(), getattr(graphed, name).state_dict().items()):
            assert torch.equal(p, q), (name, kp)
    assert torch.equal(eager.log_ent_coef, graphed.log_ent_coef)
    ms = []
    for a in agents:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.train(50)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) / 50 * 1e3)
    print(f"learner step: eager {ms[0]:.3f} ms, captured {ms[1]:.3f} ms")
    assert ms[1] < ms[0]


def _fused_agent(B=64, env_offset=0, **cfg):
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    from pnp_amd.tqc import TQC, TQCConfig
    env = BatchedFrankaShelfPNPEnv(B, config=EnvConfig(**SHORT), env_offset=env_offset)
    a = TQC(env, TQCConfig(**cfg))
    a.total_timesteps = 10 ** 6
    a.reset()
    for _ in range(12):            # 768 transitions: past learning_starts and one batch
        a.collect_step()
    return a


def test_fused_sample_matches_pytorch():
    """pnp_tqc_sample (one launch) against DictReplayBuffer.sample + VecNormalize.normalize +
    flat_obs (pnp_amd/tqc.py TQC._sample_norm) from the same generator state: the same rows, the
    normalised observations bit for bit, on a partly filled buffer (indices below `upper`) and with
    statistics that clip (achieved_goal's variance shrunk so |x| > clip_obs)."""
    a = _fused_agent(graph=False, device_rng=False)   # u from the agent's generator, as _sample_norm's
    for trial in range(3):
        a.vecnorm.obs_rms["achieved_goal"].var.fill_(1e-12)   # these three columns clip at +-10
        gs = a.gen.get_state()
        ref = [t.clone() for t in a._sample_norm()]
        a.gen.set_state(gs)
        got = a._sample_fused()
        torch.cuda.synchronize()
        for name, x, y in zip(("obs", "act", "next_obs", "done", "reward"), got, ref):
            assert x.shape == y.shape and torch.equal(x, y), (trial, name, float((x - y).abs().max()))
        assert float(got[0][:, :3].abs().max()) == a.vecnorm.clip_obs > float(got[0][:, 3:].abs().max())
        a.collect_step()


@pytest.mark.parametrize("batch", [512, 48, 80])
def test_fused_learner_step_matches_pytorch(batch):
    """pnp_tqc_update (csrc/tqc_fused.hip: the whole TQC gradient step on the matrix cores) against
    the PyTorch step (pnp_amd/tqc.py _update_torch, autograd) from the same state, replay sample and
    Gaussian draws: every gradient tensor it applies within 1e-4 (critics) / 1e-3 (actor, computed
    against the Adam-updated critics) of the PyTorch gradient in norm, the logged losses within
    1e-4, and the parameters after Adam (actor, critics, Polyak targets, log entropy coefficient)
    within a small fraction of the learning rate.  train.py's batch (512) and two multiples of 16
    whose 16 weight-gradient waves get row ranges that are not multiples of the 4-row load group
    (48: 3 rows per wave, 80: 5; round 5 summed rows of the next wave twice there)."""
    _check_fused_against_pytorch(_fused_agent(graph=False, batch_size=batch))


def _check_fused_against_pytorch(a):
    """One fused step of agent `a` (eager; several ranks: the data-parallel split) against its
    PyTorch step from the same state and draws; returns the parameters after the fused step."""
    import copy
    from pnp_amd import _lib
    for _ in range(3):
        a.train()                  # the first creates the Adam state (PyTorch), then fused steps
    assert a._fdesc is not None
    L = _lib.load()
    na, nc = C.c_int32(), C.c_int32()
    L.pnp_tqc_param_counts(C.byref(na), C.byref(nc))
    na, nc = na.value, nc.value
    pa, pc, pt = a._fused_params()
    a.cfg.device_rng = False       # this step's draws from the generator, like the PyTorch step's
    sd = copy.deepcopy(a.state_dict())
    gs = a.gen.get_state()
    g = torch.zeros(na + nc, device=a.device)
    lf = [float(t) for t in a._update_fused(g)]
    after_f = [p.detach().clone() for p in pa + pc + pt] + [a.log_ent_coef.detach().clone()]
    a.load_state_dict(sd)
    a.gen.set_state(gs)
    rec = {}
    lt = [float(t) for t in a._update_torch(rec)]
    after_t = [p.detach().clone() for p in pa + pc + pt] + [a.log_ent_coef.detach().clone()]
    byid = {id(p): gr for p, gr in zip(list(a.actor.parameters()), rec["actor"])}
    byid.update({id(p): gr for p, gr in zip(list(a.critic.parameters()), rec["critic"])})
    o = 0
    worst = {}
    for name, ps in (("actor", pa), ("critic", pc)):
        for i, p in enumerate(ps):
            n = p.numel()
            gf, gt = g[o:o + n].view_as(p), byid[id(p)]
            o += n
            e = float((gf - gt).norm() / gt.norm().clamp_min(1e-30))
            worst[f"{name}{i}"] = e
            assert e < (1e-4 if name == "critic" else 1e-3), (name, i, e)
    print("fused vs PyTorch gradient (relative norm):", {k: f"{v:.1e}" for k, v in worst.items()})
    print("logs fused", lf, "PyTorch", lt)
    for x, y in zip(lf, lt):
        assert abs(x - y) <= 1e-4 * max(1.0, abs(y)), (lf, lt)
    lr = float(a._lr)
    for x, y in zip(after_f, after_t):
        d = (x - y).abs()
        assert float(d.max()) <= 2.5 * lr and float(d.median()) <= 1e-3 * lr, (float(d.max()), float(d.median()), lr)
    return after_f


def test_fused_draw_counter_survives_checkpoint(tmp_path):
    """A run resumed from a checkpoint continues the device draw stream (pnp_tqc_sample_draw's
    counter, `fused_rng_draws`) instead of replaying it from index 0: a freshly built agent that
    loads the checkpoint draws, at its first fused step, what the original agent draws at its next."""
    a = _fused_agent(graph=False)
    a.train(4)                     # one PyTorch step (Adam state), three fused: counter at 3
    torch.cuda.synchronize()
    assert int(a._fctr[0]) == 3
    p = tmp_path / "tqc.pt"
    a.save(p)
    b = _fused_agent(graph=False)
    b.load(p)
    assert int(b._fctr[0]) == 3, int(b._fctr[0])
    ua = [t.clone() for t in a._sample_fused()]
    ub = [t.clone() for t in b._sample_fused()]
    torch.cuda.synchronize()
    assert torch.equal(a._fu_dev, b._fu_dev) and torch.equal(a._feps[0], b._feps[0])
    logs = a.train()               # eager fused step: the returned logs are copies
    kept = float(logs["critic_loss"])
    a.train()
    assert float(logs["critic_loss"]) == kept


def _dp_fused_worker(rank, world, port, out):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mujoco-panda-pnp_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import test_tqc_gpu as T
        a = T._fused_agent(graph=False, env_offset=64 * rank)
        a.train(3)                 # a PyTorch step (Adam state), then two data-parallel fused steps
        assert a._fused_ok() and a._fdesc is not None and a._fgrads is not None
        a.cfg.device_rng = False   # the compared step: draws from the per-rank generator
        after = T._check_fused_against_pytorch(a)
        a.train(2)
        flat = torch.cat([p.detach().reshape(-1) for p in list(a.actor.parameters()) + list(a.critic.parameters())])
        res = dict(params=flat.cpu().numpy(), batch=a._fsb[0].cpu().numpy(),
                   after=torch.cat([t.reshape(-1) for t in after]).cpu().numpy())
        got = [None] * world
        dist.all_gather_object(got, res)
        if rank == 0:
            out.put(got)
        dist.barrier()
    except BaseException as e:   # report instead of hanging the other rank's collective
        out.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_fused_learner_data_parallel_two_ranks():
    """the fused step on two ranks (one GPU, gloo: RCCL refuses two ranks on one
    device) runs pnp_tqc_update_phase with the gradients all-reduced between the phases.  On each
    rank the step matches the data-parallel PyTorch step (_update_torch, whose gradients are
    all-reduced the same way) on the bars of test_fused_learner_step_matches_pytorch, the ranks'
    batches differ, and after further steps both ranks hold the same parameters bit for bit."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    procs = [ctx.Process(target=_dp_fused_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    got = out.get(timeout=280)
    for p in procs:
        p.join(60)
    assert not isinstance(got, str), got
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r0, r1 = got
    assert not np.array_equal(r0["batch"], r1["batch"])        # each rank its own replay sample
    assert np.array_equal(r0["after"], r1["after"])            # the averaged step, identical
    assert np.array_equal(r0["params"], r1["params"])          # lockstep after two more steps


def test_fused_device_draws():
    """pnp_tqc_sample_draw (TQC.train's default, cfg.device_rng): the batch's two U[0, 1) replay
    draws and the actor's two N(0, 1) draws per row from Philox on the device, at the draw index
    the gradient step advances on the device (pnp_tqc_desc.draw_counter: one per step).  The uniform
    draws it reports give, through pnp_tqc_sample, the same batch bit for bit; the draws have the
    moments of U[0, 1) and N(0, 1) (64 indices: 65,536 uniforms, 458,752 Gaussians); consecutive
    indices draw different numbers, the same index the same ones."""
    from pnp_amd import _lib
    L = _lib.load()
    a = _fused_agent(graph=False)
    assert a.cfg.device_rng
    a.train()                      # the first (PyTorch) step builds the fused descriptors' state
    r = a._fused_replay()
    B = a.cfg.batch_size
    a.train(3)                     # fused steps: the draw index advances once per step
    torch.cuda.synchronize()
    assert int(a._fctr[0]) == 3, int(a._fctr[0])
    us, es = [], []
    for k in range(64):
        if k:
            a._fctr[0] += 1            # what the next gradient step would do
        got = [t.clone() for t in a._sample_fused()]
        u = a._fu_dev.clone()
        us.append(u)
        es.append(torch.cat([e.clone().flatten() for e in a._feps]))
        if k < 3:
            ref = [torch.empty_like(t) for t in got]
            _lib.check(L.pnp_tqc_sample(C.byref(r), u.data_ptr(), B, *[t.data_ptr() for t in ref], None), "pnp_tqc_sample")
            torch.cuda.synchronize()
            for name, x, y in zip(("obs", "act", "next_obs", "done", "reward"), got, ref):
                assert torch.equal(x, y), (k, name)
    again = [t.clone() for t in a._sample_fused()]   # the same index: the same draws
    torch.cuda.synchronize()
    assert torch.equal(a._fu_dev, us[-1]) and torch.equal(again[0], got[0])
    U, E = torch.stack(us).double(), torch.stack(es).double()
    assert float(U.min()) >= 0.0 and float(U.max()) < 1.0
    assert abs(float(U.mean()) - 0.5) < 0.005 and abs(float(U.var()) - 1 / 12) < 0.002
    # (bounds ~5 standard errors of each moment at these sample sizes)
    assert abs(float(E.mean())) < 0.008 and abs(float(E.var()) - 1.0) < 0.01
    assert abs(float((E ** 3).mean())) < 0.03 and abs(float((E ** 4).mean()) - 3.0) < 0.08
    assert not torch.equal(us[0], us[1]) and not torch.equal(es[0], es[1])


def test_fused_learner_step_captured_and_timed():
    """The fused step inside TQC.train (HIP-graph captured, replayed gradient_steps times) equals
    the uncaptured fused step bit for bit (fixed-order reductions, no atomics), stays finite, and
    is timed against the PyTorch captured step (printed; the bench's tqc leg records both)."""
    import time
    agents = [_fused_agent(graph=g) for g in (False, True)]
    for n in (5, 7):
        le, lg = agents[0].train(n), agents[1].train(n)
        for k in ("critic_loss", "actor_loss", "ent_coef_loss", "ent_coef"):
            assert torch.equal(le[k], lg[k]), k
            assert math.isfinite(float(le[k])), k
    assert agents[1]._graph is not None and agents[0]._fdesc is not None
    for name in ("actor", "critic", "critic_target"):
        for (kp, p), (_, q) in zip(getattr(agents[0], name).state_dict().items(),
                                   getattr(agents[1], name).state_dict().items()):
            assert torch.equal(p, q), (name, kp)
    ref = _fused_agent(graph=True, fused=False)
    ms = []
    for a in (agents[1], ref):
        a.train(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.train(200)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) / 200 * 1e3)
    print(f"learner step (captured): fused HIP {ms[0]:.3f} ms, PyTorch {ms[1]:.3f} ms")
    assert ms[0] < ms[1]
