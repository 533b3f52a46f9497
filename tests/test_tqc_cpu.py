"""TQC learner (pnp_amd/tqc.py; the C5 caller, reference scripts/train.py:63-116) on CPU: its parts
against direct restatements of the sb3 / sb3-contrib 2.2.1 formulas, the rollout / replay
semantics on a toy dict-obs vector env with the BatchedFrankaShelfPNPEnv step contract, checkpoint
round trips, and the data-parallel path on two gloo ranks.  sb3 itself is absent, so
the formulas are the published ones, restated in the test."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pnp_amd import tqc as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class ToyReach:
    """num_envs point masses in 3-D reaching a goal; obs dict like FrankaShelfPNP (19 / 3 / 3),
    reward = -distance, terminated within 0.05, truncated after `horizon` steps, auto-reset with
    final_* in info (the BatchedFrankaShelfPNPEnv contract)."""

    def __init__(self, num_envs, horizon=20, seed=0, scale=1.0):
        self.scale = scale
        self.num_envs, self.horizon = num_envs, horizon
        self.device = torch.device("cpu")
        self.g = torch.Generator().manual_seed(seed)
        self.pos = torch.zeros(num_envs, 3)
        self.goal = torch.zeros(num_envs, 3)
        self.t = torch.zeros(num_envs, dtype=torch.int32)

    def _reset_idx(self, m):
        n = int(m.sum())
        self.pos[m] = torch.rand(n, 3, generator=self.g) - 0.5
        self.goal[m] = torch.rand(n, 3, generator=self.g) - 0.5
        self.t[m] = 0

    def _obs(self):
        o = torch.zeros(self.num_envs, 19)
        o[:, :3] = self.pos
        o[:, 3:6] = self.goal - self.pos
        return {"observation": o, "achieved_goal": self.pos.clone(), "desired_goal": self.goal.clone()}

    def reset(self, mask=None):
        self._reset_idx(torch.ones(self.num_envs, dtype=torch.bool) if mask is None else mask.bool())
        return self._obs()

    def step(self, a):
        self.pos += 0.05 * a[:, :3].clamp(-1, 1)
        self.t += 1
        d = torch.linalg.norm(self.pos - self.goal, dim=1)
        r = -self.scale * d
        term = d < 0.05
        trunc = (self.t >= self.horizon) & ~term
        info = {"is_success": term.float()}
        fin = self._obs()
        info.update(final_observation=fin["observation"], final_achieved_goal=fin["achieved_goal"],
                    final_desired_goal=fin["desired_goal"])
        done = term | trunc
        if bool(done.any()):
            self._reset_idx(done)
        return self._obs(), r, term, trunc, info


def test_quantile_huber_loss_matches_loop():
    g = torch.Generator().manual_seed(1)
    cur = torch.randn(4, 2, 5, generator=g) * 2
    tgt = torch.randn(4, 1, 8, generator=g) * 2
    got = T.quantile_huber_loss(cur, tgt)
    tot, n = 0.0, 0
    for b in range(4):
        for c in range(2):
            for i in range(5):
                tau = (i + 0.5) / 5
                for j in range(8):
                    u = float(tgt[b, 0, j] - cur[b, c, i])
                    h = abs(u) - 0.5 if abs(u) > 1 else 0.5 * u * u
                    tot += abs(tau - (1.0 if u < 0 else 0.0)) * h
                    n += 1
    assert abs(float(got) - tot / n) < 1e-6
    got_sum = T.quantile_huber_loss(cur, tgt, sum_over_quantiles=True)
    assert abs(float(got_sum) - tot / n * 5) < 1e-5


def test_running_mean_std_is_the_pooled_moments():
    rng = np.random.default_rng(0)
    rms = T.RunningMeanStd((4,), "cpu")
    chunks = [rng.normal(3, 2, size=(n, 4)) for n in (7, 50, 1, 33)]
    for c in chunks:
        rms.update(torch.as_tensor(c))
    allx = np.concatenate(chunks)
    eps = 1e-4     # initial count with mean 0, var 1
    n = len(allx)
    mean = allx.sum(0) / (n + eps)
    m2 = ((allx - allx.mean(0)) ** 2).sum(0) + eps * 1.0 + (allx.mean(0) ** 2) * eps * n / (n + eps)
    np.testing.assert_allclose(rms.mean.numpy(), mean, rtol=1e-10)
    np.testing.assert_allclose(rms.var.numpy(), m2 / (n + eps), rtol=1e-9)
    assert abs(rms.count - (n + eps)) < 1e-9


def test_vecnormalize_clip_and_eps():
    vn = T.VecNormalize({"x": 2}, "cpu", clip_obs=10.0)
    vn.obs_rms["x"].mean = torch.tensor([1.0, -1.0], dtype=torch.float64)
    vn.obs_rms["x"].var = torch.tensor([4.0, 1e-6], dtype=torch.float64)
    out = vn.normalize({"x": torch.tensor([[3.0, 5.0]])})["x"]
    assert abs(float(out[0, 0]) - 2.0 / math.sqrt(4.0 + 1e-8)) < 1e-6
    assert float(out[0, 1]) == 10.0


def test_actor_log_prob_is_squashed_gaussian():
    torch.manual_seed(0)
    actor = T.Actor(25, 7, (32, 32))
    x = torch.randn(16, 25)
    g = torch.Generator().manual_seed(5)
    a, lp = actor.action_log_prob(x, g)
    mu, log_std = actor.dist_params(x)
    eps = torch.randn(mu.shape, generator=torch.Generator().manual_seed(5))
    gauss = mu + log_std.exp() * eps
    ref = torch.distributions.Normal(mu, log_std.exp()).log_prob(gauss).sum(-1)
    ref = ref - torch.log(1 - torch.tanh(gauss) ** 2 + 1e-6).sum(-1)
    torch.testing.assert_close(a, torch.tanh(gauss))
    torch.testing.assert_close(lp, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(actor(x, deterministic=True), torch.tanh(mu))


def test_critic_stack_equals_separate_mlps():
    torch.manual_seed(0)
    cr = T.QuantileCritics(25, 7, (16, 16), 2, 25)
    o, a = torch.randn(9, 25), torch.randn(9, 7)
    q = cr(o, a)
    assert q.shape == (9, 2, 25)
    for c in range(2):
        h = torch.cat([o, a], 1)
        for k in range(3):
            h = h @ cr.weights[k][c] + cr.biases[k][c]
            if k < 2:
                h = torch.relu(h)
        torch.testing.assert_close(q[:, c], h)


def test_rollout_stores_terminal_obs_and_terminated_only():
    env = ToyReach(8, horizon=3)
    m = T.TQC(env, T.TQCConfig(net_arch=(16, 16), buffer_size=64, batch_size=8, learning_starts=10 ** 9))
    m.reset()
    prev = T.flat_obs(m._last_raw).clone()
    for _ in range(3):
        _, done, info = m.collect_step()
    b = m.buffer
    assert b.pos == 3 and not b.full
    # row 0's obs = the reset obs; the third step truncates every env (horizon 3)
    torch.testing.assert_close(b.obs[0], prev)
    assert bool(done.all())
    fin = T.flat_obs({"observation": info["final_observation"], "achieved_goal": info["final_achieved_goal"],
                      "desired_goal": info["final_desired_goal"]})
    torch.testing.assert_close(b.next_obs[2], fin)
    assert torch.equal(b.dones[2], info["is_success"])          # terminated only (truncation is not)
    # obs statistics: reset + 3 steps of 8 envs
    assert abs(m.vecnorm.obs_rms["observation"].count - (32 + 1e-4)) < 1e-9
    # wrap-around (size = 64 // 8 = 8 rows)
    for _ in range(6):
        m.collect_step()
    assert b.full and b.pos == 1
    o, a, no, d, r = b.sample(5)
    assert o.shape == (5, 25) and a.shape == (5, 7) and d.shape == (5, 1) and r.shape == (5, 1)


def test_train_step_targets_and_polyak():
    env = ToyReach(16)
    cfg = T.TQCConfig(net_arch=(32, 32), buffer_size=1024, batch_size=64, learning_starts=0)
    m = T.TQC(env, cfg)
    m.total_timesteps = 10 ** 6
    m.reset()
    for _ in range(5):
        m.collect_step()
    tgt0 = [p.clone() for p in m.critic_target.parameters()]
    crit0 = [p.clone() for p in m.critic.parameters()]
    logs = m.train()
    assert all(math.isfinite(v) for v in logs.values())
    assert abs(logs["lr"] - 3e-4 * (1 - 80 / 10 ** 6)) < 1e-12
    for t0, c0, t1, c1 in zip(tgt0, crit0, m.critic_target.parameters(), m.critic.parameters()):
        torch.testing.assert_close(t1, 0.995 * t0 + 0.005 * c1, rtol=1e-5, atol=1e-7)
        assert torch.equal(t0, c0)          # the target starts as a copy
    assert m.log_ent_coef.item() != 0.0    # the entropy coefficient moved


def test_target_quantiles_drop_top_per_net():
    """The TD target of one gradient step, recomputed by hand (sb3-contrib tqc.py train())."""
    env = ToyReach(4)
    cfg = T.TQCConfig(net_arch=(8,), n_quantiles=5, top_quantiles_to_drop_per_net=2, batch_size=3)
    m = T.TQC(env, cfg)
    no = torch.randn(3, 25)
    na = torch.rand(3, 7) * 2 - 1
    q = m.critic_target(no, na)                       # [3, 2, 5]
    srt, _ = torch.sort(q.reshape(3, -1))
    kept = srt[:, :6]                                 # 10 - 2 * 2
    for b in range(3):
        allq = sorted(q[b].reshape(-1).tolist())
        np.testing.assert_allclose(kept[b].detach().numpy(), allq[:6], rtol=1e-6)


def test_learning_improves_toy_reach():
    """End to end: the learner solves a reaching task (dense reward -10 * distance) that a random
    policy does not."""
    torch.manual_seed(0)
    env = ToyReach(32, horizon=20, seed=1, scale=10)
    cfg = T.TQCConfig(net_arch=(64, 64), buffer_size=20000, batch_size=128, learning_starts=320,
                      gradient_steps=4, learning_rate=1e-3, gamma=0.9, ent_coef_init=0.05)
    m = T.TQC(env, cfg)
    m.learn(32 * 300)
    m.vecnorm.training = False
    r, s = m.evaluate(ToyReach(64, horizon=20, seed=99, scale=10), 64)
    rand_env = ToyReach(64, horizon=20, seed=99, scale=10)
    rand_env.reset()
    rr = torch.zeros(64)
    live = torch.ones(64, dtype=torch.bool)
    for _ in range(20):
        _, rw, te, tr, _ = rand_env.step(torch.rand(64, 7) * 2 - 1)
        rr += rw * live
        live &= ~(te | tr)
    assert s > 0.5 and r > float(rr.mean()) + 50.0, (r, s, float(rr.mean()))


def test_checkpoint_round_trip(tmp_path):
    env = ToyReach(8)
    cfg = T.TQCConfig(net_arch=(16,), buffer_size=256, batch_size=16, learning_starts=0)
    m = T.TQC(env, cfg)
    m.total_timesteps = 1000
    m.reset()
    for _ in range(3):
        m.collect_step()
        m.train()
    p = tmp_path / "tqc.pt"
    m.save(p)
    m2 = T.TQC(ToyReach(8), T.TQCConfig(net_arch=(16,), buffer_size=256, batch_size=16, seed=7))
    m2.load(p)
    for a, b in zip(m.actor.parameters(), m2.actor.parameters()):
        assert torch.equal(a, b)
    for k in T.OBS_KEYS:
        assert torch.equal(m.vecnorm.obs_rms[k].mean, m2.vecnorm.obs_rms[k].mean)
    assert m2.num_timesteps == m.num_timesteps and m2.n_updates == m.n_updates


# ----------------------------------------------------------------------------- data parallel
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, out):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pnp_amd import tqc as TT
    env = ToyReach(8, seed=10 + rank)
    m = TT.TQC(env, TT.TQCConfig(net_arch=(16, 16), buffer_size=512, batch_size=16, learning_starts=0))
    m.total_timesteps = 10 ** 4
    m.reset()
    obs_seen = [T.flat_obs(m._last_raw).clone()]
    for _ in range(4):
        m.collect_step()
        obs_seen.append(T.flat_obs(m._last_raw).clone())
        m.train()
    params = torch.cat([p.detach().reshape(-1) for p in list(m.actor.parameters()) + list(m.critic.parameters())])
    mine = dict(params=params, mean=m.vecnorm.obs_rms["observation"].mean.clone(),
                var=m.vecnorm.obs_rms["observation"].var.clone(), obs=torch.stack(obs_seen))
    got = [None] * world
    dist.all_gather_object(got, mine)
    if rank == 0:      # numpy: torch tensors would travel as shared-memory handles of this process
        out.put([{k: v.numpy() for k, v in g.items()} for g in got])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_ranks_stay_in_lockstep():
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    got = out.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    a, b = [{k: torch.from_numpy(v) for k, v in g.items()} for g in got]
    assert torch.equal(a["params"], b["params"])              # averaged gradients, same steps
    assert not torch.equal(a["obs"], b["obs"])                # different env shards
    torch.testing.assert_close(a["mean"], b["mean"])          # merged statistics
    # the merged statistics are those of the pooled observations of both ranks
    rms = T.RunningMeanStd((19,), "cpu")
    for i in range(a["obs"].shape[0]):
        rms.update(torch.cat([a["obs"][i], b["obs"][i]])[:, 6:])
    torch.testing.assert_close(rms.mean, a["mean"], rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(rms.var, a["var"], rtol=1e-9, atol=1e-12)
