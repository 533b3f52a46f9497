"""TQC learner over the batched device env — the C5 caller of the hot path (reference
scripts/train.py:63-116: sb3-contrib 2.2.1 ``TQC("MultiInputPolicy", VecNormalize(SubprocVecEnv))``).

sb3 / sb3-contrib are not installed here, so this restates their published algorithm with the
reference's hyper-parameters (train.py:74-93) and keeps every tensor on the env's device:

* ``VecNormalize``  obs normalisation per dict key (norm_obs=True, norm_reward=False, clip 10,
  eps 1e-8; running mean / var with count initialised to 1e-4), updated on reset and on every
  step with the post-auto-reset observations (sb3 vec_normalize.py semantics).  Across ranks the
  batch moments are summed before the update, so every rank holds the same statistics.
* ``DictReplayBuffer``  raw (un-normalised) obs / next obs / action / reward / done, capacity
  ``buffer_size // n_envs`` rows of ``n_envs`` transitions; next obs of an ended episode is its
  terminal observation; ``done`` = terminated (TimeLimit truncation is not a terminal:
  handle_timeout_termination); samples are normalised with the current statistics.
* Policy: features = concat(achieved_goal, desired_goal, observation) (the Dict space's sorted
  keys, CombinedExtractor), actor MLP [256, 256, 256] ReLU -> mu, log_std (clamped to
  [-20, 2]) -> tanh-squashed Gaussian (log-prob correction eps 1e-6); ``log_std_init`` only
  applies to gSDE in sb3, which train.py does not enable, so it has no effect there or here.
  Critics: 2 quantile networks [256, 256, 256] -> 25 quantiles, held as one batched weight stack
  (one bmm per layer for both critics), a Polyak-averaged target copy (tau 0.005, every step).
* ``train()`` per gradient step (sb3-contrib tqc.py order): entropy-coefficient loss
  (target entropy -dim(A), log-coef starts at 0), critic loss = quantile Huber loss against the
  sorted target quantiles with the top 2 per net dropped, actor loss = ent_coef * log_prob -
  mean quantile; linear learning-rate schedule 3e-4 * progress_remaining for all three Adam
  optimisers; gamma 0.95, batch 512, learning_starts 100, train_freq 1, gradient_steps 1.

Multi-GPU: one process per GPU, each with its own env batch and replay buffer;
gradients are averaged with one all-reduce per optimiser (a single flattened bucket over RCCL /
xGMI), parameters start from rank 0's, and obs statistics are merged as above, so the ranks stay
in lockstep (data-parallel learner).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import math
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

OBS_KEYS = ("achieved_goal", "desired_goal", "observation")   # gymnasium Dict sorts its keys


@dataclasses.dataclass
class TQCConfig:
    """train.py:74-93 plus the sb3 / sb3-contrib defaults it relies on."""
    learning_rate: float = 3e-4          # linear_schedule(3e-4)
    buffer_size: int = 500_000
    batch_size: int = 512
    gamma: float = 0.95
    tau: float = 0.005
    learning_starts: int = 100           # OffPolicyAlgorithm default
    train_freq: int = 1
    gradient_steps: int = 1
    target_update_interval: int = 1
    n_critics: int = 2
    n_quantiles: int = 25
    top_quantiles_to_drop_per_net: int = 2
    net_arch: tuple = (256, 256, 256)
    log_std_init: float = -3.0           # gSDE only (no effect without use_sde, as in sb3)
    ent_coef_init: float = 1.0           # ent_coef="auto"
    clip_obs: float = 10.0               # VecNormalize
    norm_eps: float = 1e-8
    seed: int = 0
    # one gradient step captured in a HIP graph and replayed gradient_steps times per train() (single
    # process only; the data-parallel learner all-reduces eagerly)
    graph: bool = True
    # the hand-written fused gradient step (csrc/tqc_fused.hip, pnp_tqc_update) when the shapes are
    # train.py's (obs 25, action 7, [256, 256, 256], 2 x 25 quantiles, batch a multiple of 16);
    # with several ranks its data-parallel split (pnp_tqc_update_phase: the gradients all-reduced
    # between the phases); else (and for the first gradient step, which creates the optimisers'
    # state) the PyTorch step
    fused: bool = True
    # the fused step's random numbers (replay indices, the actor's two Gaussian draws) drawn on the
    # device with the replay sample (pnp_tqc_sample_draw: Philox keyed by `seed`, a device draw
    # counter) instead of by the agent's torch generator: three generator kernels and the captured
    # graph's generator bookkeeping less per gradient step.  Same distributions, other numbers
    # than the generator's; False draws from the generator (the tests' bit-exact comparisons)
    device_rng: bool = True


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


# ----------------------------------------------------------------------------- normalisation
class RunningMeanStd:
    """sb3 common/running_mean_std.py (parallel-variance update), fp64 on the device."""

    def __init__(self, shape, device, epsilon=1e-4):
        self.mean = torch.zeros(shape, dtype=torch.float64, device=device)
        self.var = torch.ones(shape, dtype=torch.float64, device=device)
        self.count = epsilon

    def update(self, x):
        x = x.to(torch.float64)
        n = x.shape[0]
        s, ss = x.sum(0), (x * x).sum(0)
        if _world() > 1:                  # sum the batch moments over ranks (one all-reduce)
            buf = torch.cat([s, ss, torch.tensor([float(n)], dtype=torch.float64, device=x.device)])
            dist.all_reduce(buf)
            d = s.numel()
            s, ss, n = buf[:d], buf[d:2 * d], float(buf[-1])
        bmean = s / n
        bvar = torch.clamp(ss / n - bmean * bmean, min=0.0)
        self.update_from_moments(bmean, bvar, n)

    def update_from_moments(self, bmean, bvar, bcount):
        # in place: the captured learner step (TQC._capture) reads mean / var at fixed addresses
        delta = bmean - self.mean
        tot = self.count + bcount
        m2 = self.var * self.count + bvar * bcount + delta * delta * self.count * bcount / tot
        self.mean.copy_(self.mean + delta * bcount / tot)
        self.var.copy_(m2 / tot)
        self.count = tot

    def state_dict(self):
        return {"mean": self.mean, "var": self.var, "count": torch.tensor(self.count, dtype=torch.float64)}

    def load_state_dict(self, d):
        self.mean.copy_(d["mean"].to(self.mean))
        self.var.copy_(d["var"].to(self.var))
        self.count = float(d["count"])


class VecNormalize:
    """Observation normalisation of a dict-obs vector env (norm_obs=True, norm_reward=False)."""

    def __init__(self, dims, device, clip_obs=10.0, epsilon=1e-8):
        self.obs_rms = {k: RunningMeanStd((d,), device) for k, d in dims.items()}
        self.clip_obs, self.epsilon = clip_obs, epsilon
        self.training = True

    def update(self, obs):
        if self.training:
            for k, rms in self.obs_rms.items():
                rms.update(obs[k])

    def normalize(self, obs):
        out = {}
        for k, rms in self.obs_rms.items():
            x = (obs[k].to(torch.float64) - rms.mean) / torch.sqrt(rms.var + self.epsilon)
            out[k] = torch.clamp(x, -self.clip_obs, self.clip_obs).to(torch.float32)
        return out

    def state_dict(self):
        return {k: r.state_dict() for k, r in self.obs_rms.items()}

    def load_state_dict(self, d):
        for k, r in self.obs_rms.items():
            r.load_state_dict(d[k])


def flat_obs(obs):
    """CombinedExtractor: flatten and concatenate the dict keys in sorted order -> [B, 25]."""
    return torch.cat([obs[k].reshape(obs[k].shape[0], -1).to(torch.float32) for k in OBS_KEYS], dim=1)


# ----------------------------------------------------------------------------- replay buffer
class DictReplayBuffer:
    """sb3 DictReplayBuffer (optimize_memory_usage=False, handle_timeout_termination=True) on the
    device; the dict keys are stored flattened (flat_obs order)."""

    def __init__(self, buffer_size, n_envs, obs_dim, act_dim, device):
        self.size = max(buffer_size // n_envs, 1)
        self.n_envs = n_envs
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=device)
        self.obs = z(self.size, n_envs, obs_dim)
        self.next_obs = z(self.size, n_envs, obs_dim)
        self.actions = z(self.size, n_envs, act_dim)
        self.rewards = z(self.size, n_envs)
        self.dones = z(self.size, n_envs)
        self.pos, self.full = 0, False
        self.device = device
        # rows filled so far, on the device: sample() draws indices from it without a host value,
        # so the captured learner step samples the buffer as it grows
        self.upper = torch.zeros((), dtype=torch.float32, device=device)

    def add(self, obs, next_obs, action, reward, done):
        self.obs[self.pos].copy_(obs)
        self.next_obs[self.pos].copy_(next_obs)
        self.actions[self.pos].copy_(action)
        self.rewards[self.pos].copy_(reward)
        self.dones[self.pos].copy_(done)
        self.pos += 1
        if self.pos == self.size:
            self.full, self.pos = True, 0
        self.upper.fill_(float(self.size if self.full else self.pos))

    def sample(self, batch_size, generator=None):
        """Uniform (row, env) pairs over the filled rows: floor(U[0, 1) * upper), the row count read
        on the device (sb3 samples the same distribution with randint on the host's upper bound)."""
        u = torch.rand(2, batch_size, device=self.device, generator=generator)
        bi = torch.clamp((u[0] * self.upper).long(), max=self.size - 1)
        ei = torch.clamp((u[1] * self.n_envs).long(), max=self.n_envs - 1)
        return (self.obs[bi, ei], self.actions[bi, ei], self.next_obs[bi, ei], self.dones[bi, ei, None],
                self.rewards[bi, ei, None])


# ----------------------------------------------------------------------------- networks
def _mlp(sizes):
    layers = []
    for a, b in zip(sizes[:-1], sizes[1:]):
        layers += [nn.Linear(a, b), nn.ReLU()]
    return nn.Sequential(*layers)


class Actor(nn.Module):
    """sb3 SAC/TQC Actor without gSDE: latent MLP -> (mu, log_std) -> squashed Gaussian."""
    LOG_STD_MIN, LOG_STD_MAX, EPS = -20.0, 2.0, 1e-6

    def __init__(self, obs_dim, act_dim, net_arch):
        super().__init__()
        self.latent = _mlp((obs_dim,) + tuple(net_arch))
        self.mu = nn.Linear(net_arch[-1], act_dim)
        self.log_std = nn.Linear(net_arch[-1], act_dim)

    def dist_params(self, x):
        h = self.latent(x)
        return self.mu(h), torch.clamp(self.log_std(h), self.LOG_STD_MIN, self.LOG_STD_MAX)

    def action_log_prob(self, x, generator=None):
        mu, log_std = self.dist_params(x)
        std = log_std.exp()
        eps = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype, generator=generator)
        g = mu + std * eps
        a = torch.tanh(g)
        # Normal(mu, std).log_prob(g).sum(-1) - sum(log(1 - tanh(g)^2 + eps))
        lp = (-0.5 * eps * eps - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        lp = lp - torch.log(1 - a * a + self.EPS).sum(-1)
        return a, lp

    def forward(self, x, deterministic=False, generator=None):
        if deterministic:
            return torch.tanh(self.dist_params(x)[0])
        return self.action_log_prob(x, generator)[0]


class QuantileCritics(nn.Module):
    """n_critics quantile networks as one stacked MLP: layer k weight [n_critics, in, out]; each
    critic's slice initialised like nn.Linear (U(+-1/sqrt(in)))."""

    def __init__(self, obs_dim, act_dim, net_arch, n_critics, n_quantiles):
        super().__init__()
        sizes = (obs_dim + act_dim,) + tuple(net_arch) + (n_quantiles,)
        self.weights = nn.ParameterList()
        self.biases = nn.ParameterList()
        for a, b in zip(sizes[:-1], sizes[1:]):
            bound = 1.0 / math.sqrt(a)
            w = torch.empty(n_critics, a, b).uniform_(-bound, bound)
            bb = torch.empty(n_critics, 1, b).uniform_(-bound, bound)
            self.weights.append(nn.Parameter(w))
            self.biases.append(nn.Parameter(bb))
        self.n_critics, self.n_quantiles = n_critics, n_quantiles

    def forward(self, obs, act):
        """-> quantiles [B, n_critics, n_quantiles]."""
        h = torch.cat([obs, act], dim=1).unsqueeze(0).expand(self.n_critics, -1, -1)
        last = len(self.weights) - 1
        for k, (w, b) in enumerate(zip(self.weights, self.biases)):
            h = torch.baddbmm(b, h, w)
            if k < last:
                h = F.relu(h)
        return h.transpose(0, 1)


def quantile_huber_loss(current, target, sum_over_quantiles=False):
    """sb3-contrib common/utils.py quantile_huber_loss: current [B, n_critics, n_q], target
    [B, 1, n_target]."""
    n_q = current.shape[-1]
    cum_prob = (torch.arange(n_q, device=current.device, dtype=torch.float32) + 0.5) / n_q
    cum_prob = cum_prob.view(1, 1, -1, 1)
    delta = target.unsqueeze(-2) - current.unsqueeze(-1)       # [B, n_critics, n_q, n_target]
    ad = delta.abs()
    huber = torch.where(ad > 1, ad - 0.5, delta * delta * 0.5)
    loss = (cum_prob - (delta.detach() < 0).float()).abs() * huber
    return loss.sum(dim=-2).mean() if sum_over_quantiles else loss.mean()


# ----------------------------------------------------------------------------- the algorithm
class TQC:
    """Truncated Quantile Critics over a batched dict-obs env (``BatchedFrankaShelfPNPEnv`` or
    anything with the same reset() / step() tensors)."""

    def __init__(self, env, config: TQCConfig | None = None, device=None):
        self.env = env
        self.cfg = c = config or TQCConfig()
        self.device = torch.device(device) if device is not None else env.device
        self.n_envs = env.num_envs
        self.act_dim = 7
        dims = {"achieved_goal": 3, "desired_goal": 3, "observation": 19}
        self.obs_dim = sum(dims.values())
        self.rank = dist.get_rank() if _world() > 1 else 0
        torch.manual_seed(c.seed)             # same initial weights on every rank (broadcast below too)
        self.actor = Actor(self.obs_dim, self.act_dim, c.net_arch).to(self.device)
        self.critic = QuantileCritics(self.obs_dim, self.act_dim, c.net_arch, c.n_critics,
                                      c.n_quantiles).to(self.device)
        self.critic_target = QuantileCritics(self.obs_dim, self.act_dim, c.net_arch, c.n_critics,
                                             c.n_quantiles).to(self.device)
        self.log_ent_coef = torch.full((1,), math.log(c.ent_coef_init), device=self.device, requires_grad=True)
        if _world() > 1:
            for p in list(self.actor.parameters()) + list(self.critic.parameters()):
                dist.broadcast(p.data, 0)
        self.critic_target.load_state_dict(self.critic.state_dict())
        self.critic_target.requires_grad_(False)
        self.target_entropy = -float(self.act_dim)
        # fused Adam with the learning rate as a device tensor (the linear schedule writes it in place,
        # so a captured step follows it); capturable: step counts on the device
        cuda = self.device.type == "cuda"
        self._lr = torch.full((), c.learning_rate, dtype=torch.float32, device=self.device) if cuda else c.learning_rate
        kw = dict(lr=self._lr, fused=True, capturable=True) if cuda else dict(lr=c.learning_rate)
        self.actor_opt = torch.optim.Adam(self.actor.parameters(), **kw)
        self.critic_opt = torch.optim.Adam(self.critic.parameters(), **kw)
        self.ent_opt = torch.optim.Adam([self.log_ent_coef], **kw)
        self._graph = None          # the captured gradient step (TQC._capture)
        self._graph_out = None
        self._fdesc = None          # pnp_tqc_desc of the fused step (TQC._fused_desc)
        self._frb = None            # pnp_tqc_replay of the fused sample (TQC._fused_replay)
        # device draw counter of pnp_tqc_sample_draw (cfg.device_rng), allocated here so that a
        # checkpoint's `fused_rng_draws` restores it before the first fused step of a resumed run
        self._fctr = torch.zeros(2, dtype=torch.int64, device=self.device) if cuda else None
        self._eager_updates = 0     # steps run eagerly before the capture (allocator / optimiser state)
        self.vecnorm = VecNormalize(dims, self.device, c.clip_obs, c.norm_eps)
        self.buffer = DictReplayBuffer(c.buffer_size, self.n_envs, self.obs_dim, self.act_dim, self.device)
        # per-rank sampling streams (exploration, replay indices); identical init weights
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(c.seed * 1000003 + self.rank + 1)
        self.num_timesteps = 0          # this rank's env transitions (sb3: num_envs per step)
        self.n_updates = 0
        self.total_timesteps = 1
        self._last_raw = None
        self._last_norm = None
        self.ep_reward = torch.zeros(self.n_envs, device=self.device)
        self.stats = {"episodes": 0, "ep_reward_sum": 0.0, "success_sum": 0.0}
        self.logs = {}

    # ------------------------------------------------------------------ schedule / optimisers
    def _progress_remaining(self):
        return 1.0 - float(self.num_timesteps) / float(self.total_timesteps)

    def _update_lr(self):
        lr = self.cfg.learning_rate * self._progress_remaining()
        if isinstance(self._lr, torch.Tensor):
            self._lr.fill_(lr)      # shared by the three optimisers' param groups
        else:
            for opt in (self.actor_opt, self.critic_opt, self.ent_opt):
                for g in opt.param_groups:
                    g["lr"] = lr
        return lr

    @staticmethod
    def _allreduce_grads(params):
        """Average gradients over ranks: one flattened bucket, one all-reduce."""
        ps = [p for p in params if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        dist.all_reduce(flat)
        flat /= dist.get_world_size()
        o = 0
        for p in ps:
            n = p.numel()
            p.grad.copy_(flat[o:o + n].view_as(p.grad))
            o += n

    def _step_opt(self, opt, loss, params, record=None):
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if _world() > 1:
            self._allreduce_grads(params)
        if record is not None:   # (tests: the gradients the step applies)
            record.extend(p.grad.detach().clone() for p in params)
        opt.step()

    # ------------------------------------------------------------------ rollout
    def _norm(self, raw):
        return flat_obs(self.vecnorm.normalize(raw))

    def reset(self):
        obs = self.env.reset()
        raw = {k: obs[k].clone() for k in OBS_KEYS}
        self.vecnorm.update(raw)
        self._last_raw = raw
        self._last_norm = self._norm(raw)

    @torch.no_grad()
    def predict(self, obs_norm, deterministic=False):
        return self.actor(obs_norm, deterministic=deterministic, generator=self.gen)

    @torch.no_grad()
    def collect_step(self):
        """One vector step of every env (sb3 collect_rollouts with train_freq = 1 step)."""
        if self.num_timesteps < self.cfg.learning_starts:
            act = torch.rand(self.n_envs, self.act_dim, device=self.device, generator=self.gen) * 2 - 1
        else:
            act = self.predict(self._last_norm)
        obs, reward, term, trunc, info = self.env.step(act)
        done = term | trunc
        new_raw = {k: obs[k] for k in OBS_KEYS}
        next_raw = dict(new_raw)
        if "final_observation" in info:      # terminal observation of the ended envs
            fin = {"observation": info["final_observation"], "achieved_goal": info["final_achieved_goal"],
                   "desired_goal": info["final_desired_goal"]}
            next_raw = {k: torch.where(done[:, None], fin[k], new_raw[k]) for k in OBS_KEYS}
        self.buffer.add(flat_obs(self._last_raw), flat_obs(next_raw), act, reward, term.float())
        self.vecnorm.update(new_raw)
        self._last_raw = {k: v.clone() for k, v in new_raw.items()}
        self._last_norm = self._norm(self._last_raw)
        self.num_timesteps += self.n_envs
        self.ep_reward += reward
        nd = int(done.sum())
        if nd:
            self.stats["episodes"] += nd
            self.stats["ep_reward_sum"] += float(self.ep_reward[done].sum())
            self.stats["success_sum"] += float(info["is_success"][done].sum())
            self.ep_reward[done] = 0
        return reward, done, info

    # ------------------------------------------------------------------ gradient steps
    def _sample_norm(self):
        o, a, no, d, r = self.buffer.sample(self.cfg.batch_size, self.gen)
        def norm(x):
            parts = torch.split(x, [3, 3, 19], dim=1)
            return flat_obs(self.vecnorm.normalize(dict(zip(OBS_KEYS, parts))))
        return norm(o), a, norm(no), d, r

    def _update(self):
        """One gradient step (sb3-contrib tqc.py train() order) on device tensors, no host sync:
        entropy coefficient, critics, actor, Polyak target update.  Returns the logged values as
        device scalars.  The fused HIP step when it applies (_fused_ok), else PyTorch."""
        if self._fused_ok() and self._fused_state_ready():
            return self._update_fused()
        return self._update_torch()

    def _update_torch(self, record=None):
        """The PyTorch gradient step.  record (tests): a dict that receives the applied gradients,
        'actor' and 'critic', in _fused_params order."""
        c = self.cfg
        rc = ra = None
        if record is not None:
            rc, ra = record.setdefault("critic", []), record.setdefault("actor", [])
        obs, act, nobs, done, rew = self._sample_norm()
        a_pi, lp = self.actor.action_log_prob(obs, self.gen)
        lp = lp.reshape(-1, 1)
        ent_coef = torch.exp(self.log_ent_coef.detach())
        ent_loss = -(self.log_ent_coef * (lp + self.target_entropy).detach()).mean()
        self._step_opt(self.ent_opt, ent_loss, [self.log_ent_coef])
        with torch.no_grad():
            na, nlp = self.actor.action_log_prob(nobs, self.gen)
            nq = self.critic_target(nobs, na)
            keep = c.n_quantiles * c.n_critics - c.top_quantiles_to_drop_per_net * c.n_critics
            nq, _ = torch.sort(nq.reshape(c.batch_size, -1))
            nq = nq[:, :keep]
            tq = nq - ent_coef * nlp.reshape(-1, 1)
            tq = rew + (1 - done) * c.gamma * tq
            tq = tq.unsqueeze(1)
        cq = self.critic(obs, act)
        critic_loss = quantile_huber_loss(cq, tq, sum_over_quantiles=False)
        self._step_opt(self.critic_opt, critic_loss, list(self.critic.parameters()), rc)
        qpi = self.critic(obs, a_pi).mean(dim=2).mean(dim=1, keepdim=True)
        actor_loss = (ent_coef * lp - qpi).mean()
        self._step_opt(self.actor_opt, actor_loss, list(self.actor.parameters()), ra)
        if (self.n_updates + 1) % c.target_update_interval == 0:
            with torch.no_grad():
                tps, ps = list(self.critic_target.parameters()), list(self.critic.parameters())
                torch._foreach_mul_(tps, 1 - c.tau)
                torch._foreach_add_(tps, ps, alpha=c.tau)
        self.n_updates += 1
        return ent_coef, critic_loss.detach(), actor_loss.detach(), ent_loss.detach()

    # ------------------------------------------------------------------ the fused gradient step
    def _fused_ok(self):
        c = self.cfg
        return (c.fused and self.device.type == "cuda" and tuple(c.net_arch) == (256, 256, 256)
                and c.n_critics == 2 and c.n_quantiles == 25 and c.top_quantiles_to_drop_per_net == 2
                and c.batch_size % 16 == 0 and self.obs_dim == 25 and self.act_dim == 7
                and c.target_update_interval == 1)

    def _fused_params(self):
        a = self.actor
        pa = [a.latent[0].weight, a.latent[0].bias, a.latent[2].weight, a.latent[2].bias, a.latent[4].weight,
              a.latent[4].bias, a.mu.weight, a.mu.bias, a.log_std.weight, a.log_std.bias]
        pc = [t for pair in zip(self.critic.weights, self.critic.biases) for t in pair]
        pt = [t for pair in zip(self.critic_target.weights, self.critic_target.biases) for t in pair]
        return pa, pc, pt

    def _fused_state_ready(self):
        pa, pc, _ = self._fused_params()
        return (all(p in self.actor_opt.state and "exp_avg" in self.actor_opt.state[p] for p in pa)
                and all(p in self.critic_opt.state and "exp_avg" in self.critic_opt.state[p] for p in pc)
                and self.log_ent_coef in self.ent_opt.state)

    def _fused_desc(self):
        """pnp_tqc_desc over the live parameter, target and Adam-state tensors (built once they all
        exist; rebuilt after load_state_dict, which replaces the optimiser state)."""
        if self._fdesc is not None:
            return self._fdesc
        from . import _lib
        L = _lib.load()
        c = self.cfg
        pa, pc, pt = self._fused_params()
        d = _lib.PnpTqcDesc()
        d.batch, d.obs_dim, d.act_dim, d.hidden = c.batch_size, self.obs_dim, self.act_dim, c.net_arch[0]
        d.n_critics, d.n_quantiles, d.n_drop_per_net = c.n_critics, c.n_quantiles, c.top_quantiles_to_drop_per_net
        d.gamma, d.tau, d.target_entropy = c.gamma, c.tau, self.target_entropy
        b1, b2 = self.actor_opt.defaults["betas"]
        d.beta1, d.beta2, d.adam_eps = b1, b2, self.actor_opt.defaults["eps"]
        keep = []
        for name, opt, ps in (("actor", self.actor_opt, pa), ("critic", self.critic_opt, pc)):
            for i, p in enumerate(ps):
                st = opt.state[p]
                for suffix, t in (("", p), ("_m", st["exp_avg"]), ("_v", st["exp_avg_sq"]), ("_step", st["step"])):
                    assert t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device, (name, suffix)
                    getattr(d, name + suffix)[i] = t.data_ptr()
                    keep.append(t)
        for i, t in enumerate(pt):
            d.target[i] = t.data_ptr()
        es = self.ent_opt.state[self.log_ent_coef]
        d.log_ent_coef, d.ent_m, d.ent_v, d.ent_step = (self.log_ent_coef.data_ptr(), es["exp_avg"].data_ptr(),
                                                          es["exp_avg_sq"].data_ptr(), es["step"].data_ptr())
        d.lr = self._lr.data_ptr()
        n = L.pnp_tqc_workspace_floats(C.byref(d))
        if n < 0:
            _lib.check(int(n), "pnp_tqc_workspace_floats")
        self._fws = torch.empty(int(n), dtype=torch.float32, device=self.device)
        self._flogs = torch.zeros(4, dtype=torch.float32, device=self.device)
        d.workspace, d.workspace_floats, d.logs = self._fws.data_ptr(), int(n), self._flogs.data_ptr()
        if self._fctr is None:
            self._fctr = torch.zeros(2, dtype=torch.int64, device=self.device)
        d.draw_counter = self._fctr.data_ptr()   # pnp_tqc_sample_draw's draw index, advanced per step
        self._fkeep = keep + list(pt) + [es["exp_avg"], es["exp_avg_sq"], es["step"]]
        self._fdesc = d
        return d

    def _fused_replay(self):
        """pnp_tqc_replay over the replay buffer's and the normaliser's device tensors (fixed
        addresses: the buffer is written in place, VecNormalize updates its statistics in place),
        and the sampled batch's buffers."""
        if self._frb is not None:
            return self._frb
        from . import _lib
        rb, vn, B = self.buffer, self.vecnorm, self.cfg.batch_size
        r = _lib.PnpTqcReplay()
        r.obs, r.next_obs, r.actions, r.rewards, r.dones, r.upper = (
            t.data_ptr() for t in (rb.obs, rb.next_obs, rb.actions, rb.rewards, rb.dones, rb.upper))
        r.rows, r.n_envs, r.obs_dim, r.act_dim, r.n_keys = rb.size, rb.n_envs, self.obs_dim, self.act_dim, len(OBS_KEYS)
        for k, key in enumerate(OBS_KEYS):
            rms = vn.obs_rms[key]
            r.key_dim[k], r.mean[k], r.var[k] = rms.mean.numel(), rms.mean.data_ptr(), rms.var.data_ptr()
        r.clip_obs, r.norm_eps = vn.clip_obs, vn.epsilon
        z = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)
        self._fsb = (z(B, self.obs_dim), z(B, self.act_dim), z(B, self.obs_dim), z(B, 1), z(B, 1))
        # device draws (cfg.device_rng): the uniform and Gaussian draws' buffers, the draw counter
        # (kept across load_state_dict: `fused_rng_draws` restores it) and the Philox key
        self._fu_dev, self._feps = z(2, B), (z(B, self.act_dim), z(B, self.act_dim))
        if self._fctr is None:
            self._fctr = torch.zeros(2, dtype=torch.int64, device=self.device)
        # per-rank key (each rank samples its own replay buffer with its own noise, as the
        # generator's per-rank seed does for the PyTorch step)
        self._fseed = ((int(self.cfg.seed) * 1000003 + self.rank) * 0x9E3779B97F4A7C15
                       + 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF
        self._frb = r
        return r

    def _sample_fused(self):
        """_sample_norm in one launch (pnp_tqc_sample): the same U[0, 1) draw, the same batch bit
        for bit (tests/test_tqc_gpu.py)."""
        from . import _lib
        L = _lib.load()
        r = self._fused_replay()
        B = self.cfg.batch_size
        out = self._fsb
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if self.cfg.device_rng:
            _lib.check(L.pnp_tqc_sample_draw(C.byref(r), self._fseed, self._fctr.data_ptr(), B, self._fu_dev.data_ptr(),
                                             self._feps[0].data_ptr(), self._feps[1].data_ptr(),
                                             *[t.data_ptr() for t in out], stream), "pnp_tqc_sample_draw")
            return out
        u = torch.rand(2, B, device=self.device, generator=self.gen)
        _lib.check(L.pnp_tqc_sample(C.byref(r), u.data_ptr(), B, *[t.data_ptr() for t in out], stream), "pnp_tqc_sample")
        self._fu = u   # alive until the launch has read it
        return out

    def _update_fused(self, grads_out=None):
        """One gradient step by pnp_tqc_sample + pnp_tqc_update (csrc/tqc_fused.hip): the same
        replay sample and the same two N(0, 1) draws as _update (sb3's order), then the whole step
        -- entropy coefficient, critics, Polyak, actor.  grads_out (tests): the step's gradients,
        actor then critics."""
        from . import _lib
        L = _lib.load()
        d = self._fused_desc()
        c = self.cfg
        obs, act, nobs, done, rew = self._sample_fused()
        B = c.batch_size
        if self.cfg.device_rng:   # drawn by pnp_tqc_sample_draw with the batch
            eps_pi, eps_next = self._feps
        else:
            eps_pi = torch.randn(B, self.act_dim, device=self.device, generator=self.gen)
            eps_next = torch.randn(B, self.act_dim, device=self.device, generator=self.gen)
        ts = [t.contiguous() for t in (obs, act, nobs, done, rew, eps_pi, eps_next)]
        b = _lib.PnpTqcBatch(*[t.data_ptr() for t in ts])
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if _world() > 1:
            self._update_fused_dp(L, d, b, stream, grads_out)
        else:
            gp = None if grads_out is None else C.c_void_p(grads_out.data_ptr())
            _lib.check(L.pnp_tqc_update(C.byref(d), C.byref(b), gp, stream), "pnp_tqc_update")
        self._fbatch = ts   # (alive until the launch has read them; in a capture, the graph's pool)
        self.n_updates += 1
        lg = self._flogs
        if torch.cuda.is_current_stream_capturing():
            return lg[0], lg[1], lg[2], lg[3]   # the graph's static outputs (train() clones them)
        # eager: the next step overwrites _flogs in place, so a caller keeping these gets copies
        lg = lg.clone()
        return lg[0], lg[1], lg[2], lg[3]

    def _update_fused_dp(self, L, d, b, stream, grads_out=None):
        """The fused step on several ranks (pnp_tqc_update_phase): critic gradients (and the
        entropy coefficient's) -> all-reduce -> critics' Adam, the actor against the updated
        critics -> actor gradients -> all-reduce -> actor's Adam.  Two flattened buckets per step
        over RCCL (gloo in the CPU-side tests), averaged like _allreduce_grads; the ranks stay in
        lockstep.  grads_out (tests): the averaged gradients, actor then critics."""
        from . import _lib
        if getattr(self, "_fgrads", None) is None:
            na, nc = C.c_int32(), C.c_int32()
            _lib.check(L.pnp_tqc_param_counts(C.byref(na), C.byref(nc)), "pnp_tqc_param_counts")
            self._fna, self._fnc = na.value, nc.value
            self._fgrads = torch.zeros(self._fna + self._fnc + 1, dtype=torch.float32, device=self.device)
        g, na, w = self._fgrads, self._fna, dist.get_world_size()
        gp = C.c_void_p(g.data_ptr())
        _lib.check(L.pnp_tqc_update_phase(C.byref(d), C.byref(b), gp, 0, stream), "pnp_tqc_update_phase(0)")
        crit = g[na:]
        dist.all_reduce(crit)
        crit.div_(w)
        _lib.check(L.pnp_tqc_update_phase(C.byref(d), C.byref(b), gp, 1, stream), "pnp_tqc_update_phase(1)")
        act = g[:na]
        dist.all_reduce(act)
        act.div_(w)
        _lib.check(L.pnp_tqc_update_phase(C.byref(d), C.byref(b), gp, 2, stream), "pnp_tqc_update_phase(2)")
        if grads_out is not None:
            grads_out.copy_(g[:grads_out.numel()])

    def _graph_ok(self):
        return (self.cfg.graph and _world() == 1 and self.device.type == "cuda"
                and self.cfg.target_update_interval == 1)

    def _capture(self):
        """Capture one gradient step in a HIP graph (torch.cuda.graph): every kernel of the step
        -- replay sampling, the three losses' forward and backward passes, fused Adam, the Polyak
        update -- replayed with one launch instead of ~400 (the eager step is launch-bound: batch
        512, 256-wide layers).  The exploration / replay generator is registered with the graph,
        so each replay draws the numbers the eager step would at that point of the stream.  Called
        after 3 eager steps (autograd / allocator / optimiser state exist); gradients are dropped
        first so the captured backward passes allocate them in the graph's pool, as set_to_none
        does eagerly.  The capture itself runs nothing."""
        for opt in (self.actor_opt, self.critic_opt, self.ent_opt):
            opt.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        g.register_generator_state(self.gen)
        n0 = self.n_updates
        with torch.cuda.graph(g):
            self._graph_out = self._update()
        self.n_updates = n0
        self._graph = g

    def train(self, gradient_steps=None):
        """gradient_steps (default cfg.gradient_steps) gradient steps; with a captured step each
        is one graph replay.  Results are the eager steps' bit for bit (tests/test_tqc_gpu.py).
        Returns (and keeps in self.logs) the last step's losses as 0-d device tensors, not floats
        (sb3's logger gets floats; here `float(v)` where a host value is wanted)."""
        c = self.cfg
        lr = self._update_lr()
        n = gradient_steps or c.gradient_steps
        out = None
        for _ in range(n):
            if not self._graph_ok():
                out = self._update()
                continue
            if self._graph is None and self._eager_updates < 3:
                side = torch.cuda.Stream(device=self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    out = self._update()
                torch.cuda.current_stream(self.device).wait_stream(side)
                self._eager_updates += 1
                continue
            if self._graph is None:
                self._capture()
            self._graph.replay()
            self.n_updates += 1
            out = self._graph_out
        # the logs are device tensors (no host sync per call); on the graph path `out` is the
        # captured graph's static outputs, which the next replay overwrites in place -- cloned, so
        # a caller that keeps a returned dict across train() calls keeps this call's values
        if out is self._graph_out:
            out = tuple(t.clone() for t in out)
        self.logs = {"lr": lr, "ent_coef": out[0], "critic_loss": out[1], "actor_loss": out[2],
                     "ent_coef_loss": out[3]}
        return self.logs

    def learn(self, total_timesteps, callback=None, log_every=0):
        """sb3 learn(): vector env steps, a gradient step after each once past learning_starts.
        total_timesteps counts this rank's transitions (n_envs per step)."""
        self.total_timesteps = int(total_timesteps)
        if self._last_raw is None:
            self.reset()
        t0 = time.perf_counter()
        it = 0
        while self.num_timesteps < self.total_timesteps:
            self.collect_step()
            if self.num_timesteps > self.cfg.learning_starts and it % self.cfg.train_freq == 0:
                self.train()
            it += 1
            if callback is not None and callback(self) is False:
                break
            if log_every and it % log_every == 0 and self.rank == 0:
                s = self.stats
                n = max(s["episodes"], 1)
                print(f"steps {self.num_timesteps * _world()}  {self.num_timesteps * _world() / (time.perf_counter() - t0):.0f} "
                      f"transitions/s  episodes {s['episodes']}  ep_rew {s['ep_reward_sum'] / n:.2f}  "
                      f"success {s['success_sum'] / n:.3f}  {({k: float(v) for k, v in self.logs.items()})}", flush=True)
        return self

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self):
        return {"actor": self.actor.state_dict(), "critic": self.critic.state_dict(),
                "critic_target": self.critic_target.state_dict(), "log_ent_coef": self.log_ent_coef.detach(),
                "actor_opt": self.actor_opt.state_dict(), "critic_opt": self.critic_opt.state_dict(),
                "ent_opt": self.ent_opt.state_dict(), "vecnormalize": self.vecnorm.state_dict(),
                "num_timesteps": self.num_timesteps, "n_updates": self.n_updates,
                "fused_rng_draws": int(self._fctr[0]) if getattr(self, "_fctr", None) is not None else 0}

    def load_state_dict(self, d):
        self.actor.load_state_dict(d["actor"])
        self.critic.load_state_dict(d["critic"])
        self.critic_target.load_state_dict(d["critic_target"])
        with torch.no_grad():
            self.log_ent_coef.copy_(d["log_ent_coef"])
        self.actor_opt.load_state_dict(d["actor_opt"])
        self.critic_opt.load_state_dict(d["critic_opt"])
        self.ent_opt.load_state_dict(d["ent_opt"])
        self.vecnorm.load_state_dict(d["vecnormalize"])
        self.num_timesteps, self.n_updates = int(d["num_timesteps"]), int(d["n_updates"])
        if getattr(self, "_fctr", None) is not None:
            self._fctr.zero_()
            self._fctr[0] = int(d.get("fused_rng_draws", 0))
        # the optimisers now hold new state tensors: the schedule's shared lr tensor back in their
        # groups, and a captured step (which read the old ones) is re-captured
        if isinstance(self._lr, torch.Tensor):
            for opt in (self.actor_opt, self.critic_opt, self.ent_opt):
                for g in opt.param_groups:
                    g["lr"] = self._lr
        self._graph, self._graph_out, self._eager_updates = None, None, 0
        self._fdesc = None

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, eval_env, n_episodes=10, max_steps=None):
        """EvalCallback (deterministic, the training env's obs statistics, not updated): the first
        episode of each of ``n_episodes`` envs; returns (mean reward, success rate)."""
        n = eval_env.num_envs
        if n < n_episodes:
            raise ValueError("eval_env needs at least n_episodes envs")
        obs = eval_env.reset()
        ret = torch.zeros(n, device=self.device)
        live = torch.ones(n, dtype=torch.bool, device=self.device)
        succ = torch.zeros(n, device=self.device)
        steps = 0
        while bool(live[:n_episodes].any()):
            a = self.actor(self._norm({k: obs[k] for k in OBS_KEYS}), deterministic=True)
            obs, r, term, trunc, info = eval_env.step(a)
            ret += r * live
            done = (term | trunc) & live
            succ[done] = info["is_success"][done]
            live &= ~done
            steps += 1
            if max_steps and steps >= max_steps:
                break
        return float(ret[:n_episodes].mean()), float(succ[:n_episodes].mean())
