"""GPU parity of the fused gym env (libpnp.so pnp_env_init / pnp_env_reset / pnp_env_step through
the C ABI, via pnp_amd.envs) against the CPU env oracle (oracle/env_oracle.py: the reference's
FrankaEnv logic over the fp64 physics oracle).

The scene is chaotic over a full gym step: the fp64 oracle itself turns a 1e-12 velocity
perturbation into 1e-4 .. 4e-3 within 200-250 sub-steps (tests/test_env_oracle.py pins this), so
no two implementations — MuJoCo included — agree to 1e-8 over 250 sub-steps.  The env logic
(_set_action, _get_obs, reward, success, task sequencing, TimeLimit, reset draws) is therefore
checked exactly on a short-physics configuration (n_calls = 2 x n_substeps = 2 sub-steps per gym
step, inside the divergence horizon), and the full configuration with bounds:
  * short physics, fp64: observation / state within 1e-9, rewards within 1e-9, flags identical;
  * short physics, fp32: observation within 1e-4, rewards within 1e-4, flags identical;
  * full 250 sub-steps, one gym step from the same state: observation within 5e-3, flags identical.
"""
import os
import numpy as np
import pytest
import torch

import physics_states as PS
from oracle.env_oracle import EnvConfig as OCfg, EnvOracle

pytestmark = pytest.mark.gpu

B = 4


def _env(dtype, B=B, **cfg):
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    return BatchedFrankaShelfPNPEnv(B, dtype=dtype, autoreset=False, config=EnvConfig(**cfg))


def _actions(n, seed):
    return np.random.default_rng(seed).uniform(-1, 1, size=(n, 7)).astype(np.float32).astype(np.float64)


SHORT = dict(n_substeps=2, n_calls=2)


@pytest.fixture(scope="module")
def pair64(model):
    return _env(torch.float64), EnvOracle(B, model=model)


@pytest.fixture(scope="module")
def short64(model):
    return _env(torch.float64, **SHORT), EnvOracle(B, cfg=OCfg(**SHORT), model=model)


def test_init_matches_oracle(pair64):
    g, o = pair64
    np.testing.assert_allclose(g.state["qpos"].cpu().numpy(), o.st["qpos"], atol=1e-9)
    np.testing.assert_allclose(g.env["qpos_kin"].cpu().numpy(), o.qpos_kin, atol=1e-9)
    np.testing.assert_allclose(g.env["obj_height0"].cpu().numpy(), o.obj_height0, atol=1e-9)
    np.testing.assert_allclose(g.env["init_qvel"].cpu().numpy(), o.init_qvel, atol=1e-8)
    np.testing.assert_allclose(g.env["init_mocap"].cpu().numpy(), o.init_mocap, atol=1e-12)
    np.testing.assert_allclose(g.env["goal"].cpu().numpy(), o.goal, atol=1e-12)
    assert np.allclose(g.env["init_time"].cpu().numpy(), 0.5)
    # the dummy object rests on the floor: initial_object_height ~ its radius (App. B quirk 4)
    assert np.all(np.abs(o.obj_height0 - 0.001) < 5e-4)


def test_reset_matches_oracle_f64(pair64):
    g, o = pair64
    obs = g.reset()
    ref = o.reset()
    for b in range(B):
        np.testing.assert_allclose(obs["observation"][b].cpu().numpy(), ref[b]["observation"], atol=1e-9)
        np.testing.assert_allclose(obs["desired_goal"][b].cpu().numpy(), ref[b]["desired_goal"], atol=1e-12)
    np.testing.assert_allclose(g.state["qpos"].cpu().numpy(), o.st["qpos"], atol=1e-12)   # same Philox draws


def _compare_steps(g, o, nsteps, tol, seed0=10):
    for k in range(nsteps):
        a = _actions(B, seed0 + k)
        obs, r, term, trunc, info = g.step(torch.as_tensor(a, dtype=g.dtype))
        res = o.step(a)
        for b in range(B):
            np.testing.assert_allclose(obs["observation"][b].double().cpu().numpy(), res[b]["obs"]["observation"],
                                       atol=tol)
            np.testing.assert_allclose(obs["desired_goal"][b].double().cpu().numpy(), res[b]["obs"]["desired_goal"],
                                       atol=tol)
            np.testing.assert_allclose(float(r[b]), res[b]["reward"], atol=tol)
            assert float(info["is_success"][b]) == res[b]["is_success"]
            assert bool(term[b]) == res[b]["terminated"] and bool(trunc[b]) == res[b]["truncated"]
        np.testing.assert_allclose(g.state["ctrl"].double().cpu().numpy(), o.st["ctrl"], atol=tol)
        np.testing.assert_allclose(g.state["mocap_pos"].double().cpu().numpy(), o.st["mocap_pos"], atol=tol)
        np.testing.assert_allclose(g.state["mocap_quat"].double().cpu().numpy(), o.st["mocap_quat"], atol=tol)


def test_env_logic_short_physics_f64(short64):
    g, o = short64
    g.reset()
    o.reset()
    _compare_steps(g, o, 5, 1e-9)
    np.testing.assert_allclose(g.state["qpos"].cpu().numpy(), o.st["qpos"], atol=1e-9)
    np.testing.assert_allclose(g.env["qpos_kin"].cpu().numpy(), o.qpos_kin, atol=1e-9)
    assert np.array_equal(g.env["task"].cpu().numpy(), o.task)
    assert np.array_equal(g.env["elapsed"].cpu().numpy(), o.elapsed)


def _sync_oracle(g, o):
    for k in ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time"):
        o.st[k][:] = g.state[k].double().cpu().numpy()
    o.qpos_kin[:] = g.env["qpos_kin"].double().cpu().numpy()
    o.goal[:] = g.env["goal"].double().cpu().numpy()


def test_env_logic_short_physics_f32(model):
    g = _env(torch.float32, **SHORT)
    o = EnvOracle(B, cfg=OCfg(**SHORT), model=model)
    g.reset()
    o.reset()
    _sync_oracle(g, o)
    _compare_steps(g, o, 3, 1e-4)


def test_gym_step_wide_tier_pressed_fingers(model):
    """Gym steps from closed fingers pressed into each other (52-63 contacts: the full tier) and,
    in every other env, the cubes piled on board2 too (76-87: the wide tier finishes those
    sub-steps, env_dev.h), fp32 short physics against the oracle env: observations and rewards
    within 1e-3, flags identical, no truncation warning."""
    g = _env(torch.float32, **SHORT)
    o = EnvOracle(B, cfg=OCfg(**SHORT), model=model)
    g.reset()
    o.reset()
    g.state["qpos"][:, 7:9] = -torch.linspace(0.001, 0.004, B, dtype=torch.float32, device="cuda")[:, None]
    PS.cube_pile(g.state["qpos"], model, slice(None, None, 2))
    _sync_oracle(g, o)
    o.st["warn"][:] = 0
    for k in range(3):
        a = _actions(B, 40 + k)
        a[:, 6] = -1.0                       # keep closing
        obs, r, term, trunc, info = g.step(torch.as_tensor(a, dtype=torch.float32))
        res = o.step(a)
        for b in range(B):
            np.testing.assert_allclose(obs["observation"][b].double().cpu().numpy(), res[b]["obs"]["observation"],
                                       atol=1e-3)
            np.testing.assert_allclose(float(r[b]), res[b]["reward"], atol=1e-3)
            assert float(info["is_success"][b]) == res[b]["is_success"]
    assert int((g.state["warn"] & 0xFFFF).max()) == 0 and not o.st["warn"].any()


def _gym_run(mode, B, nsteps, pressed=False, route="1", tiers=None, **extra_env):
    import os
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    env = {"PNP_GYM_COMPACT": mode, "PNP_GYM_ROUTE": route, **extra_env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        g = BatchedFrankaShelfPNPEnv(B, autoreset=True)
        g.reset()
        if pressed:
            g.state["qpos"][::3, 7:9] = -0.002          # a third of the envs: pads pressed together
            PS.cube_pile(g.state["qpos"], g.engine.model, slice(None, None, 6))   # half of those: cubes piled too (> 64)
        rng = np.random.default_rng(21)
        outs = []
        for k in range(nsteps):
            a = torch.as_tensor(rng.uniform(-1, 1, size=(B, 7)), dtype=torch.float32, device="cuda")
            obs, r, term, trunc, info = g.step(a)
            outs.append((obs["observation"].clone(), r.clone(), term.clone(), trunc.clone(), info["is_success"].clone()))
            if tiers is not None:
                tiers.append(g.env["tier"].clone())
        torch.cuda.synchronize()
        return g, outs
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_gym_compact_tier_is_exact():
    """The fp32 gym step starts in the compact tier (8 envs per CU) and hands envs over to the full
    and wide tiers (env_compact.hip, env_dev.h): bit-identical to starting in the full tier, on a
    batch whose envs stay under 20 contacts, pass 20 (random grippers), pass 48 (pads pressed)
    and pass 64 (pads pressed, cubes piled)."""
    a, oa = _gym_run("1", 96, 3, pressed=True)
    b, ob = _gym_run("0", 96, 3, pressed=True)
    for x, y in zip(oa, ob):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
    for k in a.env:
        if k != "tier":   # where the next step starts (a routing hint, not env state)
            assert torch.equal(a.env[k], b.env[k]), k
    w = a.state["warn"].to(torch.int64) & 0xFFFFFFFF
    assert not bool((w >> 16).any()) and int((w & 0xFFFF).max()) == 0


@pytest.mark.parametrize("share", ["0", "50"])
def test_gym_routing_is_exact(share):
    """Routed gym steps (env_dev.h: envs whose last step finished in the full / wide tier start
    there, on side streams concurrent with the compact pass) are bit-identical to every env
    starting in the compact tier; with the routing shares at 0 (a tier any one sub-step needed:
    round 3's rule) the routing engages on a batch with pressed pads, and with the default shares
    (50 %: PNP_GYM_WIDE_PCT / PNP_GYM_FULL_PCT) the results are the same bits."""
    tiers = []
    shares = dict(PNP_GYM_WIDE_PCT=share, PNP_GYM_FULL_PCT=share)
    a, oa = _gym_run("1", 96, 4, pressed=True, route="1", tiers=tiers, **shares)
    b, ob = _gym_run("1", 96, 4, pressed=True, route="0", **shares)
    for x, y in zip(oa, ob):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
    for k in a.env:
        if k != "tier":
            assert torch.equal(a.env[k], b.env[k]), k
    for t in tiers:
        assert int(t.max()) <= 2                        # committed: no pending bits left
    if share == "0":
        assert any(bool((t[::3] > 0).any()) for t in tiers[:-1])   # pressed envs routed past compact
    w = a.state["warn"].to(torch.int64) & 0xFFFFFFFF
    assert not bool((w >> 16).any()) and int((w & 0xFFFF).max()) == 0


@pytest.mark.parametrize("grid", ["2", "224"])
def test_gym_hand_over_queue_is_exact(grid):
    """The hand-over queue (env_dev.h hq_publish / hq_take: the full-tier passes publish the envs
    they hand to the wide tier, a persistent wide consumer grid resumes them concurrently) gives
    the bits of the wide resume pass that starts after the full passes -- with 2 consumer
    workgroups (each waits for and drains many entries) and with the default grid; no env is left
    with resume bits (a consumer that timed out would leave them)."""
    a, oa = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="1", PNP_GYM_QUEUE_CU=grid)
    b, ob = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="0")
    for x, y in zip(oa, ob):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
    for k in a.env:
        assert torch.equal(a.env[k], b.env[k]), k
    w = a.state["warn"].to(torch.int64) & 0xFFFFFFFF
    assert not bool((w >> 16).any()) and int((w & 0xFFFF).max()) == 0


def test_gym_full_order_is_exact():
    """The full tier's resume pass in order of remaining sub-steps (resume_order_kernel, env_dev.h;
    PNP_GYM_FULL_ORDER, default on) against env order: the same bits -- only which workgroup runs
    an env changes, never its arithmetic -- with envs handed over at many sub-steps (pressed pads,
    piled cubes, random actions)."""
    a, oa = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_FULL_ORDER="1")
    b, ob = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_FULL_ORDER="0")
    for x, y in zip(oa, ob):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
    for k in a.env:
        assert torch.equal(a.env[k], b.env[k]), k


def test_gym_queue_timeout_falls_back_exactly():
    """A consumer of the hand-over queue that gives up waiting (here after 1 us:
    PNP_GYM_QUEUE_TIMEOUT_US) leaves its env's resume bits, and the list-based wide resume pass
    after the join finishes it (env_dev.h, PNP_HQ_LATE): the bits of the queue-less step, no env
    left mid-step, and the give-ups counted by pnp_env_queue_status.  With no consumer at all the
    fallback pass finishes every published hand-over, and with the default timeout nothing times
    out and every published hand-over is consumed by the queue."""
    from pnp_amd import _lib
    a, oa = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="1", PNP_GYM_QUEUE_TIMEOUT_US="1")
    st_fast = _lib.env_queue_status()
    # no consumer at all (PNP_GYM_QUEUE_MIN=0, PNP_GYM_QUEUE_PCT=0): the fallback pass finishes every
    # published hand-over
    d, od = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="1", PNP_GYM_QUEUE_MIN="0",
                     PNP_GYM_QUEUE_PCT="0")
    st_none = _lib.env_queue_status()
    b, ob = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="0")
    c, oc = _gym_run("1", 96, 3, pressed=True, route="1", PNP_GYM_QUEUE="1")
    st_def = _lib.env_queue_status()
    print("queue status, 1 us timeout:", st_fast, " no consumer:", st_none, " default:", st_def)
    for x, y, z, q in zip(oa, ob, oc, od):
        for u, v, w, r in zip(x, y, z, q):
            assert torch.equal(u, v) and torch.equal(w, v) and torch.equal(r, v)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]) and torch.equal(c.state[k], b.state[k]), k
        assert torch.equal(d.state[k], b.state[k]), k
    for g in (a, c, d):
        w = g.state["warn"].to(torch.int64) & 0xFFFFFFFF
        assert not bool((w >> 16).any()) and int((w & 0xFFFF).max()) == 0
    assert st_fast["fallback"] <= st_fast["timeouts"] and st_fast["timeouts"] >= 1
    assert st_none["published"] > 0 and st_none["fallback"] == st_none["published"] and st_none["claims"] == 0
    assert st_def["timeouts"] == 0 and st_def["fallback"] == 0
    assert st_def["producers_done"] == 2 * 96 and st_def["claims"] >= st_def["published"]


def test_two_routed_gym_steps_in_flight_on_two_streams():
    """Two batches' routed fp32 gym steps issued on two streams with no host sync between them
    share the device's selection lists and hand-over queue; the second waits (on the GPU) for the
    first (env_dev.h RouteStreams::last).  Each batch's results equal its steps run alone."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv

    def make(off, B):
        g = BatchedFrankaShelfPNPEnv(B, autoreset=True, env_offset=off)
        g.reset()
        g.state["qpos"][::3, 7:9] = -0.002
        return g
    Ba, Bb = 96, 64
    rng = np.random.default_rng(5)
    acts = [(torch.as_tensor(rng.uniform(-1, 1, size=(Ba, 7)), dtype=torch.float32, device="cuda"),
             torch.as_tensor(rng.uniform(-1, 1, size=(Bb, 7)), dtype=torch.float32, device="cuda")) for _ in range(3)]
    # serial
    ga, gb = make(0, Ba), make(1000, Bb)
    ser = []
    for x, y in acts:
        oa = ga.step(x)[0]["observation"].clone()
        torch.cuda.synchronize()
        ob = gb.step(y)[0]["observation"].clone()
        torch.cuda.synchronize()
        ser.append((oa, ob))
    # in flight on two streams
    ha, hb = make(0, Ba), make(1000, Bb)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    par = []
    for x, y in acts:
        with torch.cuda.stream(s1):
            oa = ha.step(x)[0]["observation"].clone()
        with torch.cuda.stream(s2):
            ob = hb.step(y)[0]["observation"].clone()
        par.append((oa, ob))
    torch.cuda.synchronize()
    for (u, v), (p, q) in zip(ser, par):
        assert torch.equal(u, p) and torch.equal(v, q)
    for k in ga.state:
        assert torch.equal(ga.state[k], ha.state[k]) and torch.equal(gb.state[k], hb.state[k]), k


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_full_gym_step_bounded(model, dtype):
    g = _env(dtype)
    o = EnvOracle(B, model=model)
    g.reset()
    o.reset()
    _sync_oracle(g, o)
    a = _actions(B, 3)
    a[:, 6] = 1.0
    obs, r, term, trunc, info = g.step(torch.as_tensor(a, dtype=dtype))
    res = o.step(a)
    for b in range(B):
        np.testing.assert_allclose(obs["observation"][b].double().cpu().numpy(), res[b]["obs"]["observation"], atol=5e-3)
        np.testing.assert_allclose(float(r[b]), res[b]["reward"], atol=5e-3)
        assert bool(term[b]) == res[b]["terminated"]


def _place_cube(g, o, k):
    """Put task object k exactly on its target site (placed = True at the next step's obs)."""
    m = o.m
    a = o.obj_qadr[k]
    tgt = o.goal[0].copy()
    for st_q in (o.st["qpos"],):
        st_q[:, a:a + 3] = tgt
        st_q[:, a + 3:a + 7] = [1, 0, 0, 0]
    g.state["qpos"].copy_(torch.as_tensor(o.st["qpos"], dtype=g.dtype))
    return m


def test_task_sequencing_and_termination(model):
    g = _env(torch.float64, B=2, **SHORT)
    o = EnvOracle(2, cfg=OCfg(**SHORT), model=model)
    g.reset()
    o.reset()
    seen = []
    for k in range(3):
        g.env["task"].fill_(k)
        o.task[:] = k
        sx, _, _, _ = o._frames(0, o.ee)
        o.goal[:] = sx[o.target_site[k]]
        g.env["goal"].copy_(torch.as_tensor(o.goal, dtype=g.dtype))
        _place_cube(g, o, k)
        a = np.zeros((2, 7))
        obs, r, term, trunc, info = g.step(torch.as_tensor(a, dtype=torch.float64))
        res = o.step(a)
        seen.append((float(info["is_success"][0]), bool(term[0]), int(g.env["task"][0])))
        for b in range(2):
            assert float(info["is_success"][b]) == res[b]["is_success"]
            assert bool(term[b]) == res[b]["terminated"]
            np.testing.assert_allclose(float(r[b]), res[b]["reward"], atol=1e-8)
            np.testing.assert_allclose(g.env["goal"][b].cpu().numpy(), o.goal[b], atol=1e-12)
            assert int(g.env["task"][b]) == int(o.task[b])
    # a cube dropped on its target is placed: success, task index advances, last one terminates
    assert [s[0] for s in seen] == [1.0, 1.0, 1.0]
    assert [s[1] for s in seen] == [False, False, True]
    assert [s[2] for s in seen] == [1, 2, 3]


def test_truncation_autoreset_and_mask(model):
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
    g = BatchedFrankaShelfPNPEnv(3, dtype=torch.float32, autoreset=True, config=EnvConfig(max_episode_steps=2))
    first = {k: v.clone() for k, v in g.reset().items()}
    a = torch.zeros(3, 7)
    _, _, _, trunc, _ = g.step(a)
    assert not trunc.any()
    obs, _, _, trunc, info = g.step(a)
    assert trunc.all()
    assert "final_observation" in info
    assert torch.equal(g.env["elapsed"], torch.zeros(3, dtype=torch.int32, device=g.device))
    assert torch.equal(g.env["episode"].cpu(), torch.full((3,), 2, dtype=torch.int32))
    # the new episode's objects are re-drawn around the objects' current positions
    assert not torch.equal(obs["observation"], first["observation"])
    # masked reset touches only the selected env
    before = g.state["qpos"].clone()
    g.reset(torch.tensor([0, 1, 0], dtype=torch.uint8))
    assert torch.equal(g.state["qpos"][0], before[0]) and torch.equal(g.state["qpos"][2], before[2])
    assert not torch.equal(g.state["qpos"][1], before[1])


def test_shard_invariant_resets():
    """Envs [2, 4) of a 4-env batch == a 2-env batch with env_offset 2 (Philox by global index)."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    full = BatchedFrankaShelfPNPEnv(4, dtype=torch.float32, autoreset=False)
    half = BatchedFrankaShelfPNPEnv(2, dtype=torch.float32, autoreset=False, env_offset=2)
    a = full.reset()["observation"].clone()
    b = half.reset()["observation"].clone()
    assert torch.equal(a[2:], b)
    act = torch.as_tensor(_actions(4, 5), dtype=torch.float32, device=full.device)
    oa = full.step(act)[0]["observation"]
    ob = half.step(act[2:])[0]["observation"]
    assert torch.equal(oa[2:], ob)


def test_single_env_facade_envs_test():
    """reference test/envs_test.py equivalent: reset + 20 random steps per id, obs shapes / bounds,
    reset on done, double close; plus reward_test.py:118-126 (static steps -> total < 0)."""
    from pnp_amd.envs import ENV_IDS, make
    for env_id in ENV_IDS:
        env = make(env_id)
        obs, info = env.reset(seed=0)
        assert obs["observation"].shape == (19,) and obs["achieved_goal"].shape == (3,)
        assert np.allclose(env.home_pos, [1.23843967, 0.0, 0.49740014], atol=1e-6)
        total = 0.0
        for _ in range(20):
            obs, r, term, trunc, info = env.step(env.action_space.sample())
            assert np.all(np.isfinite(obs["observation"]))
            assert isinstance(r, np.float32) and "is_success" in info
            if term or trunc:
                env.reset()
        env.reset()
        for _ in range(5):
            _, r, _, _, _ = env.step(np.zeros(7, np.float32))
            total += float(r)
        assert total < 0
        with pytest.raises(ValueError):
            env.step(np.zeros(6))
        env.close()
        env.close()


class _GpuAdapter:
    """pnp_amd.envs B = 1 env behind the golden replay interface (tests/test_env_oracle.py)."""

    def __init__(self, env_index, cfg, dtype):
        from pnp_amd.envs import BatchedFrankaShelfPNPEnv, EnvConfig
        rt = cfg.pop("reward_type")
        self.g = BatchedFrankaShelfPNPEnv(1, reward_type=rt, dtype=dtype, env_offset=env_index, autoreset=False,
                                          config=EnvConfig(**cfg))

    def _np(self, t):
        return t.double().cpu().numpy()

    def init_values(self):
        return float(self.g.env["obj_height0"][0]), self._np(self.g.env["init_mocap"][0])

    def reset(self):
        obs = self.g.reset()
        return self._np(obs["observation"][0]), self._np(self.g.env["goal"][0])

    def place(self):
        g = self.g
        k = min(int(g.env["task"][0]), len(g.task_sequence) - 1)
        a = g.params.obj_qadr[k]
        q = g.state["qpos"]
        q[0, a:a + 3] = g.env["goal"][0]
        q[0, a + 3:a + 7] = torch.tensor([1.0, 0, 0, 0], dtype=q.dtype)
        g.env["qpos_kin"][0] = q[0]

    def step(self, a):
        g = self.g
        obs, r, term, trunc, info = g.step(torch.as_tensor(np.asarray(a)[None], dtype=g.dtype))
        return dict(obs=self._np(obs["observation"][0]), reward=float(r[0]), success=float(info["is_success"][0]),
                    terminated=bool(term[0]), ctrl=self._np(g.state["ctrl"][0]), mocap_pos=self._np(g.state["mocap_pos"][0]),
                    mocap_quat=self._np(g.state["mocap_quat"][0]), task=int(g.env["task"][0]),
                    goal=self._np(g.env["goal"][0]))


def _close(a, b, tol, what):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), atol=tol, rtol=0, err_msg=what)


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-9), (torch.float32, 2e-4)])
def test_gpu_env_matches_reference_env_golden(dtype, tol):
    """The fused env kernel against the reference's own FrankaEnv code (golden fixture)."""
    from test_env_oracle import replay_golden
    replay_golden(lambda idx, cfg: _GpuAdapter(idx, dict(cfg), dtype), _close, tol)


@pytest.mark.timeout(600)
def test_gym_full_size_random_actions():
    """The bench's gym leg at full size -- the workload whose clamped-index build faulted in round
    2 (profiles/r02/ab_branchless_fault.log): 4096 fp32 envs, routed tiers, 4 gym steps of uniform
    random actions (pads pressing, cubes knocked over: every tier and the hand-overs run).  No
    fault, finite state and outputs, no bad-state reset or truncation, no leaked hand-over bits,
    and the routed run equals the unrouted one bit for bit."""
    from pnp_amd.envs import BatchedFrankaShelfPNPEnv
    B = 4096
    acts = torch.as_tensor(np.random.default_rng(7).uniform(-1, 1, size=(4, B, 7)), dtype=torch.float32, device="cuda")
    runs = []
    for route in ("1", "0"):
        old = os.environ.get("PNP_GYM_ROUTE")
        os.environ["PNP_GYM_ROUTE"] = route
        try:
            env = BatchedFrankaShelfPNPEnv(B, autoreset=False)
            env.reset()
            rewards = []
            for i in range(4):
                obs, r, term, trunc, info = env.step(acts[i])
                rewards.append(r)
                assert bool(torch.isfinite(obs["observation"]).all()) and bool(torch.isfinite(r).all())
            torch.cuda.synchronize()
        finally:
            if old is None:
                del os.environ["PNP_GYM_ROUTE"]
            else:
                os.environ["PNP_GYM_ROUTE"] = old
        assert bool(torch.isfinite(env.state["qpos"]).all()) and bool(torch.isfinite(env.state["qvel"]).all())
        w = env.state["warn"].to(torch.int64) & 0xFFFFFFFF
        assert int((w & 0x1F).max()) == 0, "bad-state reset or contact / row truncation"
        assert not bool((w >> 16).any()), "a tier hand-over bit leaked out of the call"
        runs.append((env, torch.stack(rewards)))
    (a, ra), (b, rb) = runs
    assert torch.equal(ra, rb)
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
