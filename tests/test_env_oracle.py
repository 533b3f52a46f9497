"""CPU checks of the env oracle (oracle/env_oracle.py) and of the scene property the GPU env
tests are built around (tests/test_env_gpu.py)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle.env_oracle import (HORIZONTAL_QUAT, VERTICAL_QUAT, EnvConfig, EnvOracle, euler2quat, mat2euler,
                               quat_mul)

HOME_WPT = np.array([1.23843967, 0.0, 0.49740014])   # execute_pnp.py:38, reward_test.py:47


@pytest.fixture(scope="module")
def env(model):
    e = EnvOracle(2, model=model)
    e.reset()
    return e


def test_rotation_helpers():
    assert np.allclose(VERTICAL_QUAT, [1, 0, 0, 0])
    assert np.allclose(HORIZONTAL_QUAT, [np.cos(np.pi / 4), -np.sin(np.pi / 4), 0, 0])
    rng = np.random.default_rng(0)
    for _ in range(20):
        e = rng.uniform([-3, -1.5, -3], [3, 1.5, 3])
        q = euler2quat(e)
        R = np.array([[1 - 2 * (q[2] ** 2 + q[3] ** 2), 2 * (q[1] * q[2] - q[0] * q[3]), 2 * (q[1] * q[3] + q[0] * q[2])],
                      [2 * (q[1] * q[2] + q[0] * q[3]), 1 - 2 * (q[1] ** 2 + q[3] ** 2), 2 * (q[2] * q[3] - q[0] * q[1])],
                      [2 * (q[1] * q[3] - q[0] * q[2]), 2 * (q[2] * q[3] + q[0] * q[1]), 1 - 2 * (q[1] ** 2 + q[2] ** 2)]])
        assert np.allclose(mat2euler(R), e, atol=1e-12)
        assert np.isclose(np.linalg.norm(quat_mul(q, euler2quat(-e))), 1.0)


def test_reset_observation_known_answers(env, model):
    ob = env._observe(0, 0, env.goal[0])
    assert np.allclose(ob["observation"][:3], HOME_WPT, atol=1e-8)      # ee at the home waypoint
    assert np.allclose(env.goal[0], [1.0, -0.1, 0.3])                    # target_cube1 site
    assert env.st["time"][0] == pytest.approx(0.5)                       # initial_time after setup
    # cube1 re-drawn around its site: x within +-0.02, y within +-0.2 of the pre-reset position
    a = env.obj_qadr[0]
    assert abs(env.st["qpos"][0, a + 2] - 0.7299) < 1e-3


def test_static_steps_negative_reward(model):
    """reward_test.py:118-126: standing still gives a negative total (time + reach penalties)."""
    e = EnvOracle(1, model=model)
    e.reset()
    total = sum(e.step(np.zeros((1, 7)))[0]["reward"] for _ in range(3))
    assert -3 * 0.053 - 1e-9 <= total < 0


def test_sparse_reward_values(model):
    e = EnvOracle(1, cfg=EnvConfig(reward_type="sparse", n_substeps=2, n_calls=1), model=model)
    e.reset()
    assert e.step(np.zeros((1, 7)))[0]["reward"] == -1.0
    a = e.obj_qadr[0]
    e.st["qpos"][0, a:a + 3] = e.goal[0]
    r = e.step(np.zeros((1, 7)))[0]
    assert r["reward"] == 0.0 and r["is_success"] == 1.0 and e.task[0] == 1


def test_grip_and_lift_terms(model):
    """gripped (+2 + alignment), lifted (+4) as panda_env.py:214-239 define them."""
    e = EnvOracle(1, cfg=EnvConfig(n_substeps=1, n_calls=1), model=model)
    e.reset()
    a = e.obj_qadr[0]
    ee = e._observe(0, 0, e.goal[0])["ee_pos"]
    e.st["qpos"][0, a:a + 3] = ee + [0, 0, -0.01]              # object in the hand
    e.st["qpos"][0, e.finger_qadr] = 0.02                       # width 0.04 < 0.045
    e.qpos_kin[0] = e.st["qpos"][0]
    r = e.step(np.zeros((1, 7)))[0]
    # d_reach small, gripped and (object high above the floor dummy) lifted: 2 + align + 4
    assert r["reward"] > 2.0 + 4.0 - 0.06


def test_scene_is_chaotic_over_a_gym_step(model):
    """Why the GPU env tests compare whole gym steps with bounds: the oracle amplifies a 1e-12
    velocity perturbation by > 1e5 within 250 sub-steps (measured 1e-4 .. 4e-3)."""
    e = EnvOracle(4, model=model)
    e.reset()
    a = np.random.default_rng(10).uniform(-1, 1, size=(4, 7))
    a[:, 6] = 1.0
    e.step(a)
    A = {k: v.copy() for k, v in e.st.items()}
    Bs = {k: v.copy() for k, v in e.st.items()}
    Bs["qvel"][:, :9] += 1e-12
    O.step(A, nsub=250, nthreads=8, model=model)
    O.step(Bs, nsub=250, nthreads=8, model=model)
    growth = np.abs(A["qvel"] - Bs["qvel"]).max() / 1e-12
    assert growth > 1e5


# ---------------------------------------------------------------- reference golden vectors
import os  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "env_golden.npz")


def replay_golden(make_env, check, tol):
    """Replays tests/golden/env_golden.npz (the reference's own FrankaEnv code, stub-imported,
    see make_env_golden.py) through an env adapter: make_env(env_index, cfg) -> adapter with
    .init_values(), .reset() -> (obs, goal), .place(), .step(action) -> dict."""
    G = np.load(GOLDEN)
    n_sub = int(G["n_substeps"])
    for i in range(len(G["env_index"])):
        cfg = dict(reward_type="dense" if G["reward_dense"][i] else "sparse", n_substeps=n_sub, n_calls=10)
        env = make_env(int(G["env_index"][i]), cfg)
        h0, mocap = env.init_values()
        check(h0, G["obj_height0"][i], tol, "obj_height0")
        check(mocap, G["init_mocap"][i], tol, "init_mocap")
        obs, goal = env.reset()
        check(obs, G["reset_obs"][i], tol, "reset obs")
        check(goal, G["reset_goal"][i], tol, "reset goal")
        for k in range(G["actions"].shape[1]):
            if G["place"][i][k]:
                env.place()
            r = env.step(G["actions"][i][k])
            tag = f"episode {i} step {k}"
            check(r["obs"], G["obs"][i][k], tol, tag + " obs")
            check(r["reward"], G["reward"][i][k], tol, tag + " reward")
            assert r["success"] == G["success"][i][k], tag
            assert r["terminated"] == bool(G["terminated"][i][k]), tag
            check(r["ctrl"], G["ctrl"][i][k], tol, tag + " ctrl")
            check(r["mocap_pos"], G["mocap_pos"][i][k], tol, tag + " mocap_pos")
            check(r["mocap_quat"], G["mocap_quat"][i][k], tol, tag + " mocap_quat")
            assert r["task"] == int(G["task"][i][k]), tag
            check(r["goal"], G["goal"][i][k], tol, tag + " goal")


def _close(a, b, tol, what):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), atol=tol, rtol=0, err_msg=what)


class _OracleAdapter:
    def __init__(self, env_index, cfg, model):
        self.e = EnvOracle(1, cfg=EnvConfig(**cfg), env_index=[env_index], model=model)

    def init_values(self):
        return self.e.obj_height0[0], self.e.init_mocap[0]

    def reset(self):
        r = self.e.reset()[0]
        return r["observation"], self.e.goal[0]

    def place(self):
        e = self.e
        a = e.obj_qadr[min(int(e.task[0]), len(e.obj_qadr) - 1)]
        e.st["qpos"][0, a:a + 7] = np.concatenate([e.goal[0], [1, 0, 0, 0]])
        e.qpos_kin[0] = e.st["qpos"][0]

    def step(self, a):
        e = self.e
        r = e.step(np.asarray(a)[None])[0]
        return dict(obs=r["obs"]["observation"], reward=r["reward"], success=r["is_success"],
                    terminated=r["terminated"], ctrl=e.st["ctrl"][0], mocap_pos=e.st["mocap_pos"][0],
                    mocap_quat=e.st["mocap_quat"][0], task=int(e.task[0]), goal=e.goal[0])


def test_golden_fixture_covers_paths():
    G = np.load(GOLDEN)
    assert G["success"].sum() >= 3 and G["terminated"].sum() >= 1
    assert (~G["reward_dense"]).any() and G["reward_dense"].any()
    assert len(set(G["env_index"].tolist())) >= 3


def test_oracle_matches_reference_env_golden(model):
    replay_golden(lambda idx, cfg: _OracleAdapter(idx, cfg, model), _close, 1e-12)
