"""The reference's own behavioural tests, run on this engine's single-env facade.

These are the only checks the reference holds that exercise contact dynamics end to end (a grasp
has to happen for a +6 reward), so they are ported as they are written -- same protocol, same
thresholds -- with gym.make / py_trees replaced by pnp_amd.envs.make / pnp_amd.bt:

  * test/reward_test.py:118-125   static: 10 physics steps from reset, cumulative reward < 0
  * test/reward_test.py:128-136   behaviour-tree PnP episode (250 ticks, close-until-width each
                                  tick, 4 recorded physics steps per tick): some step reward >= 6
                                  (grip + lift) and -300 < total < 2500
  * test/reward_test.py:138-154   80 random gym steps (gripper closed every 4th): some reward < 0
  * test/envs_test.py:10-25       100 random gym steps per registered id, reset on done, close twice

The RewardSampler below restates reward_test.py:56-112 (its reward record is _get_obs +
compute_reward, here pnp_env_evaluate on the device).  reward_test's task builder
(reward_test.py:28-53) equals scripts/execute_pnp.py's (pnp_amd.execute_pnp).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CUBE_EDGE = 0.04                                   # reward_test.py:22-25
GRIPPER_CLEARANCE = 0.004
GRIP_WIDTH_THRESH = CUBE_EDGE + GRIPPER_CLEARANCE


class RewardSampler:
    """reward_test.py:56-112 on the facade."""

    def __init__(self, seed=0):
        from pnp_amd.envs import make
        self.env = make("FrankaShelfPNPDense-v0")
        self.env.action_space.seed(seed)
        self.reset_env()

    def reset_env(self):
        self.env.reset()
        self.env.unwrapped.task_sequence[:] = ["cube1", "cube2", "cube3"]
        self.rewards, self.total = [], 0.0

    def _record_reward(self):
        sim = self.env.unwrapped
        obs = sim._get_obs()
        r = float(sim.compute_reward(obs["achieved_goal"], obs["desired_goal"], {}))
        self.rewards.append(r)
        self.total += r

    def physics_step_and_record(self, n=1):
        sim = self.env.unwrapped
        for _ in range(n):
            sim._mujoco.mj_step(sim.model, sim.data, nstep=1)
            self._record_reward()

    def _close_until_width(self, width_thresh=GRIP_WIDTH_THRESH, max_ctrl_steps=40):
        close_act = np.zeros(self.env.action_space.shape, dtype=np.float32)
        close_act[-1] = -1.0
        for _ in range(max_ctrl_steps):
            self.env.step(close_act)
            self.physics_step_and_record(1)
            if self.env.unwrapped.get_fingers_width() < width_thresh:
                break

    def run_behavior_tree(self, ticks=200, sim_steps=4):
        from pnp_amd.bt import Status, build_pnp_tree
        from pnp_amd.execute_pnp import build_pick_place_tasks
        tasks = [{"obj_meta": t["pick_meta"], "place_meta": t["place_meta"]}
                 for t in build_pick_place_tasks(self.env)]
        tree = build_pnp_tree(self.env, tasks, retry_pick=1)
        root = tree.root
        n = 0
        for _ in range(ticks):
            tree.tick()
            self._close_until_width()
            self.physics_step_and_record(sim_steps)
            n += 1
            if root.status == Status.SUCCESS:
                break
        return n

    def stats(self):
        arr = np.asarray(self.rewards) if self.rewards else np.zeros(1)
        return dict(total=self.total, min=float(arr.min()), max=float(arr.max()), n=len(self.rewards))

    def close(self):
        self.env.close()


def test_static_negative_reward():
    """reward_test.py:118-125."""
    rs = RewardSampler()
    rs.reset_env()
    rs.physics_step_and_record(10)
    st = rs.stats()
    assert st["total"] < 0, f"Static reward should be negative, got {st}"
    rs.close()


@pytest.mark.timeout(900)
def test_episode_positive_spike():
    """reward_test.py:128-136: a grip + lift (+6) happens within 250 behaviour-tree ticks and the
    episode's summed step rewards stay in (-300, 2500)."""
    rs = RewardSampler()
    rs.reset_env()
    ticks = rs.run_behavior_tree(ticks=250, sim_steps=4)
    st = rs.stats()
    print(f"episode: {ticks} ticks, {st['n']} recorded steps, total {st['total']:.2f}, max {st['max']:.3f}")
    assert st["max"] >= 6.0, f"No +6 reward triggered, stats={st}"
    assert -300 < st["total"] < 2500, f"Total reward not in reasonable range, stats={st}"
    rs.close()


def test_reward_has_negative():
    """reward_test.py:138-154."""
    rs = RewardSampler(seed=1)
    rs.reset_env()
    for i in range(80):
        act = rs.env.action_space.sample()
        if i % 4 == 0:
            act[-1] = -1.0
        rs.env.step(act)
        rs._record_reward()
    arr = np.asarray(rs.rewards)
    assert (arr < 0).any(), "Random step should have negative reward"
    assert np.isfinite(arr).all()
    rs.close()


@pytest.mark.parametrize("env_id", ["FrankaShelfPNPSparse-v0", "FrankaShelfPNPDense-v0"])
def test_env(env_id):
    """envs_test.py:10-25: reset + 100 random steps (reset on done), obs within the observation
    space's shapes and finite, close twice."""
    from pnp_amd.envs import ENV_IDS, make
    assert env_id in ENV_IDS
    env = make(env_id)
    env.action_space.seed(3)
    obs, info = env.reset()
    for _ in range(100):
        action = env.action_space.sample()
        obs, r, terminated, truncated, info = env.step(action)
        assert obs["observation"].shape == (19,) and obs["achieved_goal"].shape == (3,)
        assert np.isfinite(obs["observation"]).all() and np.isfinite(r)
        assert isinstance(r, np.float32) and set(info) >= {"is_success"}
        assert env.unwrapped.data.warn & 7 == 0, "bad-state reset during random steps"
        if terminated or truncated:
            env.reset()
    env.close()
    env.close()


def test_get_obs_and_reward_match_step():
    """The facade's _get_obs / compute_reward (pnp_env_evaluate) right after a step reproduce what
    that step returned (same data.site_* semantics, same reward formula; goal before the task
    update), and _is_success agrees."""
    from pnp_amd.envs import make
    env = make("FrankaShelfPNPDense-v0")
    env.reset()
    env.action_space.seed(5)
    for _ in range(3):
        obs, r, term, trunc, info = env.step(env.action_space.sample())
        if info["is_success"]:       # the task index (and goal) moved on after this step
            continue
        o2 = env.unwrapped._get_obs()
        for k in ("observation", "achieved_goal", "desired_goal"):
            np.testing.assert_allclose(o2[k], obs[k], rtol=0, atol=1e-12)
        r2 = env.unwrapped.compute_reward(obs["achieved_goal"], obs["desired_goal"], {})
        assert isinstance(r2, np.float32) and r2 == r
        assert env.unwrapped._is_success(obs["achieved_goal"], obs["desired_goal"]) == info["is_success"]
    # a goal at the cube itself is a success (+10 placed) under the same state
    ag = obs["achieved_goal"]
    assert env.unwrapped._is_success(ag, ag) == 1.0
    assert env.unwrapped.compute_reward(ag, ag, {}) >= r + 10.0 - 1e-5
