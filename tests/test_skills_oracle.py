"""Skills (pnp_amd.skills, reference panda_mujoco_gym/skills) against the reference skills' own
golden episode (tests/golden/make_skill_golden.py), on the CPU: the env under the skills is the
fp64 oracle with the facade's surface, so physics and env logic match the golden's exactly and
the comparison pins the skills' control logic (waypoints, tick counts, done conditions)."""
import numpy as np
import pytest

import skill_harness as H


@pytest.fixture(scope="module")
def golden():
    return H.load_golden()


def test_golden_fixture_shape(golden):
    G = golden
    assert G["ticks"].tolist()[0] >= 20 and G["ticks"].sum() == len(G["action"])
    assert len(G["moveik_traj"]) >= 3
    assert G["done"].sum() == len(G["ticks"])                   # every skill finished
    # the gripper ticks send a finger-only action: a[6] = -1 (close) / +1 (open)
    close0 = G["ticks"][:2].sum()
    assert G["action"][close0][6] == -1.0 and G["action"][-1][6] == 1.0


def test_plan_ik_waypoints_matches_reference(golden, model):
    from pnp_amd.skills import plan_ik_waypoints
    G = golden
    pos, quat = plan_ik_waypoints(H.OracleIK(model), G["moveik_start_ee"], G["moveik_start_quat"],
                                  G["moveik_start_qpos"][:7], G["moveik_target"], log=lambda *_: None)
    np.testing.assert_allclose(np.array(pos), G["moveik_traj"], atol=1e-12, rtol=0)
    np.testing.assert_allclose(np.array(quat), G["moveik_quat_traj"], atol=1e-12, rtol=0)


def test_skills_match_reference_episode(golden, model, monkeypatch):
    import pnp_amd.skills.move as move
    monkeypatch.setattr(move, "JacobianIKController", H.OracleIK)
    env = H.OracleFacadeEnv(model, int(golden["n_substeps"]))
    np.testing.assert_allclose(env.data.qpos, golden["reset_qpos"], atol=1e-12, rtol=0)
    out = H.run_episode(env, golden)
    H.compare(out, golden, 1e-10)


def test_planner_fallbacks(model):
    """An unreachable target drives the planner through its failure path (move.py:136-186):
    plain retries count twice, the fallbacks run after three, and planning stops with the target
    appended as the last waypoint."""
    from pnp_amd.skills import plan_ik_waypoints

    class Failing:
        calls = 0

        def solve(self, target, q):
            Failing.calls += 1
            from pnp_amd.ik_solver import IKResult
            return IKResult(False, np.asarray(q), np.zeros(3), 1.0, 100, False)

    logs = []
    pos, quat = plan_ik_waypoints(Failing(), np.zeros(3), np.array([1.0, 0, 0, 0]), np.zeros(7),
                                  np.array([0.5, 0.2, 0.0]), log=logs.append)
    # solve #1 fails (failures 1 -> 2, retry), #2 fails (3: fallbacks), then fallback 1 and 2 fail
    assert Failing.calls == 4
    assert logs == ["IK failed 3 times, trying fallback strategies...",
                    "All fallback strategies failed, stopping at point 0"]
    assert len(pos) == 2 and np.allclose(pos[-1], [0.5, 0.2, 0.0])


def test_gripper_width_fallback():
    """FrankaEnv has no get_gripper_width: the width predicate always holds (gripper.py:60-71)."""
    from pnp_amd.skills import GripperSkill

    class Env:
        action_space = None

    assert GripperSkill.close(Env())._current_width() == 0.0
    assert GripperSkill.open(Env())._current_width() == np.inf

    class WithWidth:
        def get_gripper_width(self):
            return float("nan")

    assert GripperSkill.close(WithWidth())._current_width() == 0.0
