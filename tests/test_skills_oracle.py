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


def test_batched_planner_fallbacks_match_sequential():
    """BatchedMoveIKPlanner's lockstep state machine == plan_ik_waypoints per env, driven by a
    scripted solver with a wall at x = 0.05 (targets beyond it exhaust retries and fallbacks)."""
    from pnp_amd.ik_solver import IKResult
    from pnp_amd.skills import plan_ik_waypoints
    from pnp_amd.skills.batched import BatchedMoveIKPlanner

    def fake(goal, q):
        ok = goal[0] <= 0.05
        return np.asarray(q) + 0.001 * goal.sum(), np.asarray(goal, float), 0.0 if ok else 1.0, ok

    class Seq:
        def solve(self, goal, q):
            qn, fp, err, ok = fake(np.asarray(goal), q)
            return IKResult(bool(ok), qn, fp, err, 10, bool(ok))

    def batch(goals, qs):
        r = [fake(g, q) for g, q in zip(goals, qs)]
        return (np.array([x[0] for x in r]), np.array([x[1] for x in r]), np.array([x[2] for x in r]),
                np.array([x[3] for x in r]))

    rng = np.random.default_rng(3)
    B = 10
    start = np.zeros((B, 3))
    tgt = np.concatenate([rng.uniform(-0.04, 0.04, size=(5, 3)),                 # reachable
                          [[0.2, 0, 0], [0.2, 0.1, 0], [0.3, -0.2, 0.1], [0.06, 0.0, 0.0], [0.1, 0.3, -0.2]]])
    quat = np.tile([1.0, 0, 0, 0], (B, 1))
    q0 = np.zeros((B, 7))
    logs = [[] for _ in range(B)]
    planner = BatchedMoveIKPlanner(solve_fn=batch)
    got = planner.plan(start, quat, q0, tgt, logs=logs)
    for b in range(B):
        lb = []
        pos, qt = plan_ik_waypoints(Seq(), start[b], quat[b], q0[b], tgt[b], log=lb.append)
        assert len(got[b][0]) == len(pos), b
        np.testing.assert_array_equal(np.array(got[b][0]), np.array(pos))
        assert logs[b] == lb, (b, logs[b], lb)
    assert sum(bool(lg) for lg in logs) >= 4
