"""The facade's MuJoCo-binding surface (pnp_amd/mjshim.py) and the skills on the device.

* mj_step / mj_forward / mj_jacSite / mju_mat2Quat / mujoco_utils accessors against the oracle;
* the reference skills' golden episode (tests/golden/make_skill_golden.py) replayed with
  pnp_amd.skills on the real facade (FrankaShelfPNPEnv, fp64 device physics, the product IK
  kernel inside MoveIKSkill).  Tick counts and done flags must match exactly; trajectories
  within 1e-6 (fp64 device vs fp64 oracle over ~300 sub-steps: measured well below that).
"""
import copy

import numpy as np
import pytest
import torch

import skill_harness as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from pnp_amd.envs import EnvConfig, FrankaShelfPNPEnv
    e = FrankaShelfPNPEnv(config=EnvConfig(n_substeps=1))
    e.reset()
    return e


def _oracle_state(d):
    st = {k: np.array(v, np.float64)[None] for k, v in
          (("qpos", d.qpos), ("qvel", d.qvel), ("ctrl", d.ctrl), ("mocap_pos", d.mocap_pos.reshape(-1)),
           ("mocap_quat", d.mocap_quat.reshape(-1)), ("qacc_warmstart", d.qacc_warmstart))}
    st["time"] = np.array([d.time])
    st["warn"] = np.array([d.warn], np.uint32)
    return st


def test_binding_surface(env):
    u = env.unwrapped
    assert u.model is env.model and u.data is env.data
    for f in ("mj_step", "mj_forward", "mj_kinematics", "mj_jacSite", "mju_mat2Quat", "mj_resetData"):
        assert callable(getattr(u._mujoco, f))
    d2 = copy.deepcopy(env.data)                      # skills/move.py:83-84
    d2.qpos[:7] += 0.1
    assert not np.allclose(d2.qpos[:7], env.data.qpos[:7])


def test_mj_step_matches_oracle(env, model):
    from pnp_amd.mjshim import MjData
    d = copy.deepcopy(env.data)
    d.ctrl[:] = model.actuator_ctrlrange[:, 0] + 0.3 * np.diff(model.actuator_ctrlrange, axis=1)[:, 0]
    ref = _oracle_state(d)
    env._mujoco.mj_step(env.model, d, nstep=7)
    pre = {k: v.copy() for k, v in ref.items()}
    O.step(pre, nsub=6, model=model)
    qk = pre["qpos"][0].copy()
    O.step(pre, nsub=1, model=model)
    assert isinstance(d, MjData)
    np.testing.assert_allclose(d.qpos, pre["qpos"][0], atol=1e-10, rtol=0)
    np.testing.assert_allclose(d.qvel, pre["qvel"][0], atol=1e-8, rtol=0)
    assert d.time == pytest.approx(pre["time"][0], abs=1e-12)
    np.testing.assert_allclose(d.qpos_kin, qk, atol=1e-10, rtol=0)    # site_* = last forward
    sx, sm = O.site_kinematics(qk[None], pre["mocap_pos"], pre["mocap_quat"], model=model)
    np.testing.assert_allclose(d.site_xpos, sx[0], atol=1e-10, rtol=0)
    np.testing.assert_allclose(d.site_xmat, sm[0].reshape(-1, 9), atol=1e-10, rtol=0)


def test_mj_jacsite_and_velocities(env, model):
    d = copy.deepcopy(env.data)
    d.qvel[:] = np.random.default_rng(1).normal(size=model.nv)
    env._mujoco.mj_forward(env.model, d)
    for name in ("ee_center_site", "cube1_site", "cube3_site"):
        sid = model.site_id(name)
        jp, jr = np.zeros((3, model.nv)), np.zeros((3, model.nv))
        env._mujoco.mj_jacSite(env.model, d, jp, jr, sid)
        _, _, rjp, rjr = O.site_jac2(d.qpos[None], name, d.mocap_pos.reshape(1, -1), d.mocap_quat.reshape(1, -1),
                                     model=model)
        np.testing.assert_allclose(jp, rjp[0], atol=1e-12, rtol=0)
        np.testing.assert_allclose(jr, rjr[0], atol=1e-12, rtol=0)
        np.testing.assert_allclose(env._utils.get_site_xvelp(env.model, d, name), rjp[0] @ d.qvel, atol=1e-12)
        np.testing.assert_allclose(env._utils.get_site_xvelr(env.model, d, name), rjr[0] @ d.qvel, atol=1e-12)
    q = np.zeros(4)
    env._mujoco.mju_mat2Quat(q, d.site_xmat[model.site_id("ee_center_site")].reshape(9, 1))
    np.testing.assert_allclose(q, O.mat2quat(d.site_xmat[model.site_id("ee_center_site")]), atol=1e-14)


def test_data_writes_reach_the_device(env):
    """data is the state of record: a qpos write before step() is what the kernel integrates."""
    from pnp_amd.envs import EnvConfig, FrankaShelfPNPEnv
    e = FrankaShelfPNPEnv(config=EnvConfig(n_substeps=1))
    e.reset()
    e.set_mocap_pose(e.get_ee_position() + [0, 0, 0.05], e.get_ee_orientation())
    e.unwrapped._mujoco.mj_step(e.model, e.data, nstep=50)
    assert e.get_ee_position()[2] > e.home_pos[2] + 0.005         # the weld pulled the hand up
    e.set_joint_neutral()
    e.unwrapped._mujoco.mj_forward(e.model, e.data)
    np.testing.assert_allclose(e.get_ee_position(), e.home_pos, atol=1e-10)
    assert e.get_fingers_width().shape == (1,)


def test_skills_replay_reference_episode_on_device():
    from pnp_amd.envs import EnvConfig, FrankaShelfPNPEnv
    G = H.load_golden()
    env = FrankaShelfPNPEnv(config=EnvConfig(n_substeps=int(G["n_substeps"])), dtype=torch.float64)
    env.reset()
    np.testing.assert_allclose(env.data.qpos, G["reset_qpos"], atol=1e-12, rtol=0)
    out = H.run_episode(env, G)
    worst = H.compare(out, G, 1e-6)
    print("skill episode worst |diff|:", {k: f"{v:.1e}" for k, v in worst.items()})


def test_batched_moveik_planner_matches_sequential(model):
    """BatchedMoveIKPlanner (one IK launch per round for all envs) == plan_ik_waypoints per env
    with the single-solve JacobianIKController (the fallback logic is covered on the CPU by
    tests/test_skills_oracle.py::test_batched_planner_fallbacks_match_sequential)."""
    from pnp_amd.engine import get_engine
    from pnp_amd.ik_solver import JacobianIKController
    from pnp_amd.skills import plan_ik_waypoints
    from pnp_amd.skills.batched import BatchedMoveIKPlanner
    from pnp_amd.workloads import NEUTRAL
    eng = get_engine()
    rng = np.random.default_rng(7)
    B = 12
    qpos = np.tile(model.qpos0, (B, 1))
    qpos[:, :9] = NEUTRAL
    qpos[:, :7] += rng.uniform(-0.3, 0.3, size=(B, 7))
    sx, sm = eng.site_kinematics(torch.as_tensor(qpos, dtype=torch.float64, device=eng.device))
    ee = model.site_id("ee_center_site")
    start = sx[:, ee].cpu().numpy()
    quat = np.tile([1.0, 0, 0, 0], (B, 1))
    tgt = start + rng.uniform(-0.08, 0.08, size=(B, 3))
    logs = [[] for _ in range(B)]
    planner = BatchedMoveIKPlanner()
    got = planner.plan(start, quat, qpos[:, :7], tgt, logs=logs)
    ik = JacobianIKController(model)
    for b in range(B):
        lb = []
        pos, qt = plan_ik_waypoints(ik, start[b], quat[b], qpos[b, :7], tgt[b], log=lb.append)
        assert len(got[b][0]) == len(pos), b
        np.testing.assert_allclose(np.array(got[b][0]), np.array(pos), atol=1e-12, rtol=0)
        np.testing.assert_allclose(np.array(got[b][1]), np.array(qt), atol=0, rtol=0)
        assert logs[b] == lb, b
    n_solves = sum(len(p) for p, _ in got)
    assert planner.launches < n_solves                             # batching saved launches


def test_device_slerp_matches_scipy():
    """RotateSkill's trajectory on the device (pnp_slerp_track_f64) against scipy itself
    (Rotation composition + Slerp at np.linspace(0, 1, steps), reference skills/rotate.py:39-46)
    on random and near-identity rotations: within 1e-14."""
    from scipy.spatial.transform import Rotation, Slerp
    from pnp_amd.engine import get_engine
    rng = np.random.default_rng(0)
    B, steps = 64, 50
    q0 = rng.normal(size=(B, 4))
    dq = rng.normal(size=(B, 4))
    dq[::4] = Rotation.from_euler("y", -90, degrees=True).as_quat()
    dq[1::4] = [0, 0, 1e-6, 1.0]                       # small-angle branch of as_rotvec / from_rotvec
    tgt, trk = get_engine().slerp_track(q0, dq, steps)
    for b in range(B):
        t_ref = (Rotation.from_quat(q0[b]) * Rotation.from_quat(dq[b])).as_quat()
        ref = Slerp([0, 1], Rotation.from_quat([q0[b] / np.linalg.norm(q0[b]), t_ref]))(
            np.linspace(0, 1, steps, endpoint=True)).as_quat()
        assert np.abs(tgt[b] - t_ref).max() < 1e-14
        assert np.abs(trk[b] - ref).max() < 1e-14, b
