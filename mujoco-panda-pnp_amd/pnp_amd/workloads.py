"""Synthetic workloads of BASELINE.json's configs (BASELINE.md "Baseline plan").

C2 (IK only, free space): q_init ~ U(inner 90% of jnt_range[:7]) per joint (limits from
panda_mocap.xml via the compiled model), target = FK(q_init) + delta with
delta ~ U(+-0.02 m)^3 ("MoveIK waypoint" regime, reference skills/move.py:114-117) or
U(+-0.1 m)^3 (ik_test regime, reference test/ik_test.py:26).  Parameter sets: the
JacobianIKController.solve defaults (100, 1e-3, 1e-2, 0.1) (skills/ik_solver.py:35-37) and the
ik_test ones (100, 1e-4, 0.05, 0.1) (test/ik_test.py:33-37).

C3/C4 (full env-step on the shelf_pnp scene): the reference's reset distribution
(envs/panda_env.py:124-158): neutral arm (panda_env.py:65) with the arm servo targets at neutral
(:127), mocap at the ee_center_site pose, cubes at their XML sites + U(+-0.02, +-0.2) in x/y
(shelf_pnp.py:23-24) with identity orientation; then per step ctrl ~ U(actuator_ctrlrange)
(SURVEY §8d).  Cube offsets use Philox stream 3; the ctrl of step s uses stream 16 + s.

FK (IK targets, mocap pose, site positions) is supplied by the caller (the engine's own site
kinematics on the device, or the oracle in tests), so this module is pure input generation.
"""
from __future__ import annotations

import numpy as np

from . import rng
from .mjcf import mat2quat

NEUTRAL = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00])   # panda_env.py:65
CUBES = ("cube1", "cube2", "cube3")

IK_PARAMS = {
    "default": dict(max_iters=100, pos_thresh=1e-3, damping=1e-2, step_limit=0.1),
    "ik_test": dict(max_iters=100, pos_thresh=1e-4, damping=0.05, step_limit=0.1),
}
IK_REGIMES = {"waypoint": 0.02, "ik_test": 0.1}


def ik_inputs(model, env_index, regime="waypoint", seed=rng.SEED):
    """Returns (q_init [N,7], delta [N,3]) float64; target = FK(q_init) + delta."""
    u = rng.uniform(env_index, 10, seed=seed, stream=2)
    lo, hi = model.jnt_range[:7, 0], model.jnt_range[:7, 1]
    span = hi - lo
    q = (lo + 0.05 * span) + u[:, :7] * (0.9 * span)
    r = IK_REGIMES[regime]
    delta = (u[:, 7:10] * 2.0 - 1.0) * r
    return q, delta


def c3_reset(model, env_index, site_xpos, site_xmat, seed=rng.SEED):
    """Reset-distribution states for the given global env indices (float64 SoA dict).

    site_xpos [nsite,3] / site_xmat [nsite,9]: site poses at the neutral arm pose (FK by the caller).
    """
    env_index = np.asarray(env_index)
    n = env_index.size
    u = rng.uniform(env_index, 6, seed=seed, stream=3)
    qpos = np.tile(model.qpos0, (n, 1))
    qpos[:, :9] = NEUTRAL
    ctrl = np.zeros((n, model.nu))
    ctrl[:, :7] = NEUTRAL[:7]
    ee = model.site_id("ee_center_site")
    for k, name in enumerate(CUBES):
        a = int(model.jnt_qposadr[model.joint_id(f"{name}_joint")])
        c = site_xpos[model.site_id(f"{name}_site")]
        qpos[:, a] = c[0] + (u[:, 2 * k] * 2 - 1) * 0.02
        qpos[:, a + 1] = c[1] + (u[:, 2 * k + 1] * 2 - 1) * 0.2
        qpos[:, a + 2] = c[2]
        qpos[:, a + 3:a + 7] = [1, 0, 0, 0]
    mq = mat2quat(np.asarray(site_xmat[ee]).reshape(3, 3))
    return dict(qpos=qpos, qvel=np.zeros((n, model.nv)), ctrl=ctrl,
                mocap_pos=np.tile(site_xpos[ee], (n, 1)), mocap_quat=np.tile(mq, (n, 1)),
                qacc_warmstart=np.zeros((n, model.nv)), time=np.zeros(n), warn=np.zeros(n, np.uint32))


def c3_ctrl(model, env_index, step, seed=rng.SEED):
    """ctrl ~ U(actuator_ctrlrange) for one step of the given envs: [N, nu] float64."""
    u = rng.uniform(env_index, model.nu, seed=seed, stream=16 + int(step))
    lo, hi = model.actuator_ctrlrange[:, 0], model.actuator_ctrlrange[:, 1]
    return lo + u * (hi - lo)
