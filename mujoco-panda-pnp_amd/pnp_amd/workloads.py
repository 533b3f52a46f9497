"""Synthetic workloads of BASELINE.json's configs (BASELINE.md "Baseline plan").

C2 (IK only, free space): q_init ~ U(inner 90% of jnt_range[:7]) per joint (limits from
panda_mocap.xml via the compiled model), target = FK(q_init) + delta with
delta ~ U(+-0.02 m)^3 ("MoveIK waypoint" regime, reference skills/move.py:114-117) or
U(+-0.1 m)^3 (ik_test regime, reference test/ik_test.py:26).  Parameter sets: the
JacobianIKController.solve defaults (100, 1e-3, 1e-2, 0.1) (skills/ik_solver.py:35-37) and the
ik_test ones (100, 1e-4, 0.05, 0.1) (test/ik_test.py:33-37).

FK(q_init) is supplied by the caller (it is the engine's own site kinematics on the device, or
the oracle in tests), so this module is pure input generation.
"""
from __future__ import annotations

import numpy as np

from . import rng

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
