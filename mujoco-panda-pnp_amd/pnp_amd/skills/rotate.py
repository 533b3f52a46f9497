"""In-place end-effector rotation (reference panda_mujoco_gym/skills/rotate.py:12-74).

Quaternion convention, as in the reference: the env reports MuJoCo wxyz quaternions and the skill
hands them to scipy (xyzw) unchanged, composes with ``delta_quat`` (given as xyzw) and sends
scipy's output back as a mocap wxyz quaternion.  Kept as is: the
behaviour tree's waypoints and thresholds were tuned against exactly this arithmetic.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation, Slerp

from .base import Skill


def slerp_track(start_quat, target_quat, steps):
    """``steps`` quaternions from start to target inclusive (scipy Slerp, rotate.py:42-46)."""
    keys = Rotation.from_quat([start_quat, target_quat])
    return Slerp([0, 1], keys)(np.linspace(0, 1, steps, endpoint=True)).as_quat()


class RotateSkill(Skill):
    """Rotate the end-effector in place by ``delta_quat`` over ``steps`` ticks."""

    def __init__(self, env, delta_quat: np.ndarray, steps: int = 50, err_thresh: float = 0.01):
        super().__init__(env)
        assert len(delta_quat) == 4, "delta_quat must be xyzw quaternion"
        self.delta_quat = np.asarray(delta_quat, dtype=float)
        self.steps = max(1, steps)
        self.err_thresh = err_thresh

    def reset(self):
        self.i = 0
        self.done = False
        self.start_pos = self.env.get_ee_position().copy()
        self.start_quat = self.env.get_ee_orientation().copy()
        dev = getattr(self.env.unwrapped, "slerp_track", None)
        if dev is not None:
            # on the device (pnp_slerp_track_f64: scipy's composition + Slerp restated, within
            # 1e-15 of them); batched envs serve many resets in one launch (pnp_amd.batched_bt)
            self.target_quat, self.quat_traj = dev(self.start_quat, self.delta_quat, self.steps)
        else:
            self.target_quat = (Rotation.from_quat(self.start_quat) * Rotation.from_quat(self.delta_quat)).as_quat()
            self.quat_traj = slerp_track(self.start_quat, self.target_quat, self.steps)

    def step(self) -> np.ndarray:
        if self.done:
            return self.zero_action()
        if self.i >= self.steps:
            self.done = True
            return self.zero_action()
        self.env.set_mocap_pose(self.start_pos, self.quat_traj[self.i])
        self._step_sim(n=5)
        self.i += 1
        if Skill.quat_close(self.env.get_ee_orientation(), self.target_quat, self.err_thresh):
            self.done = True
        return self.zero_action()
