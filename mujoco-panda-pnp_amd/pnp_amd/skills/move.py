"""Cartesian move skills (reference panda_mujoco_gym/skills/move.py).

``MoveSkill``    straight-line mocap interpolation at fixed orientation (move.py:13-58).
``MoveIKSkill``  waypoints planned with the DLS IK solver, then replayed (move.py:61-208).
``plan_ik_waypoints`` is MoveIKSkill's planner on its own (move.py:76-191), so that callers
(and the batched planner in pnp_amd/skills/batched.py) share one statement of it.
"""
from __future__ import annotations

import copy

import numpy as np

from ..ik_solver import JacobianIKController
from .base import Skill

MAX_MOCAP_STEP = 0.02          # largest waypoint spacing the weld follows stably (move.py:117)
MAX_CONSECUTIVE_FAILURES = 3   # move.py:103


def interpolation_steps(distance: float) -> int:
    """MoveSkill's tick count for a straight move of `distance` metres (move.py:32-40)."""
    if distance > 1.0:
        return 120
    if distance > 0.5:
        return 60
    return 20


class MoveSkill(Skill):
    """Move the end-effector along a straight line to ``target_pos``, orientation held."""

    def __init__(self, env, target_pos: np.ndarray, steps: int = 30, pos_thresh: float = 0.02):
        super().__init__(env)
        assert pos_thresh > 0, "pos_thresh must be positive"
        self.target_pos = np.asarray(target_pos, float)
        self.steps = steps
        self.pos_thresh = pos_thresh
        self.i = 0

    def reset(self):
        self.i = 0
        self.done = False
        self.start_pos = self.env.get_ee_position().copy()
        self.quat = self.env.get_ee_orientation().copy()
        self.steps = interpolation_steps(np.linalg.norm(self.start_pos - self.target_pos))
        self.pos_traj = np.linspace(self.start_pos, self.target_pos, self.steps)

    def step(self):
        if self.done:
            return self.zero_action()
        if self.i < self.steps:
            # interpolation phase: one waypoint per tick, 5 sub-steps each
            self.env.set_mocap_pose(self.pos_traj[self.i], self.quat)
            self._step_sim(n=5)
            self.i += 1
        else:
            # settle phase: hold the target until the end-effector is within pos_thresh
            self.env.set_mocap_pose(self.target_pos, self.quat)
            if Skill.pos_close(self.env.get_ee_position(), self.target_pos, self.pos_thresh):
                self.done = True
        return self.zero_action()


def plan_ik_waypoints(ik, start_pos, start_quat, q_start, target_pos, pos_thresh=0.01,
                      max_traj_points=200, step_size=0.01, log=print):
    """MoveIKSkill's adaptive planner (move.py:95-191): march towards ``target_pos`` in IK-checked
    steps of at most min(step_size, 0.1 * remaining, 0.02) m, halved after a failure; after three
    failures in a row try a ten-times smaller step, then the same step with y frozen, else stop.
    Returns (pos_traj, quat_traj): lists of 3-vectors / quaternions (orientation held)."""
    target = np.asarray(target_pos, float)
    pos = np.asarray(start_pos, float).copy()
    quat = np.asarray(start_quat, float).copy()
    q = np.asarray(q_start, float).copy()
    pos_traj, quat_traj = [pos.copy()], [quat.copy()]

    def accept(res):
        nonlocal pos, q
        pos_traj.append(res.final_pos.copy())
        quat_traj.append(quat.copy())
        pos = res.final_pos.copy()
        q = res.q.copy()

    points = 0
    failures = 0
    while np.linalg.norm(pos - target) > pos_thresh and points < max_traj_points:
        direction = target - pos
        distance = np.linalg.norm(direction)
        step = min(min(step_size, distance * 0.1), MAX_MOCAP_STEP)
        if failures > 0:
            step *= 0.5
        goal = pos + direction * step / distance if distance > step else target.copy()
        res = ik.solve(goal, q)
        if res.success and res.pos_error < step_size * 2:
            accept(res)
            failures = 0
        else:
            failures += 1
            if failures < MAX_CONSECUTIVE_FAILURES:
                failures += 1          # the reference counts a plain retry twice (move.py:188-190)
                continue
            log(f"IK failed {failures} times, trying fallback strategies...")
            tiny = step * 0.1                                    # fallback 1: much shorter step
            if distance > tiny:
                res = ik.solve(pos + direction * tiny / distance, q)
                if res.success:
                    accept(res)
                    failures = 0
                    continue
            flat = direction.copy()                               # fallback 2: keep y fixed
            flat[1] = 0
            if np.linalg.norm(flat) > 0.001:
                flat = flat / np.linalg.norm(flat)
                res = ik.solve(pos + flat * step, q)
                if res.success:
                    accept(res)
                    failures = 0
                    continue
            log(f"All fallback strategies failed, stopping at point {points}")
            break
        points += 1
    if np.linalg.norm(pos - target) > pos_thresh:
        pos_traj.append(target.copy())
        quat_traj.append(quat.copy())
    return pos_traj, quat_traj


class MoveIKSkill(Skill):
    """IK-planned move to ``target_pos`` (planning in reset(), replay in step())."""

    def __init__(self, env, target_pos: np.ndarray, pos_thresh: float = 0.01,
                 max_traj_points: int = 200, step_size: float = 0.01):
        super().__init__(env)
        self.target_pos = np.asarray(target_pos, float)
        self.pos_thresh = pos_thresh
        self.max_traj_points = max_traj_points
        self.step_size = step_size
        self.i = 0

    def reset(self):
        self.i = 0
        self.done = False
        model = self.env.unwrapped.model
        data = self.env.unwrapped.data
        self.tmp_data = copy.deepcopy(data)          # the planner's scratch copy (move.py:83-85)
        self.ik_controller = JacobianIKController(model, self.tmp_data)
        self.pos_traj, self.quat_traj = plan_ik_waypoints(
            self.ik_controller, self.env.get_ee_position().copy(), self.env.get_ee_orientation().copy(),
            data.qpos[:7].copy(), self.target_pos, self.pos_thresh, self.max_traj_points, self.step_size)

    def step(self):
        if self.done:
            return self.zero_action()
        if self.i < len(self.pos_traj):
            self.env.set_mocap_pose(self.pos_traj[self.i], self.quat_traj[self.i])
            self._step_sim(n=5)
            self.i += 1
        else:
            self.done = True
        return self.zero_action()
