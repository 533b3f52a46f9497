"""Scripted-skill base class (reference panda_mujoco_gym/skills/base.py:11-80).

A skill emits one 7-d action per ``step()`` and may drive the simulation itself through the env's
MuJoCo-binding surface (``env.unwrapped._mujoco.mj_step``, base.py:38-44), which on this engine is
pnp_amd/mjshim.py: the sub-steps run on the device.
"""
from __future__ import annotations

import abc

import numpy as np


class Skill(abc.ABC):
    """Abstract scripted skill; subclasses implement ``reset`` and ``step``."""

    def __init__(self, env):
        self.env = env
        self.done = False

    @abc.abstractmethod
    def reset(self):
        """Re-arm the skill (pre-compute its trajectory)."""
        self.done = False

    @abc.abstractmethod
    def step(self) -> np.ndarray:
        """One control tick; returns a 7-d action."""

    def is_done(self) -> bool:
        return self.done

    def zero_action(self) -> np.ndarray:
        return np.zeros_like(self.env.action_space.low, dtype=np.float32)

    def _step_sim(self, n: int = 1):
        """Advance the physics by n sub-steps (base.py:38-47).  The reference issues n
        mj_step(nstep=1) calls; one mj_step(nstep=n) is the same computation and leaves the same
        data.site_* (the last sub-step's forward), with one device round trip instead of n."""
        u = self.env.unwrapped
        if n > 0:
            u._mujoco.mj_step(u.model, u.data, nstep=n)
        if hasattr(self.env, "render") and self.env.render_mode is not None:
            self.env.render()

    # ---- termination predicates shared by the skills and the behaviour tree (base.py:50-80)
    @staticmethod
    def pos_close(pos1: np.ndarray, pos2: np.ndarray, thresh: float = 0.01) -> bool:
        return np.linalg.norm(pos1 - pos2) < thresh

    @staticmethod
    def quat_close(q1: np.ndarray, q2: np.ndarray, thresh: float = 0.01) -> bool:
        """Same rotation up to sign: 1 - |<q1, q2>| below thresh."""
        return 1.0 - abs(np.dot(q1, q2)) < thresh

    @staticmethod
    def fingers_closed(width: float, thresh: float = 0.2) -> bool:
        return width < thresh

    @staticmethod
    def fingers_open(width: float, thresh: float = 0.08) -> bool:
        return width > thresh

    @staticmethod
    def retreated_enough(p_now: np.ndarray, p_target: np.ndarray, thresh: float = 0.01) -> bool:
        return np.linalg.norm(p_now - p_target) < thresh
