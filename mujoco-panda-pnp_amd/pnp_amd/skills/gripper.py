"""Gripper open / close primitive (reference panda_mujoco_gym/skills/gripper.py:20-89).

Each tick sends a gym action that only drives the finger channel (a[6] = -1 close, +1 open:
one full env.step, i.e. 250 sub-steps), then 5 more sub-steps.  Done once ``duration`` ticks have
passed and the width predicate holds.  The width comes from ``env.get_gripper_width()`` if the
env has one; FrankaEnv (and this engine's facade) does not, so the predicate falls back to its
default and always holds (0.0 for close, inf for open: gripper.py:60-71) -- the skill is
effectively timed.  Kept as is for drop-in behaviour.
"""
from __future__ import annotations

from typing import Literal

import numpy as np

from .base import Skill

DEFAULTS = {"close": (10, 0.02), "open": (15, 0.08)}    # (duration ticks, width threshold)


class GripperSkill(Skill):

    def __init__(self, env, mode: Literal["close", "open"], *, duration: int | None = None,
                 thresh: float | None = None):
        super().__init__(env)
        assert mode in ("close", "open"), "mode must be 'close' or 'open'"
        self.mode = mode
        d, t = DEFAULTS[mode]
        self.duration = d if duration is None else duration
        self.thresh = t if thresh is None else thresh
        self.i = 0

    @classmethod
    def close(cls, env, **kw):
        return cls(env, "close", **kw)

    @classmethod
    def open(cls, env, **kw):
        return cls(env, "open", **kw)

    def reset(self):
        self.i = 0
        self.done = False

    def _current_width(self) -> float:
        fallback = 0.0 if self.mode == "close" else np.inf
        getter = getattr(self.env, "get_gripper_width", None)
        if not callable(getter):
            return fallback
        try:
            w = float(getter())
        except Exception:
            return fallback
        return w if np.isfinite(w) else fallback

    def step(self):
        if self.done:
            return np.zeros(7, dtype=np.float32)
        action = np.zeros(7, dtype=np.float32)
        action[-1] = -1.0 if self.mode == "close" else 1.0
        self.env.step(action)
        self._step_sim(n=5)
        self.i += 1
        width = self._current_width()
        ok = (Skill.fingers_closed(width, self.thresh) if self.mode == "close"
              else Skill.fingers_open(width, self.thresh))
        if self.i >= self.duration and ok:
            self.done = True
        return action
