"""Drop-in ``JacobianIKController`` / ``IKResult`` backed by the HIP DLS-IK kernel.

Mirrors reference ``panda_mujoco_gym/skills/ik_solver.py`` (IKResult :16-24, constructor
:27-33, solve :35-101): same names, argument meaning, defaults and result fields, so callers such
as ``MoveIKSkill.reset`` (reference skills/move.py:84-85,128) keep working.  Every solve runs on
the device; there is no host fallback.

``BatchedIK`` is the batched form (the hot path of BASELINE config C2): B solves per launch.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .engine import Engine, get_engine
from .model import load_model


_MODEL_ENGINES = {}


def _engine_for(model, device):
    """The engine whose device image is `model`: site ids and joint limits are looked up in the
    model the caller passed, so the kinematics solved must be that model's too."""
    eng = get_engine(device)
    if model is eng.model:
        return eng
    key = (id(model), eng.device.type, eng.device.index)
    hit = _MODEL_ENGINES.get(key)
    if hit is None or hit[0] is not model:
        hit = (model, Engine(model=model, device=eng.device))
        _MODEL_ENGINES[key] = hit
    return hit[1]


@dataclass
class IKResult:
    """Result of IK solving (reference skills/ik_solver.py:16-24)."""
    success: bool
    q: np.ndarray
    final_pos: np.ndarray
    pos_error: float
    iterations: int
    converged: bool


class JacobianIKController:
    """Position-only damped-least-squares IK on a site (reference skills/ik_solver.py:26-101).

    ``model`` is the compiled model (``PandaModel``, MjModel field names) and ``data`` any object
    with a writable ``qpos`` array; like the reference, solve() leaves ``data.qpos[:7]`` at the
    returned joint angles.  Single solves run the fp64 instantiation of the kernel (bitwise close
    to the reference's numpy/fp64 arithmetic); ``dtype=torch.float32`` selects the product path.
    """

    def __init__(self, model=None, data=None, site_name: str = "ee_center_site",
                 device=None, dtype=torch.float64):
        self.model = model if model is not None else load_model()
        self.data = data
        self.site_id = self.model.site_id(site_name)
        self.joint_ids = np.arange(7)
        self.lower = np.asarray(self.model.jnt_range)[:7, 0].copy()
        self.upper = np.asarray(self.model.jnt_range)[:7, 1].copy()
        self.dtype = dtype
        self.engine = _engine_for(self.model, device)

    def solve(self, target_pos: np.ndarray, q_init: np.ndarray, max_iters: int = 100,
              pos_thresh: float = 1e-3, damping: float = 1e-2, step_limit: float = 0.1) -> IKResult:
        dev = self.engine.device
        q0 = torch.as_tensor(np.asarray(q_init, np.float64).reshape(1, 7), dtype=self.dtype, device=dev)
        tg = torch.as_tensor(np.asarray(target_pos, np.float64).reshape(1, 3), dtype=self.dtype, device=dev)
        out = self.engine.ik_dls(q0, tg, site=self.site_id, max_iters=max_iters, pos_thresh=pos_thresh,
                                 damping=damping, step_limit=step_limit)
        q = out["q"][0].double().cpu().numpy()
        fp = out["final_pos"][0].double().cpu().numpy()
        fl = int(out["flags"][0].item())
        if self.data is not None and hasattr(self.data, "qpos"):
            self.data.qpos[:7] = q
        return IKResult(success=bool(fl & 2), q=q, final_pos=fp, pos_error=float(out["pos_error"][0].item()),
                        iterations=int(out["iterations"][0].item()), converged=bool(fl & 1))


class BatchedIK:
    """B independent solves per launch (device tensors in, device tensors out)."""

    def __init__(self, site_name: str = "ee_center_site", device=None, model=None):
        self.engine = get_engine(device) if model is None else _engine_for(model, device)
        self.model = self.engine.model
        self.site_id = self.model.site_id(site_name)

    def solve(self, target_pos: torch.Tensor, q_init: torch.Tensor, **params):
        return self.engine.ik_dls(q_init, target_pos, site=self.site_id, **params)
