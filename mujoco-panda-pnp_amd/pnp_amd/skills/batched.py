"""Batched MoveIK planning: ``plan_ik_waypoints`` (reference
skills/move.py:95-191) for B envs at once.

Every env runs the reference planner's state machine unchanged; the envs advance in lockstep,
one planner iteration per round, and each round's IK solves -- the main step, then fallback 1,
then fallback 2 for the envs that reached them -- are one batched DLS launch each (pnp_ik_dls:
the C2 hot path) instead of one launch per solve.  The control logic is host numpy over [B]
arrays.  Per env the result equals the sequential planner's (tests/test_skills_gpu.py).
"""
from __future__ import annotations

import numpy as np
import torch

from ..engine import get_engine
from .move import MAX_CONSECUTIVE_FAILURES, MAX_MOCAP_STEP


def _norms(v):
    """Row norms computed exactly as the sequential planner's np.linalg.norm(vector) (a
    vectorised norm(axis=1) may round differently in the last bit)."""
    return np.array([np.linalg.norm(r) for r in v])


class BatchedMoveIKPlanner:
    """Plans MoveIKSkill waypoints for B envs; ``plan`` returns per-env (pos_traj, quat_traj)."""

    def __init__(self, pos_thresh=0.01, max_traj_points=200, step_size=0.01, device=None, dtype=torch.float64,
                 site_name="ee_center_site", ik_params=None, solve_fn=None):
        """``solve_fn(goals [n,3], q [n,7]) -> (q, final_pos, pos_error, success)`` replaces the
        device DLS solve (tests drive the planner logic with a scripted solver)."""
        self.pos_thresh, self.max_traj_points, self.step_size = pos_thresh, max_traj_points, step_size
        self.dtype = dtype
        self.ik_params = dict(max_iters=100, pos_thresh=1e-3, damping=1e-2, step_limit=0.1)
        self.ik_params.update(ik_params or {})
        self.launches = 0
        self._custom = solve_fn
        if solve_fn is None:
            self.engine = get_engine(device)
            self.site = self.engine.model.site_id(site_name)

    def _solve(self, goals, qs):
        if self._custom is not None:
            self.launches += 1
            return self._custom(goals, qs)
        dev = self.engine.device
        out = self.engine.ik_dls(torch.as_tensor(qs, dtype=self.dtype, device=dev).contiguous(),
                                 torch.as_tensor(goals, dtype=self.dtype, device=dev).contiguous(),
                                 site=self.site, **self.ik_params)
        self.launches += 1
        fl = out["flags"].cpu().numpy().astype(np.int64)
        return (out["q"].double().cpu().numpy(), out["final_pos"].double().cpu().numpy(),
                out["pos_error"].double().cpu().numpy(), (fl & 2) != 0)

    def plan(self, start_pos, start_quat, q_start, target_pos, logs=None):
        P = np.array(start_pos, np.float64).reshape(-1, 3)
        B = P.shape[0]
        Q = np.array(q_start, np.float64).reshape(B, 7)
        quat = np.array(start_quat, np.float64).reshape(B, 4)
        tgt = np.array(target_pos, np.float64).reshape(B, 3)
        trajs = [[P[b].copy()] for b in range(B)]
        points = np.zeros(B, np.int64)
        fails = np.zeros(B, np.int64)
        live = np.ones(B, bool)
        logs = logs if logs is not None else [[] for _ in range(B)]

        def accept(idx, q, fp):
            for j, b in enumerate(idx):
                trajs[b].append(fp[j].copy())
            P[idx] = fp
            Q[idx] = q
            fails[idx] = 0

        while True:
            live &= (_norms(P - tgt) > self.pos_thresh) & (points < self.max_traj_points)
            idx = np.nonzero(live)[0]
            if idx.size == 0:
                break
            d = tgt[idx] - P[idx]
            dist = _norms(d)
            step = np.minimum(np.minimum(self.step_size, dist * 0.1), MAX_MOCAP_STEP)
            step = np.where(fails[idx] > 0, step * 0.5, step)
            far = dist > step
            # same operation order as move.py:124: pos + direction * step / distance
            goals = np.where(far[:, None], P[idx] + d * step[:, None] / np.where(far, dist, 1.0)[:, None], tgt[idx])
            q, fp, err, ok = self._solve(goals, Q[idx])
            good = ok & (err < self.step_size * 2)
            accept(idx[good], q[good], fp[good])
            points[idx[good]] += 1
            bad = ~good
            fails[idx[bad]] += 1
            retry = bad & (fails[idx] < MAX_CONSECUTIVE_FAILURES)
            fails[idx[retry]] += 1                      # a plain retry counts twice (move.py:188-190)
            fb = bad & ~retry                           # three failures: the fallbacks
            for b in idx[fb]:
                logs[b].append(f"IK failed {fails[b]} times, trying fallback strategies...")
            # fallback 1: a ten-times shorter step
            tiny = step * 0.1
            f1 = fb & (dist > tiny)
            done_fb = np.zeros(idx.size, bool)
            if f1.any():
                g = P[idx[f1]] + d[f1] * tiny[f1][:, None] / dist[f1][:, None]
                q1, fp1, _, ok1 = self._solve(g, Q[idx[f1]])
                sel = np.nonzero(f1)[0][ok1]
                accept(idx[sel], q1[ok1], fp1[ok1])
                done_fb[sel] = True
            # fallback 2: the same step with y frozen
            flat = d.copy()
            flat[:, 1] = 0
            fn = _norms(flat)
            f2 = fb & ~done_fb & (fn > 0.001)
            if f2.any():
                g = P[idx[f2]] + flat[f2] / fn[f2][:, None] * step[f2][:, None]
                q2, fp2, _, ok2 = self._solve(g, Q[idx[f2]])
                sel = np.nonzero(f2)[0][ok2]
                accept(idx[sel], q2[ok2], fp2[ok2])
                done_fb[sel] = True
            stop = fb & ~done_fb
            for b in idx[stop]:
                logs[b].append(f"All fallback strategies failed, stopping at point {points[b]}")
            live[idx[stop]] = False
        out = []
        for b in range(B):
            pos = trajs[b]
            if np.linalg.norm(P[b] - tgt[b]) > self.pos_thresh:
                pos.append(tgt[b].copy())
            out.append((pos, [quat[b].copy() for _ in pos]))
        return out
