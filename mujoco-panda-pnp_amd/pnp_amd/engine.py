"""Device-resident engine: a pnp_model handle plus batched launches on torch tensors.

All tensors are CUDA (HIP) tensors owned by the caller; launches go on
``torch.cuda.current_stream()``.  fp32 tensors use the product kernels, fp64 tensors the
debugging instantiation of the same kernels.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import torch

from . import _lib
from .model import PandaModel, PnpIKParams, load_model


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need(t, dtype, shape_tail, name):
    if t is None:
        raise ValueError(f"{name} is required")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device}); the engine has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if tuple(t.shape[1:]) != tuple(shape_tail):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected [B, {', '.join(map(str, shape_tail))}]")
    return t


class Engine:
    """Owns one device image of the compiled model (pnp_model_create)."""

    def __init__(self, model: PandaModel | None = None, device=None):
        self.model = model or load_model()
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.pnp_model_create(C.byref(self.model.desc()), C.byref(h)), "pnp_model_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.pnp_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ kinematics
    def site_kinematics(self, qpos, mocap_pos=None, mocap_quat=None, want_xmat=True):
        m = self.model
        dt = qpos.dtype
        _need(qpos, dt, (m.nq,), "qpos")
        B = qpos.shape[0]
        if mocap_pos is not None:
            _need(mocap_pos, dt, (m.nmocap * 3,), "mocap_pos")
        if mocap_quat is not None:
            _need(mocap_quat, dt, (m.nmocap * 4,), "mocap_quat")
        sx = torch.empty(B, m.nsite, 3, dtype=dt, device=qpos.device)
        sm = torch.empty(B, m.nsite, 9, dtype=dt, device=qpos.device) if want_xmat else None
        fn = self.lib.pnp_site_kinematics if dt == torch.float32 else self.lib.pnp_site_kinematics_f64
        _lib.check(fn(self._h, _ptr(qpos), _ptr(mocap_pos), _ptr(mocap_quat), _ptr(sx), _ptr(sm), B,
                      _stream()), "pnp_site_kinematics")
        return sx, sm

    def jac_site(self, qpos, site="ee_center_site"):
        m = self.model
        _need(qpos, qpos.dtype, (m.nq,), "qpos")
        B = qpos.shape[0]
        jac = torch.empty(B, 3, m.nv, dtype=qpos.dtype, device=qpos.device)
        fn = self.lib.pnp_jac_site if qpos.dtype == torch.float32 else self.lib.pnp_jac_site_f64
        sid = site if isinstance(site, int) else m.site_id(site)
        _lib.check(fn(self._h, sid, _ptr(qpos), _ptr(jac), B, _stream()), "pnp_jac_site")
        return jac

    def jac_site_full(self, qpos, site, mocap_pos=None, mocap_quat=None, want_jacp=True, want_jacr=True):
        """mj_jacSite: (jacp [B, 3, nv], jacr [B, 3, nv]) of `site` (either None when not wanted)."""
        m = self.model
        dt = qpos.dtype
        _need(qpos, dt, (m.nq,), "qpos")
        B = qpos.shape[0]
        if mocap_pos is not None:
            _need(mocap_pos, dt, (m.nmocap * 3,), "mocap_pos")
        if mocap_quat is not None:
            _need(mocap_quat, dt, (m.nmocap * 4,), "mocap_quat")
        jp = torch.empty(B, 3, m.nv, dtype=dt, device=qpos.device) if want_jacp else None
        jr = torch.empty(B, 3, m.nv, dtype=dt, device=qpos.device) if want_jacr else None
        fn = self.lib.pnp_jac_site_full if dt == torch.float32 else self.lib.pnp_jac_site_full_f64
        sid = site if isinstance(site, int) else m.site_id(site)
        _lib.check(fn(self._h, sid, _ptr(qpos), _ptr(mocap_pos), _ptr(mocap_quat), _ptr(jp), _ptr(jr), B,
                      _stream()), "pnp_jac_site_full")
        return jp, jr

    # ------------------------------------------------------------------ physics
    def new_state(self, B, dtype=torch.float32):
        """Model-default state (mj_resetData) for B envs: dict of device tensors (SoA)."""
        m, dev = self.model, self.device
        mb = int((m.body_mocapid >= 0).nonzero()[0][0])
        t = lambda a: torch.as_tensor(a, dtype=dtype, device=dev).contiguous()
        import numpy as np
        return dict(qpos=t(np.tile(m.qpos0, (B, 1))), qvel=t(np.zeros((B, m.nv))), ctrl=t(np.zeros((B, m.nu))),
                    mocap_pos=t(np.tile(m.body_pos[mb], (B, 1))), mocap_quat=t(np.tile(m.body_quat[mb], (B, 1))),
                    qacc_warmstart=t(np.zeros((B, m.nv))), time=t(np.zeros(B)),
                    warn=torch.zeros(B, dtype=torch.int32, device=dev))

    def _state_struct(self, st):
        m = self.model
        dt = st["qpos"].dtype
        B = st["qpos"].shape[0]
        shapes = dict(qpos=(m.nq,), qvel=(m.nv,), ctrl=(m.nu,), mocap_pos=(3 * m.nmocap,),
                      mocap_quat=(4 * m.nmocap,), qacc_warmstart=(m.nv,), time=(), warn=())
        for k, tail in shapes.items():
            t = st[k]
            want = torch.int32 if k == "warn" else dt
            if t.dtype != want or not t.is_cuda or not t.is_contiguous() or tuple(t.shape) != (B,) + tail:
                raise ValueError(f"state[{k}]: need contiguous {want} device tensor of shape {(B,) + tail}, "
                                 f"got {t.dtype} {tuple(t.shape)} on {t.device}")
        return _lib.PnpState(*[t.data_ptr() for t in (st[k] for k in _lib.STATE_FIELDS)]), B, dt

    def step(self, st, nsub=1):
        """nsub x mj_step in place on every env (fp32: product kernel; fp64: debug instantiation)."""
        S, B, dt = self._state_struct(st)
        fn = self.lib.pnp_step if dt == torch.float32 else self.lib.pnp_step_f64
        _lib.check(fn(self._h, C.byref(S), B, int(nsub), _stream()), "pnp_step")
        return st

    STAGES = ("check", "kinematics", "compos_crb", "factor_M", "collision", "constraints", "velocity_rne",
              "actuation_smooth", "newton_setup", "newton_grad_hess", "newton_dir", "newton_linesearch",
              "newton_update", "noslip", "finish_accel", "euler",
              # sub-stages (also inside their parent's cycles)
              "col_broadphase", "col_primitive", "col_convex", "noslip_W", "noslip_lists",
              "kin_prologue", "kin_levels", "kin_frames", "newton_gradient", "newton_converge", "newton_hessian",
              # per-sub-step counts (summed over sub-steps), not cycles
              "n_con", "n_efc", "n_newton_iter", "n_convex", "n_island", "n_noslip_sweep", "n_live",
              # ad-hoc sub-stage timers (cycles; see the sub_lap calls in csrc/step.hip)
              "aux0", "aux1", "aux2", "aux3", "aux4", "aux5", "aux6", "aux7",
              # noslip path counts (sub-steps on the dense long-list / the streaming path)
              "n_ns_dense", "n_ns_stream",
              # noslip sweeps run (mj_solNoSlip's early exit on noslip_tolerance)
              "n_noslip_iter")
    N_STAGE_CYCLES = 27

    def step_profile(self, st, nsub=1):
        """Diagnostic timed instantiation of pnp_step: per-stage shader cycles and per-step counts
        [B, len(STAGES)] (int64, summed over the nsub sub-steps; see include/pnp.h)."""
        S, B, dt = self._state_struct(st)
        if dt != torch.float32:
            raise TypeError("step_profile times the fp32 product kernel")
        prof = torch.zeros(B, len(self.STAGES), dtype=torch.int64, device=self.device)
        _lib.check(self.lib.pnp_step_profile(self._h, C.byref(S), B, int(nsub), _ptr(prof), _stream()),
                   "pnp_step_profile")
        return prof

    def forward_debug(self, st):
        """One mj_forward per env; returns the PNP_DBG_* record [B, PNP_DBG_SIZE] (float64)."""
        S, B, dt = self._state_struct(st)
        dbg = torch.zeros(B, _lib.DBG["SIZE"], dtype=torch.float64, device=self.device)
        fn = self.lib.pnp_forward_debug if dt == torch.float32 else self.lib.pnp_forward_debug_f64
        _lib.check(fn(self._h, C.byref(S), B, _ptr(dbg), _stream()), "pnp_forward_debug")
        return dbg

    # ------------------------------------------------------------------ IK
    def ik_dls_into(self, q_init, target, out, site="ee_center_site", max_iters=100, pos_thresh=1e-3,
                    damping=1e-2, step_limit=0.1):
        """Launch only (no allocation): ``out`` = dict(q, final_pos, pos_error, iterations, flags)."""
        B = q_init.shape[0]
        fn = self.lib.pnp_ik_dls if q_init.dtype == torch.float32 else self.lib.pnp_ik_dls_f64
        sid = site if isinstance(site, int) else self.model.site_id(site)
        prm = PnpIKParams(int(max_iters), float(pos_thresh), float(damping), float(step_limit))
        _lib.check(fn(self._h, sid, prm, _ptr(q_init), _ptr(target), _ptr(out["q"]), _ptr(out["final_pos"]),
                      _ptr(out["pos_error"]), _ptr(out["iterations"]), _ptr(out["flags"]), B, _stream()),
                   "pnp_ik_dls")
        return out

    def ik_dls(self, q_init, target, site="ee_center_site", **params):
        """Batched JacobianIKController.solve (reference skills/ik_solver.py:35-101)."""
        dt = q_init.dtype
        _need(q_init, dt, (7,), "q_init")
        _need(target, dt, (3,), "target")
        B, dev = q_init.shape[0], q_init.device
        out = dict(q=torch.empty(B, 7, dtype=dt, device=dev), final_pos=torch.empty(B, 3, dtype=dt, device=dev),
                   pos_error=torch.empty(B, dtype=dt, device=dev),
                   iterations=torch.empty(B, dtype=torch.int32, device=dev),
                   flags=torch.empty(B, dtype=torch.uint8, device=dev))
        return self.ik_dls_into(q_init, target, out, site=site, **params)


    # ------------------------------------------------------------------ skills
    def slerp_track(self, start_xyzw, delta_xyzw, steps):
        """RotateSkill's trajectories for B skills (pnp_slerp_track_f64, reference
        skills/rotate.py:39-46): returns (target [B,4], track [B,steps,4]), scipy x, y, z, w."""
        dev = self.device
        a = torch.as_tensor(np.asarray(start_xyzw, np.float64).reshape(-1, 4), device=dev).contiguous()
        d = torch.as_tensor(np.asarray(delta_xyzw, np.float64).reshape(-1, 4), device=dev).contiguous()
        B = a.shape[0]
        if d.shape[0] != B:
            raise ValueError("start and delta quaternions must have the same batch size")
        tgt = torch.empty(B, 4, dtype=torch.float64, device=dev)
        trk = torch.empty(B, int(steps), 4, dtype=torch.float64, device=dev)
        _lib.check(self.lib.pnp_slerp_track_f64(_ptr(a), _ptr(d), int(steps), _ptr(tgt), _ptr(trk), B, _stream()),
                   "pnp_slerp_track_f64")
        return tgt.cpu().numpy(), trk.cpu().numpy()


_ENGINES = {}


def get_engine(device=None) -> Engine:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (dev.type, dev.index)
    if key not in _ENGINES:
        _ENGINES[key] = Engine(device=dev)
    return _ENGINES[key]
