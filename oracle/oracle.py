"""ctypes binding of liboracle.so — the CPU fp64 restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package (mujoco-panda-pnp_amd/pnp_amd).
See oracle.c for the reference file:line each routine restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "mujoco-panda-pnp_amd"))
from pnp_amd.model import PnpIKParams, load_model  # noqa: E402  (host-side model data only)

# PNP_ORACLE_LIB: another build of the same sources (tools/asan_cpu_tests.sh: liboracle_asan.so)
LIB_PATH = os.environ.get("PNP_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.orc_ik_dls_batch.argtypes = [P, C.c_int, PnpIKParams, P, P, P, P, P, P, P, C.c_int, C.c_int]
        L.orc_ik_dls_batch.restype = C.c_int
        L.orc_site_kinematics_batch.argtypes = [P, P, P, P, P, P, C.c_int]
        L.orc_site_kinematics_batch.restype = C.c_int
        L.orc_jac_site_batch.argtypes = [P, C.c_int, P, P, C.c_int]
        L.orc_jac_site_batch.restype = C.c_int
        L.orc_site_jac2_batch.argtypes = [P, C.c_int, P, P, P, P, P, P, P, C.c_int]
        L.orc_site_jac2_batch.restype = C.c_int
        L.orc_mat2quat.argtypes = [P, P]
        L.orc_mat2quat.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _desc_ptr(model):
    return C.cast(C.pointer(model.desc()), C.c_void_p)


def ik_params(max_iters=100, pos_thresh=1e-3, damping=1e-2, step_limit=0.1):
    return PnpIKParams(int(max_iters), float(pos_thresh), float(damping), float(step_limit))


def ik_dls(q_init, target, site="ee_center_site", nthreads=1, model=None, **params):
    """Batched JacobianIKController.solve on the CPU (fp64)."""
    m = model or load_model()
    q_init = np.ascontiguousarray(q_init, np.float64).reshape(-1, 7)
    target = np.ascontiguousarray(target, np.float64).reshape(-1, 3)
    B = q_init.shape[0]
    out = dict(q=np.zeros((B, 7)), final_pos=np.zeros((B, 3)), pos_error=np.zeros(B),
               iterations=np.zeros(B, np.int32), flags=np.zeros(B, np.uint8))
    rc = lib().orc_ik_dls_batch(_desc_ptr(m), m.site_id(site), ik_params(**params), _p(q_init),
                                _p(target), _p(out["q"]), _p(out["final_pos"]), _p(out["pos_error"]),
                                _p(out["iterations"]), _p(out["flags"]), B, int(nthreads))
    if rc:
        raise RuntimeError("orc_ik_dls_batch failed")
    return out


def site_kinematics(qpos, mocap_pos=None, mocap_quat=None, model=None):
    m = model or load_model()
    qpos = np.ascontiguousarray(qpos, np.float64).reshape(-1, m.nq)
    B = qpos.shape[0]
    if mocap_pos is not None:
        mocap_pos = np.ascontiguousarray(mocap_pos, np.float64).reshape(B, -1)
    if mocap_quat is not None:
        mocap_quat = np.ascontiguousarray(mocap_quat, np.float64).reshape(B, -1)
    sx = np.zeros((B, m.nsite, 3))
    sm = np.zeros((B, m.nsite, 9))
    rc = lib().orc_site_kinematics_batch(_desc_ptr(m), _p(qpos), _p(mocap_pos), _p(mocap_quat),
                                         _p(sx), _p(sm), B)
    if rc:
        raise RuntimeError("orc_site_kinematics_batch failed")
    return sx, sm


def jac_site(qpos, site="ee_center_site", model=None):
    m = model or load_model()
    qpos = np.ascontiguousarray(qpos, np.float64).reshape(-1, m.nq)
    B = qpos.shape[0]
    jac = np.zeros((B, 3, m.nv))
    rc = lib().orc_jac_site_batch(_desc_ptr(m), m.site_id(site), _p(qpos), _p(jac), B)
    if rc:
        raise RuntimeError("orc_jac_site_batch failed")
    return jac


def site_jac2(qpos, site, mocap_pos=None, mocap_quat=None, model=None):
    """Site frames of every site and the full mj_jacSite (jacp, jacr) of `site` at qpos:
    returns site_xpos [B,nsite,3], site_xmat [B,nsite,9], jacp [B,3,nv], jacr [B,3,nv]."""
    m = model or load_model()
    qpos = np.ascontiguousarray(qpos, np.float64).reshape(-1, m.nq)
    B = qpos.shape[0]
    mp = None if mocap_pos is None else np.ascontiguousarray(mocap_pos, np.float64).reshape(B, -1)
    mq = None if mocap_quat is None else np.ascontiguousarray(mocap_quat, np.float64).reshape(B, -1)
    sx, sm = np.zeros((B, m.nsite, 3)), np.zeros((B, m.nsite, 9))
    jp, jr = np.zeros((B, 3, m.nv)), np.zeros((B, 3, m.nv))
    sid = site if isinstance(site, (int, np.integer)) else m.site_id(site)
    rc = lib().orc_site_jac2_batch(_desc_ptr(m), int(sid), _p(qpos), _p(mp), _p(mq), _p(sx), _p(sm), _p(jp), _p(jr), B)
    if rc:
        raise RuntimeError("orc_site_jac2_batch failed")
    return sx, sm, jp, jr


def mat2quat(mat):
    mat = np.ascontiguousarray(mat, np.float64).reshape(9)
    q = np.zeros(4)
    lib().orc_mat2quat(_p(q), _p(mat))
    return q


# ------------------------------------------------------------------ physics (physics.c)
STATE_KEYS = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time", "warn")


def _phys_lib():
    L = lib()
    if not getattr(L, "_phys_ready", False):
        P = C.c_void_p
        L.orc_step_batch.argtypes = [P, P, P, P, P, P, P, P, P, C.c_int, C.c_int, C.c_int]
        L.orc_step_batch.restype = C.c_int
        L.orc_data_new.restype = P
        L.orc_data_free.argtypes = [P]
        L.orc_set_state.argtypes = [P, P, P, P, P, P, P, P]
        L.orc_forward.argtypes = [P, P]
        L.orc_step.argtypes = [P, P]
        L.orc_field.argtypes = [P, P, C.c_char_p, P, C.c_int]
        L.orc_field.restype = C.c_int
        L.orc_convex_probe.argtypes = [P, P, C.c_int, C.c_int, P, P, P]
        L.orc_convex_probe.restype = C.c_int
        L.orc_set_boxbox_variant.argtypes = [C.c_int]
        L.orc_set_boxbox_variant.restype = None
        L.orc_mpr_stats.argtypes = [C.POINTER(C.c_longlong), C.c_int]
        L.orc_mpr_stats.restype = None
        L._phys_ready = True
    return L


def new_state(B, model=None):
    """Model-default state (mj_resetData) for B envs, float64 SoA."""
    m = model or load_model()
    mocap_body = int(np.nonzero(m.body_mocapid >= 0)[0][0])
    return dict(qpos=np.tile(m.qpos0, (B, 1)), qvel=np.zeros((B, m.nv)), ctrl=np.zeros((B, m.nu)),
                mocap_pos=np.tile(m.body_pos[mocap_body], (B, 1)),
                mocap_quat=np.tile(m.body_quat[mocap_body], (B, 1)),
                qacc_warmstart=np.zeros((B, m.nv)), time=np.zeros(B), warn=np.zeros(B, np.uint32))


def step(state, nsub=1, nthreads=1, model=None):
    """In-place: nsub mj_step's per env (fp64 oracle)."""
    m = model or load_model()
    L = _phys_lib()
    for k in STATE_KEYS:
        dt = np.uint32 if k == "warn" else np.float64
        if not (state[k].flags.c_contiguous and state[k].dtype == dt):
            state[k] = np.ascontiguousarray(state[k], dt)
    B = state["qpos"].shape[0]
    rc = L.orc_step_batch(_desc_ptr(m), *[_p(state[k]) for k in STATE_KEYS], B, int(nsub), int(nthreads))
    if rc:
        raise RuntimeError("orc_step_batch failed")
    return state


def set_boxbox_variant(bits=0):
    """Assumption probes of the box-box restatement (oracle/collision.c above box_box; 0 = the
    restatement itself).  Test infrastructure only: tools/badqacc_probe.py, tests/test_badqacc_probe_cpu.py."""
    _phys_lib().orc_set_boxbox_variant(int(bits))


def mpr_stats(reset=False):
    """MPR work counters since the last reset (oracle/convex.c g_mpr; diagnostics, single-threaded
    oracle calls only): runs, supports, discover / refine / penetration trips, capped runs, the
    largest support count of one run."""
    out = (C.c_longlong * 8)()
    _phys_lib().orc_mpr_stats(out, int(bool(reset)))
    keys = ("runs", "supports", "discover", "refine", "penetration", "capped", "max_supports_run")
    return dict(zip(keys, list(out)[:7]))


def forward_fields(state_row, fields, model=None, do_step=False):
    """One mj_forward (or mj_step) of one env; returns {field: array}."""
    m = model or load_model()
    L = _phys_lib()
    d = L.orc_data_new()
    try:
        arrs = [np.ascontiguousarray(state_row[k], np.float64) for k in STATE_KEYS[:6]]
        L.orc_set_state(_desc_ptr(m), d, *[_p(a) for a in arrs])
        (L.orc_step if do_step else L.orc_forward)(_desc_ptr(m), d)
        out = {}
        buf = np.zeros(200000)
        for f in fields:
            n = L.orc_field(_desc_ptr(m), d, f.encode(), _p(buf), buf.size)
            if n < 0:
                raise KeyError(f)
            out[f] = buf[:n].copy()
        return out
    finally:
        L.orc_data_free(d)


def convex_probe(state_row, g1, g2, model=None):
    """MPR (convex.c) on geoms g1, g2 after one forward at state_row: (dist, pos, normal) or None,
    plus the geom frames used: returns (hit, geom_xpos [ngeom,3], geom_xmat [ngeom,9])."""
    m = model or load_model()
    L = _phys_lib()
    d = L.orc_data_new()
    try:
        arrs = [np.ascontiguousarray(state_row[k], np.float64) for k in STATE_KEYS[:6]]
        L.orc_set_state(_desc_ptr(m), d, *[_p(a) for a in arrs])
        L.orc_forward(_desc_ptr(m), d)
        dist, pos, nrm = np.zeros(1), np.zeros(3), np.zeros(3)
        hit = L.orc_convex_probe(_desc_ptr(m), d, int(g1), int(g2), _p(dist), _p(pos), _p(nrm))
        buf = np.zeros(200000)
        n = L.orc_field(_desc_ptr(m), d, b"geom_xpos", _p(buf), buf.size)
        gx = buf[:n].reshape(-1, 3).copy()
        n = L.orc_field(_desc_ptr(m), d, b"geom_xmat", _p(buf), buf.size)
        gm = buf[:n].reshape(-1, 9).copy()
        return ((float(dist[0]), pos, nrm) if hit else None), gx, gm
    finally:
        L.orc_data_free(d)
