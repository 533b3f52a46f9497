"""ctypes binding of libpnp.so (include/pnp.h).  Fails loudly if the HIP library is missing:
there is no CPU fallback anywhere in the product path."""
from __future__ import annotations

import ctypes as C
import os

from .model import PnpIKParams, PnpModelDesc

# PNP_LIB: another build of the same sources (tools/asan_cpu_tests.sh: the host-sanitizer build)
LIB_PATH = os.environ.get("PNP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpnp.so")
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
ABI_VERSION = 14

# every symbol include/pnp.h declares (tests check the library exports all of them)
EXPORTS = [
    "pnp_abi_version", "pnp_model_desc_size", "pnp_last_error", "pnp_model_create",
    "pnp_model_destroy", "pnp_model_check", "pnp_site_kinematics", "pnp_site_kinematics_f64", "pnp_jac_site",
    "pnp_jac_site_f64", "pnp_jac_site_full", "pnp_jac_site_full_f64", "pnp_ik_dls", "pnp_ik_dls_f64", "pnp_step", "pnp_step_f64",
    "pnp_forward_debug", "pnp_forward_debug_f64", "pnp_step_lds_bytes", "pnp_step_profile",
    "pnp_env_params_size", "pnp_env_init", "pnp_env_init_f64", "pnp_env_reset", "pnp_env_reset_f64",
    "pnp_env_step", "pnp_env_step_f64", "pnp_env_evaluate", "pnp_env_evaluate_f64",
    "pnp_slerp_track_f64", "pnp_env_queue_status", "pnp_tqc_workspace_floats", "pnp_tqc_param_counts",
    "pnp_tqc_update", "pnp_tqc_update_phase", "pnp_tqc_sample", "pnp_tqc_sample_draw",
]

STATE_FIELDS = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart", "time", "warn")


class PnpState(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in STATE_FIELDS]


MAX_TASKS = 4
OBS_DIM = 19


class PnpEnvParams(C.Structure):
    """include/pnp.h pnp_env_params."""
    _fields_ = [("n_substeps", C.c_int32), ("n_calls", C.c_int32), ("reward_dense", C.c_int32),
                ("max_episode_steps", C.c_int32), ("n_tasks", C.c_int32), ("ee_site", C.c_int32),
                ("obj_site", C.c_int32 * MAX_TASKS), ("target_site", C.c_int32 * MAX_TASKS),
                ("obj_qadr", C.c_int32 * MAX_TASKS), ("finger_qadr", C.c_int32 * 2),
                ("neutral_qadr", C.c_int32 * 9), ("height_qadr", C.c_int32), ("arm_ctrl_n", C.c_int32),
                ("neutral", C.c_double * 9), ("distance_threshold", C.c_double), ("high_pick_z", C.c_double),
                ("grip_width", C.c_double), ("reach_thresh", C.c_double), ("lift_height", C.c_double),
                ("obj_x_range", C.c_double), ("obj_y_range", C.c_double), ("pos_scale", C.c_double),
                ("rot_scale", C.c_double), ("finger_scale", C.c_double), ("seed_lo", C.c_uint32),
                ("seed_hi", C.c_uint32)]


ENV_STATE_FIELDS = ("goal", "task", "elapsed", "qpos_kin", "obj_height0", "init_mocap", "init_qvel", "init_time",
                    "episode", "env_index", "tier")
ENV_OUT_FIELDS = ("obs", "achieved_goal", "desired_goal", "reward", "is_success", "terminated", "truncated")


class PnpEnvState(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in ENV_STATE_FIELDS]


class PnpEnvOut(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in ENV_OUT_FIELDS]


_F = C.POINTER(C.c_float)


class PnpTqcDesc(C.Structure):
    """include/pnp.h pnp_tqc_desc."""
    _fields_ = [("batch", C.c_int32), ("obs_dim", C.c_int32), ("act_dim", C.c_int32), ("hidden", C.c_int32),
                ("n_critics", C.c_int32), ("n_quantiles", C.c_int32), ("n_drop_per_net", C.c_int32),
                ("gamma", C.c_float), ("tau", C.c_float), ("target_entropy", C.c_float), ("beta1", C.c_float),
                ("beta2", C.c_float), ("adam_eps", C.c_float),
                ("actor", C.c_void_p * 10), ("actor_m", C.c_void_p * 10), ("actor_v", C.c_void_p * 10),
                ("actor_step", C.c_void_p * 10),
                ("critic", C.c_void_p * 8), ("critic_m", C.c_void_p * 8), ("critic_v", C.c_void_p * 8),
                ("critic_step", C.c_void_p * 8), ("target", C.c_void_p * 8),
                ("log_ent_coef", C.c_void_p), ("ent_m", C.c_void_p), ("ent_v", C.c_void_p), ("ent_step", C.c_void_p),
                ("lr", C.c_void_p), ("workspace", C.c_void_p), ("workspace_floats", C.c_int64), ("logs", C.c_void_p),
                ("draw_counter", C.c_void_p)]


class PnpTqcBatch(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in ("obs", "act", "next_obs", "done", "reward", "eps_pi", "eps_next")]


class PnpTqcReplay(C.Structure):
    """include/pnp.h pnp_tqc_replay."""
    _fields_ = [(f, C.c_void_p) for f in ("obs", "next_obs", "actions", "rewards", "dones", "upper")] + \
               [("rows", C.c_int32), ("n_envs", C.c_int32), ("obs_dim", C.c_int32), ("act_dim", C.c_int32),
                ("n_keys", C.c_int32), ("key_dim", C.c_int32 * 4), ("mean", C.c_void_p * 4), ("var", C.c_void_p * 4),
                ("clip_obs", C.c_double), ("norm_eps", C.c_double)]


# debug record layout (include/pnp.h PNP_DBG_*)
DBG = dict(QM=0, BIAS=1296, ACT=1332, QACC_SMOOTH=1368, QACC=1404, COUNTS=1440, CON=1444, CON_STRIDE=16,
           EFC_FORCE=4516, EFC_POS=5300, EFC_D=6084, EFC_AREF=6868, EFC_TYPE=7652, EFC_J=8436,
           QACC_NEWTON=36660, NOSLIP_ITER=36696, SIZE=36700, MAXCON=192, MAXEFC=784)

_lib = None


class PnpError(RuntimeError):
    pass


def load():
    """Load libpnp.so (build it with `make -C mujoco-panda-pnp_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PnpError(f"libpnp.so not found at {LIB_PATH}; build the HIP extension first "
                       f"(make -C {CSRC} or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, I32 = C.c_void_p, C.c_int32
    L.pnp_abi_version.restype = I32
    L.pnp_model_desc_size.restype = I32
    L.pnp_last_error.restype = C.c_char_p
    L.pnp_model_create.argtypes = [C.POINTER(PnpModelDesc), C.POINTER(P)]
    L.pnp_model_create.restype = I32
    L.pnp_model_check.argtypes = [C.POINTER(PnpModelDesc)]
    L.pnp_model_check.restype = I32
    L.pnp_model_destroy.argtypes = [P]
    L.pnp_model_destroy.restype = I32
    for name in ("pnp_site_kinematics", "pnp_site_kinematics_f64"):
        f = getattr(L, name)
        f.argtypes = [P, P, P, P, P, P, I32, P]
        f.restype = I32
    for name in ("pnp_jac_site", "pnp_jac_site_f64"):
        f = getattr(L, name)
        f.argtypes = [P, I32, P, P, I32, P]
        f.restype = I32
    for name in ("pnp_jac_site_full", "pnp_jac_site_full_f64"):
        f = getattr(L, name)
        f.argtypes = [P, I32, P, P, P, P, P, I32, P]
        f.restype = I32
    for name in ("pnp_ik_dls", "pnp_ik_dls_f64"):
        f = getattr(L, name)
        f.argtypes = [P, I32, PnpIKParams, P, P, P, P, P, P, P, I32, P]
        f.restype = I32
    for name in ("pnp_step", "pnp_step_f64"):
        f = getattr(L, name)
        f.argtypes = [P, C.POINTER(PnpState), I32, I32, P]
        f.restype = I32
    for name in ("pnp_forward_debug", "pnp_forward_debug_f64"):
        f = getattr(L, name)
        f.argtypes = [P, C.POINTER(PnpState), I32, P, P]
        f.restype = I32
    L.pnp_step_profile.argtypes = [P, C.POINTER(PnpState), I32, I32, P, P]
    L.pnp_step_profile.restype = I32
    L.pnp_step_lds_bytes.argtypes = [I32]
    L.pnp_step_lds_bytes.restype = I32
    L.pnp_env_params_size.restype = I32
    SP, EP, ES, EO = C.POINTER(PnpState), C.POINTER(PnpEnvParams), C.POINTER(PnpEnvState), C.POINTER(PnpEnvOut)
    for name in ("pnp_env_init", "pnp_env_init_f64"):
        f = getattr(L, name)
        f.argtypes = [P, SP, EP, ES, I32, P]
        f.restype = I32
    for name in ("pnp_env_reset", "pnp_env_reset_f64"):
        f = getattr(L, name)
        f.argtypes = [P, SP, EP, ES, P, EO, I32, P]
        f.restype = I32
    for name in ("pnp_env_step", "pnp_env_step_f64"):
        f = getattr(L, name)
        f.argtypes = [P, SP, EP, ES, P, EO, I32, P]
        f.restype = I32
    for name in ("pnp_env_evaluate", "pnp_env_evaluate_f64"):
        f = getattr(L, name)
        f.argtypes = [P, SP, EP, ES, P, P, EO, I32, P]
        f.restype = I32
    L.pnp_slerp_track_f64.argtypes = [P, P, I32, P, P, I32, P]
    L.pnp_slerp_track_f64.restype = I32
    L.pnp_env_queue_status.argtypes = [P]
    L.pnp_env_queue_status.restype = I32
    L.pnp_tqc_workspace_floats.argtypes = [C.POINTER(PnpTqcDesc)]
    L.pnp_tqc_workspace_floats.restype = C.c_int64
    L.pnp_tqc_param_counts.argtypes = [P, P]
    L.pnp_tqc_param_counts.restype = I32
    L.pnp_tqc_update.argtypes = [C.POINTER(PnpTqcDesc), C.POINTER(PnpTqcBatch), P, P]
    L.pnp_tqc_update.restype = I32
    L.pnp_tqc_update_phase.argtypes = [C.POINTER(PnpTqcDesc), C.POINTER(PnpTqcBatch), P, I32, P]
    L.pnp_tqc_update_phase.restype = I32
    L.pnp_tqc_sample.argtypes = [C.POINTER(PnpTqcReplay), P, I32, P, P, P, P, P, P]
    L.pnp_tqc_sample.restype = I32
    L.pnp_tqc_sample_draw.argtypes = [C.POINTER(PnpTqcReplay), C.c_uint64, P, I32, P, P, P, P, P, P, P, P, P]
    L.pnp_tqc_sample_draw.restype = I32
    if L.pnp_abi_version() != ABI_VERSION:
        raise PnpError(f"libpnp ABI {L.pnp_abi_version()} != binding ABI {ABI_VERSION}")
    if L.pnp_env_params_size() != C.sizeof(PnpEnvParams):
        raise PnpError(f"pnp_env_params size mismatch: lib {L.pnp_env_params_size()} vs "
                       f"binding {C.sizeof(PnpEnvParams)}")
    if L.pnp_model_desc_size() != C.sizeof(PnpModelDesc):
        raise PnpError(f"pnp_model_desc size mismatch: lib {L.pnp_model_desc_size()} vs "
                       f"binding {C.sizeof(PnpModelDesc)}")
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = load().pnp_last_error().decode(errors="replace")
        raise PnpError(f"{what} failed ({rc}): {msg}")


def env_queue_status():
    """pnp_env_queue_status: the hand-over queue's counts after the last routed fp32 gym step on
    the current device (synchronises): published, producers_done, claims, timeouts, fallback."""
    L = load()
    buf = (C.c_int32 * 5)()
    check(L.pnp_env_queue_status(buf), "pnp_env_queue_status")
    return dict(zip(("published", "producers_done", "claims", "timeouts", "fallback"), list(buf)))
