"""Compiled Panda shelf model: numpy arrays + the ``pnp_model_desc`` C struct (include/pnp.h).

The arrays come from ``data/panda_shelf.npz`` (written by :mod:`pnp_amd.mjcf` from the
reference MJCF, reference ``envs/panda_env.py:108``).  Field names follow MjModel so that code
written against ``env.unwrapped.model`` (reference ``skills/ik_solver.py:30-33``,
``envs/panda_env.py:89-92``) reads the same here.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

DATA_PATH = os.path.join(os.path.dirname(__file__), "data", "panda_shelf.npz")

_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)

# (name, kind) in include/pnp.h order; kind: "i" int32 scalar, "d" double scalar, "g" double[3],
# "I" int32 array, "D" double array.
_DESC_FIELDS = [
    ("nq", "i"), ("nv", "i"), ("nu", "i"), ("nbody", "i"), ("njnt", "i"), ("ngeom", "i"),
    ("nsite", "i"), ("nmocap", "i"), ("neq", "i"), ("nmesh", "i"), ("nmeshvert", "i"),
    ("timestep", "d"), ("gravity", "g"), ("noslip_iterations", "i"), ("iterations", "i"),
    ("tolerance", "d"), ("cone_pyramidal", "i"), ("multiccd", "i"), ("warmstart", "i"),
    ("integrator_euler", "i"), ("noslip_tolerance", "d"), ("stat_meaninertia", "d"),
    ("body_parentid", "I"), ("body_rootid", "I"), ("body_weldid", "I"), ("body_mocapid", "I"),
    ("body_jntadr", "I"), ("body_jntnum", "I"), ("body_dofadr", "I"), ("body_dofnum", "I"),
    ("body_pos", "D"), ("body_quat", "D"), ("body_ipos", "D"), ("body_iquat", "D"),
    ("body_mass", "D"), ("body_inertia", "D"), ("body_invweight0", "D"), ("body_subtreemass", "D"),
    ("body_treedepth", "I"),
    ("jnt_type", "I"), ("jnt_qposadr", "I"), ("jnt_dofadr", "I"), ("jnt_bodyid", "I"),
    ("jnt_limited", "I"), ("jnt_pos", "D"), ("jnt_axis", "D"), ("jnt_range", "D"),
    ("jnt_solref", "D"), ("jnt_solimp", "D"), ("jnt_margin", "D"),
    ("dof_jntid", "I"), ("dof_bodyid", "I"), ("dof_armature", "D"), ("dof_damping", "D"),
    ("dof_parentid", "I"), ("dof_invweight0", "D"),
    ("qpos0", "D"),
    ("geom_type", "I"), ("geom_bodyid", "I"), ("geom_contype", "I"), ("geom_conaffinity", "I"),
    ("geom_condim", "I"), ("geom_priority", "I"), ("geom_dataid", "I"), ("geom_size", "D"),
    ("geom_pos", "D"), ("geom_quat", "D"), ("geom_friction", "D"), ("geom_solref", "D"),
    ("geom_solimp", "D"), ("geom_margin", "D"), ("geom_gap", "D"), ("geom_solmix", "D"),
    ("geom_rbound", "D"),
    ("mesh_vertadr", "I"), ("mesh_vertnum", "I"), ("mesh_vert", "D"),
    ("site_bodyid", "I"), ("site_pos", "D"), ("site_quat", "D"),
    ("actuator_trnid", "I"), ("actuator_biastype", "I"), ("actuator_ctrllimited", "I"),
    ("actuator_forcelimited", "I"), ("actuator_gear", "D"), ("actuator_gainprm", "D"),
    ("actuator_biasprm", "D"), ("actuator_ctrlrange", "D"), ("actuator_forcerange", "D"),
    ("eq_type", "I"), ("eq_obj1id", "I"), ("eq_obj2id", "I"), ("eq_solref", "D"),
    ("eq_solimp", "D"), ("eq_data", "D"),
]

_CT = {"i": C.c_int32, "d": C.c_double, "g": C.c_double * 3, "I": _i32p, "D": _f64p}


class PnpModelDesc(C.Structure):
    _fields_ = [(n, _CT[k]) for n, k in _DESC_FIELDS]


class PnpIKParams(C.Structure):
    _fields_ = [("max_iters", C.c_int32), ("pos_thresh", C.c_double), ("damping", C.c_double),
                ("step_limit", C.c_double)]


# scalar renames between the npz (opt_*) and the C struct
_SCALAR_SRC = {"timestep": "opt_timestep", "gravity": "opt_gravity",
               "noslip_iterations": "opt_noslip_iterations", "iterations": "opt_iterations",
               "tolerance": "opt_tolerance", "cone_pyramidal": "opt_cone_pyramidal",
               "multiccd": "opt_multiccd", "warmstart": "opt_warmstart",
               "integrator_euler": "opt_integrator_euler", "noslip_tolerance": "opt_noslip_tolerance"}


class PandaModel:
    """MjModel-like view of the compiled scene (numpy, float64 / int32)."""

    def __init__(self, path: str = DATA_PATH):
        z = np.load(path, allow_pickle=False)
        self._arrays = {k: z[k] for k in z.files}
        for k, v in self._arrays.items():
            setattr(self, k, v if v.ndim else v.item())
        self.nmeshvert = int(self.mesh_vert.shape[0])
        self._desc = None
        self._keep = []

    # ---- name lookups (mujoco.MjModel.site(name).id etc.)
    def _id(self, names, name):
        idx = np.nonzero(names == name)[0]
        if idx.size != 1:
            raise KeyError(name)
        return int(idx[0])

    def site_id(self, name):
        return self._id(self.names_site, name)

    def body_id(self, name):
        return self._id(self.names_body, name)

    def joint_id(self, name):
        return self._id(self.names_jnt, name)

    def geom_id(self, name):
        return self._id(self.names_geom, name)

    # ---- C descriptor
    def desc(self) -> PnpModelDesc:
        if self._desc is not None:
            return self._desc
        d = PnpModelDesc()
        for name, kind in _DESC_FIELDS:
            src = _SCALAR_SRC.get(name, name)
            if kind == "i":
                setattr(d, name, int(getattr(self, src)))
            elif kind == "d":
                setattr(d, name, float(getattr(self, src)))
            elif kind == "g":
                setattr(d, name, (C.c_double * 3)(*[float(x) for x in getattr(self, src)]))
            else:
                dt = np.int32 if kind == "I" else np.float64
                a = np.ascontiguousarray(getattr(self, src), dtype=dt).ravel()
                if a.size == 0:
                    a = np.zeros(1, dt)
                self._keep.append(a)
                setattr(d, name, a.ctypes.data_as(_i32p if kind == "I" else _f64p))
        self._desc = d
        return d

    # ---- reference constants used by the env layer
    @property
    def arm_lower(self):
        return self.jnt_range[:7, 0].copy()

    @property
    def arm_upper(self):
        return self.jnt_range[:7, 1].copy()


_MODEL = None


def load_model() -> PandaModel:
    global _MODEL
    if _MODEL is None:
        _MODEL = PandaModel()
    return _MODEL
