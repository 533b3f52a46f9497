"""Scene states for the physics parity tests (test helper; generated with the CPU oracle).

``settled_states`` reproduces the reference's reset path: ``_env_setup`` (neutral arm, arm servo
targets = neutral, mocap at the ee_center_site pose; envs/panda_env.py:124-141) then
``_sample_object`` (cube xy + U(+-0.02, +-0.2) around the XML sites; shelf_pnp.py:23-24,
panda_env.py:146-158), then ``nsettle`` sub-steps of the oracle.  ``random_ctrl`` draws the
BASELINE C3 per-step control, U(actuator_ctrlrange).
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from pnp_amd.workloads import NEUTRAL  # noqa: F401  (re-exported for the tests)


def reset_states(B, seed=0, model=None):
    m = model or O.load_model()
    rng = np.random.default_rng(seed)
    st = O.new_state(B, model=m)
    st["qpos"][:, :9] = NEUTRAL
    st["ctrl"][:, :7] = NEUTRAL[:7]
    sx, sm = O.site_kinematics(st["qpos"], model=m)
    s = m.site_id("ee_center_site")
    st["mocap_pos"][:] = sx[:, s]
    q = O.mat2quat(sm[0, s])
    st["mocap_quat"][:] = q
    for name in ("cube1", "cube2", "cube3"):
        a = int(m.jnt_qposadr[m.joint_id(f"{name}_joint")])
        c = sx[0, m.site_id(f"{name}_site")]
        st["qpos"][:, a] = c[0] + rng.uniform(-0.02, 0.02, B)
        st["qpos"][:, a + 1] = c[1] + rng.uniform(-0.2, 0.2, B)
        st["qpos"][:, a + 2] = c[2]
        st["qpos"][:, a + 3:a + 7] = [1, 0, 0, 0]
    return st


def settled_states(B, seed=0, nsettle=250, nthreads=8, model=None):
    st = reset_states(B, seed, model)
    if nsettle:
        O.step(st, nsub=nsettle, nthreads=nthreads, model=model)
    return st


def random_ctrl(st, seed=1, model=None):
    m = model or O.load_model()
    rng = np.random.default_rng(seed)
    lo, hi = m.actuator_ctrlrange[:, 0], m.actuator_ctrlrange[:, 1]
    st["ctrl"][:] = rng.uniform(lo, hi, size=st["ctrl"].shape)
    return st


def copy_state(st):
    return {k: v.copy() for k, v in st.items()}
