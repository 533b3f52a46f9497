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


# the full tier's contact capacity (mujoco-panda-pnp_amd/csrc/phys_model.h PH_MAXCON): the fixtures
# that exercise the wide tier must pass it
FULL_MAXCON = 64

PILE_XY = (1.371, 0.48)   # on board2 (shelf_pnp.xml:51, top at z 0.71)


def cube_pile(qpos, model, rows=slice(None)):
    """Pile the three cubes on board2 for the given rows of a qpos batch: cube2 0.6 mm into cube1's
    top, cube3 0.4 mm into cube1's side, cube1 0.2 mm into the board (box-box contacts, 4-8 each).
    With the closed-finger pads pressed 1-4 mm together (52-63 contacts) that makes 76-87: past the
    full tier's capacity, so the wide tier finishes those sub-steps."""
    m = model
    top, h = 0.71, 0.02
    x, y = PILE_XY
    poses = {"cube1": [x, y, top + h - 2e-4], "cube2": [x + 0.005, y, top + 3 * h - 6e-4],
             "cube3": [x + 2 * h - 4e-4, y + 0.01, top + h - 2e-4]}
    for name, p in poses.items():
        a = int(m.jnt_qposadr[m.joint_id(f"{name}_joint")])
        v = np.array(p + [1.0, 0.0, 0.0, 0.0])
        if not isinstance(qpos, np.ndarray):   # a device tensor (the gym tests)
            import torch
            v = torch.as_tensor(v, dtype=qpos.dtype, device=qpos.device)
        qpos[rows, a:a + 7] = v
    return qpos


def copy_state(st):
    return {k: v.copy() for k, v in st.items()}
