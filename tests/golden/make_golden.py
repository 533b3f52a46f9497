"""Generate tests/golden/ik_golden.npz by running the REFERENCE's own IK code.

Runs in the build container only (needs /root/reference; the GPU box never does this).
The reference's ``panda_mujoco_gym/skills/ik_solver.py`` is imported unmodified from
/root/reference with:
  * a stub ``mujoco`` module whose mj_forward / mj_kinematics / mj_jacSite are backed by the
    CPU oracle's kinematics (MuJoCo itself is absent: SURVEY.md §8c),
  * stub parent packages so that ``panda_mujoco_gym/__init__.py`` (which needs gymnasium,
    also absent) is not executed.
``JacobianIKController.solve`` (ik_solver.py:35-101) then runs exactly as written — DLS step via
numpy.linalg.solve, clamps, convergence/success logic — and its IKResult fields are recorded.
This pins the oracle's restatement of the solve loop against the reference code itself; the
kinematics it is fed are pinned separately by the home_wpt known answer.

Only the resulting arrays are committed; no reference source or bytecode is copied.
Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mujoco-panda-pnp_amd"))
REF = "/root/reference"

from oracle import oracle as O  # noqa: E402
from pnp_amd import workloads  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402


class _Site:
    def __init__(self, i):
        self.id = i


class StubModel:
    def __init__(self, m):
        self._m = m
        self.jnt_range = m.jnt_range.copy()
        self.nv = int(m.nv)
        self.nq = int(m.nq)

    def site(self, name):
        return _Site(self._m.site_id(name))


class StubData:
    def __init__(self, m):
        self.qpos = m.qpos0.copy()
        self.site_xpos = np.zeros((m.nsite, 3))


def _make_stub_mujoco(m):
    mj = types.ModuleType("mujoco")
    mj.MjModel = StubModel
    mj.MjData = StubData

    def _kin(model, data):
        sx, _ = O.site_kinematics(data.qpos[None], model=m)
        data.site_xpos[:] = sx[0]

    mj.mj_kinematics = _kin
    mj.mj_forward = _kin

    def mj_jacSite(model, data, jacp, jacr, site_id):
        J = O.jac_site(data.qpos[None], site=str(m.names_site[site_id]), model=m)[0]
        jacp[:] = J
        if jacr is not None:
            jacr[:] = 0.0

    mj.mj_jacSite = mj_jacSite
    return mj


def import_reference_ik(m):
    sys.modules["mujoco"] = _make_stub_mujoco(m)
    for name, sub in (("panda_mujoco_gym", ""), ("panda_mujoco_gym.skills", "skills")):
        pkg = types.ModuleType(name)
        pkg.__path__ = [os.path.join(REF, "panda_mujoco_gym", sub)]
        sys.modules[name] = pkg
    return importlib.import_module("panda_mujoco_gym.skills.ik_solver")


def main():
    m = load_model()
    ik_mod = import_reference_ik(m)
    site = m.site_id("ee_center_site")
    cases = []
    # 1) the reference's own IK test scenario (test/ik_test.py:26-37): neutral pose (the state
    #    after reset, panda_env.py:64-66) -> +0.1 m in x, pos_thresh 1e-4, damping 0.05
    neutral = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79])
    q = m.qpos0.copy()
    q[:7] = neutral
    p0 = O.site_kinematics(q[None], model=m)[0][0, site]
    cases.append(("ik_test", neutral, p0 + np.array([0.1, 0.0, 0.0]), workloads.IK_PARAMS["ik_test"]))
    # 2) the C2 bench distribution, both regimes x both parameter sets
    idx = np.arange(48)
    for regime in ("waypoint", "ik_test"):
        qi, delta = workloads.ik_inputs(m, idx, regime=regime)
        qfull = np.tile(m.qpos0, (len(idx), 1))
        qfull[:, :7] = qi
        p = O.site_kinematics(qfull, model=m)[0][:, site]
        for pname, prm in workloads.IK_PARAMS.items():
            for b in range(len(idx)):
                cases.append((f"{regime}/{pname}", qi[b], p[b] + delta[b], prm))
    # 3) edge cases: target = current position (0 iterations of update), unreachable target
    #    (hits the iteration cap, joints pinned at limits), q_init outside the limits
    cases.append(("edge/at_target", neutral, p0.copy(), workloads.IK_PARAMS["default"]))
    cases.append(("edge/unreachable", neutral, np.array([3.0, 0.0, 0.5]), workloads.IK_PARAMS["default"]))
    cases.append(("edge/max_iters_1", neutral, p0 + 0.05, dict(workloads.IK_PARAMS["default"], max_iters=1)))
    cases.append(("edge/max_iters_0", neutral, p0 + 0.05, dict(workloads.IK_PARAMS["default"], max_iters=0)))
    qbad = neutral.copy()
    qbad[3] = 0.3   # joint4 above its upper limit -0.0698
    cases.append(("edge/q_outside_limits", qbad, p0 + np.array([0.0, 0.05, 0.0]), workloads.IK_PARAMS["default"]))

    rows = {k: [] for k in ("q_init", "target", "max_iters", "pos_thresh", "damping", "step_limit",
                            "q", "final_pos", "pos_error", "iterations", "success", "converged")}
    tags = []
    for tag, qi, tgt, prm in cases:
        data = sys.modules["mujoco"].MjData(m)
        ctl = ik_mod.JacobianIKController(sys.modules["mujoco"].MjModel(m), data)
        res = ctl.solve(np.array(tgt, float), np.array(qi, float), **prm)
        tags.append(tag)
        rows["q_init"].append(qi)
        rows["target"].append(tgt)
        for k in ("max_iters", "pos_thresh", "damping", "step_limit"):
            rows[k].append(prm[k])
        rows["q"].append(res.q)
        rows["final_pos"].append(res.final_pos)
        rows["pos_error"].append(res.pos_error)
        rows["iterations"].append(res.iterations)
        rows["success"].append(bool(res.success))
        rows["converged"].append(bool(res.converged))
    out = {k: np.array(v) for k, v in rows.items()}
    out["tag"] = np.array(tags)
    out["max_iters"] = out["max_iters"].astype(np.int32)
    out["iterations"] = out["iterations"].astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "ik_golden.npz"), **out)
    print(f"wrote {len(tags)} reference IK solves; converged {int(out['converged'].sum())}, "
          f"success {int(out['success'].sum())}, mean iters {out['iterations'].mean():.1f}")


if __name__ == "__main__":
    main()
