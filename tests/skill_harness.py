"""Shared pieces of the skill tests: the episode script of tests/golden/make_skill_golden.py run
with OUR skills (pnp_amd.skills), an oracle-backed env with the facade's surface (CPU tests), an
oracle-backed IK controller, and the golden comparison.

Test infrastructure only (imports oracle/); the product facade is pnp_amd.envs.FrankaShelfPNPEnv.
"""
from __future__ import annotations

import os
import types

import numpy as np

from oracle import oracle as O
from oracle.env_oracle import EnvConfig, EnvOracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "skill_golden.npz")
FIELDS = ("action", "done", "mocap_pos", "mocap_quat", "qpos", "ee_pos", "ee_quat")


def load_golden():
    return np.load(GOLDEN)


# ------------------------------------------------------------------------- oracle-backed facade
class _OracleData:
    """data.* views over EnvOracle row 0 (qpos_kin = the last forward's qpos)."""

    def __init__(self, e):
        self._e = e

    qpos = property(lambda self: self._e.st["qpos"][0])
    qvel = property(lambda self: self._e.st["qvel"][0])
    ctrl = property(lambda self: self._e.st["ctrl"][0])
    mocap_pos = property(lambda self: self._e.st["mocap_pos"][0:1])
    mocap_quat = property(lambda self: self._e.st["mocap_quat"][0:1])

    def __deepcopy__(self, memo):
        return types.SimpleNamespace(qpos=self.qpos.copy(), qvel=self.qvel.copy())


class _OracleMujoco:
    def __init__(self, e):
        self._e = e

    def mj_step(self, model, data, nstep=1):
        e = self._e
        st = e.st
        O.step(st, nsub=nstep - 1, model=e.m)
        qk = st["qpos"][0].copy()
        w0 = int(st["warn"][0])
        O.step(st, nsub=1, model=e.m)
        if (int(st["warn"][0]) & 7) & ~(w0 & 7):
            qk = e.m.qpos0.copy()
        e.qpos_kin[0] = qk


class OracleFacadeEnv:
    """The facade surface the skills use, over the fp64 env oracle (B = 1, env index 0)."""

    def __init__(self, model, n_substeps):
        self.e = EnvOracle(1, cfg=EnvConfig(n_substeps=n_substeps, n_calls=10), model=model)
        self.e.reset()
        self.model = model
        self.data = _OracleData(self.e)
        self._mujoco = _OracleMujoco(self.e)
        self.render_mode = None
        self.action_space = types.SimpleNamespace(low=-np.ones(7, np.float32), high=np.ones(7, np.float32))

    @property
    def unwrapped(self):
        return self

    def get_ee_position(self):
        sx, _, _, _ = self.e._frames(0, self.e.ee)
        return sx[self.e.ee].copy()

    def get_ee_orientation(self):
        _, sm, _, _ = self.e._frames(0, self.e.ee)
        return O.mat2quat(sm[self.e.ee])

    def set_mocap_pose(self, pos, quat):
        self.e.st["mocap_pos"][0] = pos
        self.e.st["mocap_quat"][0] = quat

    def step(self, action):
        r = self.e.step(np.asarray(action)[None])[0]
        return r["obs"], np.float32(r["reward"]), r["terminated"], r["truncated"], {"is_success": r["is_success"]}


class OracleIK:
    """JacobianIKController stand-in over the oracle's DLS (oracle/oracle.c): same solve()."""

    def __init__(self, model, data=None, site_name="ee_center_site"):
        self.model, self.data, self.site = model, data, site_name

    def solve(self, target_pos, q_init, max_iters=100, pos_thresh=1e-3, damping=1e-2, step_limit=0.1):
        from pnp_amd.ik_solver import IKResult
        r = O.ik_dls(np.asarray(q_init)[None], np.asarray(target_pos)[None], site=self.site, model=self.model,
                     max_iters=max_iters, pos_thresh=pos_thresh, damping=damping, step_limit=step_limit)
        fl = int(r["flags"][0])
        if self.data is not None:
            self.data.qpos[:7] = r["q"][0]
        return IKResult(success=bool(fl & 2), q=r["q"][0].copy(), final_pos=r["final_pos"][0].copy(),
                        pos_error=float(r["pos_error"][0]), iterations=int(r["iterations"][0]),
                        converged=bool(fl & 1))


# ------------------------------------------------------------------------- the episode
def _run(skill, env, rec, cap=60):
    skill.reset()
    n = 0
    while not skill.is_done() and n < cap:
        a = skill.step()
        rec["action"].append(np.asarray(a, np.float64))
        rec["done"].append(bool(skill.is_done()))
        rec["mocap_pos"].append(np.asarray(env.data.mocap_pos, np.float64).reshape(-1)[:3].copy())
        rec["mocap_quat"].append(np.asarray(env.data.mocap_quat, np.float64).reshape(-1)[:4].copy())
        rec["qpos"].append(np.asarray(env.data.qpos, np.float64).copy())
        rec["ee_pos"].append(np.asarray(env.get_ee_position(), np.float64).copy())
        rec["ee_quat"].append(np.asarray(env.get_ee_orientation(), np.float64).copy())
        n += 1
    return n


def run_episode(env, G):
    """make_skill_golden.py's script with pnp_amd.skills, targets taken from the golden file."""
    from pnp_amd.skills import GripperSkill, MoveIKSkill, MoveSkill, RotateSkill
    rec = {k: [] for k in FIELDS}
    ticks = [_run(MoveSkill(env, G["move_target"]), env, rec),
             _run(RotateSkill(env, G["rot_delta"], steps=8), env, rec),
             _run(GripperSkill.close(env, duration=2), env, rec)]
    mik = MoveIKSkill(env, G["moveik_target"])
    ticks.append(_run(mik, env, rec))
    ticks.append(_run(GripperSkill.open(env, duration=2), env, rec))
    out = {k: np.array(v) for k, v in rec.items()}
    out["ticks"] = np.array(ticks)
    out["moveik_traj"] = np.array(mik.pos_traj)
    return out


def compare(out, G, tol):
    """Per-skill tick counts and done flags exactly; every recorded array within tol."""
    np.testing.assert_array_equal(out["ticks"], G["ticks"])
    np.testing.assert_array_equal(out["done"], G["done"])
    worst = {}
    for k in FIELDS + ("moveik_traj",):
        if k == "done":
            continue
        assert out[k].shape == G[k].shape, (k, out[k].shape, G[k].shape)
        err = float(np.abs(out[k] - G[k]).max())
        worst[k] = err
        assert err <= tol, f"{k}: max |diff| {err:.3e} > {tol:.1e}"
    return worst
