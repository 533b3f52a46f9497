"""Generate tests/golden/skill_golden.npz by running the REFERENCE's own skills.

Runs in the build container only (needs /root/reference; the GPU box never does this).
``panda_mujoco_gym/skills/{base,move,rotate,gripper,ik_solver}.py`` are imported unmodified from
/root/reference and driven against the reference's own ``FrankaEnv`` built exactly as in
make_env_golden.py (stub ``mujoco`` / gymnasium-robotics backed by the CPU oracle, n_substeps = 1),
with the stub extended by what the skills and the IK controller need: ``mj_kinematics``,
``mj_jacSite``, ``data.site_xpos``, ``model.site(name).id``, ``model.jnt_range`` and a
deep-copyable ``data`` (skills/move.py:83-84).

One episode (env 0, dense): MoveSkill -> RotateSkill -> GripperSkill.close -> MoveIKSkill ->
GripperSkill.open, each run to done (or a tick cap).  Recorded per tick: the returned action, the
done flag, mocap pose, qpos, ee position / orientation; plus MoveIKSkill's planned waypoints and
the targets / deltas used.  Only the resulting arrays are committed.
Usage: python tests/golden/make_skill_golden.py
"""
from __future__ import annotations

import copy
import importlib
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_env_golden as EG  # noqa: E402

O = EG.O
REF = EG.REF

# the episode script (targets relative to the ee position at the start of each skill)
MOVE_OFFSET = np.array([0.06, 0.04, -0.05])
ROT_EULER_Z = np.deg2rad(25.0)
ROT_STEPS = 8
MOVEIK_OFFSET = np.array([-0.05, -0.03, 0.04])
GRIP_TICKS = 2
TICK_CAP = 60


class _Site:
    def __init__(self, i):
        self.id = i


class SkillStubModel(EG.StubModel):
    def __init__(self, m):
        super().__init__(m)
        self.jnt_range = m.jnt_range.copy()
        self.nv, self.nq = int(m.nv), int(m.nq)

    def site(self, name):
        return _Site(self._m.site_id(name))


class SkillStubData(EG.StubData):
    """StubData that deep-copies and exposes site_xpos (the last forward's frames)."""

    def __getattr__(self, k):
        d = self.__dict__
        if "st" not in d:
            raise AttributeError(k)
        if k == "site_xpos":
            m = d["_m"]
            st = d["st"]
            sx, _ = O.site_kinematics(d["qpos_kin"][None], st["mocap_pos"], st["mocap_quat"], model=m)
            return sx[0]
        return super().__getattr__(k)

    def __setattr__(self, k, v):
        if k == "_m":
            object.__setattr__(self, k, v)
        else:
            super().__setattr__(k, v)

    def __deepcopy__(self, memo):
        new = SkillStubData.__new__(SkillStubData)
        object.__setattr__(new, "_m", self.__dict__["_m"])
        object.__setattr__(new, "st", copy.deepcopy(self.__dict__["st"], memo))
        object.__setattr__(new, "qpos_kin", self.__dict__["qpos_kin"].copy())
        return new


def extend_stub_mujoco(mj, m):
    def mj_kinematics(model, data):
        data.qpos_kin = data.st["qpos"][0].copy()

    def mj_jacSite(model, data, jacp, jacr, site_id):
        st = data.st
        _, _, jp, jr = O.site_jac2(data.qpos_kin[None], str(m.names_site[site_id]), st["mocap_pos"],
                                   st["mocap_quat"], model=m)
        if jacp is not None:
            jacp[...] = jp[0].reshape(np.shape(jacp))
        if jacr is not None:
            jacr[...] = jr[0].reshape(np.shape(jacr))

    mj.mj_kinematics, mj.mj_jacSite = mj_kinematics, mj_jacSite
    mj.MjModel, mj.MjData = SkillStubModel, SkillStubData


def import_reference_skills():
    pkg = types.ModuleType("panda_mujoco_gym.skills")
    pkg.__path__ = [os.path.join(REF, "panda_mujoco_gym", "skills")]
    sys.modules["panda_mujoco_gym.skills"] = pkg
    return {n: importlib.import_module(f"panda_mujoco_gym.skills.{n}") for n in ("base", "move", "rotate", "gripper")}


def make_env(mod, mj, ut, m):
    EG.StubRobotEnv.unwrapped = property(lambda self: self)
    env = EG.new_env(mod, mj, ut, m, "dense")
    st = env.data.st
    data = SkillStubData.__new__(SkillStubData)
    object.__setattr__(data, "_m", m)
    object.__setattr__(data, "st", st)
    object.__setattr__(data, "qpos_kin", env.data.qpos_kin)
    env.data = data
    env.model = SkillStubModel(m)
    real_uniform = np.random.uniform
    np.random.uniform = EG.philox_reset(0, 0, 6)
    try:
        env._reset_sim()
    finally:
        np.random.uniform = real_uniform
    env.goal = env._sample_goal().copy()
    return env


def run_skill(skill, env, rec, cap=TICK_CAP):
    skill.reset()
    n = 0
    while not skill.is_done() and n < cap:
        a = skill.step()
        st = env.data.st
        rec["action"].append(np.asarray(a, np.float64))
        rec["done"].append(bool(skill.is_done()))
        rec["mocap_pos"].append(st["mocap_pos"][0].copy())
        rec["mocap_quat"].append(st["mocap_quat"][0].copy())
        rec["qpos"].append(st["qpos"][0].copy())
        rec["ee_pos"].append(np.asarray(env.get_ee_position(), np.float64).copy())
        rec["ee_quat"].append(np.asarray(env.get_ee_orientation(), np.float64).copy())
        n += 1
    return n


def main():
    m = EG.load_model()
    mod, mj, ut = EG.import_reference_env(m)
    extend_stub_mujoco(mj, m)
    S = import_reference_skills()
    from scipy.spatial.transform import Rotation
    env = make_env(mod, mj, ut, m)
    rec = {k: [] for k in ("action", "done", "mocap_pos", "mocap_quat", "qpos", "ee_pos", "ee_quat")}
    ticks, meta = [], {}
    ee0 = env.get_ee_position().copy()
    meta["reset_qpos"] = env.data.st["qpos"][0].copy()
    meta["move_target"] = ee0 + MOVE_OFFSET
    ticks.append(run_skill(S["move"].MoveSkill(env, meta["move_target"]), env, rec))
    meta["rot_delta"] = Rotation.from_euler("z", ROT_EULER_Z).as_quat()
    ticks.append(run_skill(S["rotate"].RotateSkill(env, meta["rot_delta"], steps=ROT_STEPS), env, rec))
    ticks.append(run_skill(S["gripper"].GripperSkill.close(env, duration=GRIP_TICKS), env, rec))
    meta["moveik_target"] = env.get_ee_position().copy() + MOVEIK_OFFSET
    mik = S["move"].MoveIKSkill(env, meta["moveik_target"])
    meta["moveik_start_qpos"] = env.data.st["qpos"][0].copy()
    meta["moveik_start_ee"] = env.get_ee_position().copy()
    meta["moveik_start_quat"] = env.get_ee_orientation().copy()
    ticks.append(run_skill(mik, env, rec))
    meta["moveik_traj"] = np.array(mik.pos_traj)
    meta["moveik_quat_traj"] = np.array(mik.quat_traj)
    ticks.append(run_skill(S["gripper"].GripperSkill.open(env, duration=GRIP_TICKS), env, rec))
    out = {k: np.array(v) for k, v in rec.items()}
    out.update({k: np.asarray(v) for k, v in meta.items()})
    out["ticks"] = np.array(ticks)
    out["n_substeps"] = np.array(EG.N_SUBSTEPS)
    np.savez_compressed(os.path.join(HERE, "skill_golden.npz"), **out)
    print(f"wrote skill episode: ticks per skill {ticks}; MoveIK waypoints {len(mik.pos_traj)}; "
          f"final ee {out['ee_pos'][-1]}")


if __name__ == "__main__":
    main()
