"""Generate tests/golden/env_golden.npz by running the REFERENCE's own gym env code.

Runs in the build container only (needs /root/reference; the GPU box never does this).
``panda_mujoco_gym/envs/panda_env.py`` is imported unmodified from /root/reference with stubs
for its absent third-party dependencies:
  * ``mujoco``: mj_step / mj_forward / mju_mat2Quat backed by the CPU physics oracle
    (oracle/physics.c), keeping MuJoCo's data.site_* semantics (site frames and Jacobians are
    those of the last forward: the pre-integration qpos of the last sub-step of mj_step),
  * ``gymnasium_robotics.utils.mujoco_utils``-style accessors (get_site_xpos / xmat / xvelp /
    xvelr, get/set_joint_qpos, set_mocap_pos / quat) over that state,
  * ``gymnasium_robotics.utils.rotations``: the restatement in oracle/env_oracle.py,
  * ``MujocoRobotEnv``: only what FrankaEnv uses from it (dt, compute_truncated, _step_callback).
``FrankaEnv._env_setup``, ``_initialize_multi_object_task``, ``_reset_sim`` and ``step`` then
run exactly as written; the global ``np.random.uniform`` draws of ``_sample_object`` are fed the
Philox values the product uses (uniform(env, 6, seed, 0x40000000 | episode), x then y per object).
Physics is short (n_substeps = 1: 10 sub-steps per gym step) so the fixture pins the env logic,
not the scene's chaotic long-horizon dynamics.

Only the resulting arrays are committed; no reference source or bytecode is copied.
Usage: python tests/golden/make_env_golden.py
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

from oracle import env_oracle as EO  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pnp_amd import rng  # noqa: E402
from pnp_amd.model import load_model  # noqa: E402

N_SUBSTEPS = 1


class _Opt:
    def __init__(self, dt):
        self.timestep = dt


class StubModel:
    def __init__(self, m):
        self._m = m
        self.nu, self.nq, self.nv, self.na, self.nmocap = m.nu, m.nq, m.nv, 0, m.nmocap
        self.actuator_ctrlrange = m.actuator_ctrlrange.copy()
        self.eq_data = m.eq_data.copy()
        self.eq_type = m.eq_type.copy()
        self.opt = _Opt(m.opt_timestep)


class StubData:
    def __init__(self, m):
        st = O.new_state(1, model=m)
        self.st = st
        self.qpos_kin = st["qpos"][0].copy()

    def __getattr__(self, k):
        st = self.__dict__["st"]
        if k in st:
            return st[k][0] if k not in ("mocap_pos", "mocap_quat") else st[k][0].reshape(1, -1)
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if k in ("st", "qpos_kin"):
            object.__setattr__(self, k, v)
        elif k in self.__dict__["st"]:
            self.__dict__["st"][k][0] = v
        else:
            object.__setattr__(self, k, v)


def make_stubs(m):
    mj = types.ModuleType("mujoco")
    mj.mjtEq = types.SimpleNamespace(mjEQ_WELD=1)

    def mj_forward(model, data):
        data.qpos_kin = data.st["qpos"][0].copy()

    def mj_step(model, data, nstep=1):
        st = data.st
        O.step(st, nsub=nstep - 1, model=m)
        qk = st["qpos"][0].copy()
        warn0 = int(st["warn"][0])
        O.step(st, nsub=1, model=m)
        if (int(st["warn"][0]) & 7) & ~(warn0 & 7):
            qk = m.qpos0.copy()
        data.qpos_kin = qk

    def mju_mat2Quat(quat, mat):
        quat[:] = O.mat2quat(np.asarray(mat).reshape(9))

    mj.mj_forward, mj.mj_step, mj.mju_mat2Quat = mj_forward, mj_step, mju_mat2Quat

    def frames(data, site):
        st = data.st
        return O.site_jac2(data.qpos_kin[None], site, st["mocap_pos"], st["mocap_quat"], model=m)

    def jaddr(name):
        j = m.joint_id(name)
        a = int(m.jnt_qposadr[j])
        n = {0: 7, 1: 4}.get(int(m.jnt_type[j]), 1)
        return a, n

    ut = types.SimpleNamespace()
    ut.get_site_xpos = lambda model, data, name: frames(data, name)[0][0, m.site_id(name)].copy()
    ut.get_site_xmat = lambda model, data, name: frames(data, name)[1][0, m.site_id(name)].reshape(3, 3).copy()
    ut.get_site_xvelp = lambda model, data, name: frames(data, name)[2][0] @ data.st["qvel"][0]
    ut.get_site_xvelr = lambda model, data, name: frames(data, name)[3][0] @ data.st["qvel"][0]

    def get_joint_qpos(model, data, name):
        a, n = jaddr(name)
        return data.st["qpos"][0, a:a + n].copy()

    def set_joint_qpos(model, data, name, value):
        a, n = jaddr(name)
        data.st["qpos"][0, a:a + n] = value

    ut.get_joint_qpos, ut.set_joint_qpos = get_joint_qpos, set_joint_qpos

    def set_mocap_pos(model, data, name, value):
        data.st["mocap_pos"][0] = value

    def set_mocap_quat(model, data, name, value):
        data.st["mocap_quat"][0] = value

    ut.set_mocap_pos, ut.set_mocap_quat = set_mocap_pos, set_mocap_quat
    return mj, ut


class StubRobotEnv:
    """What FrankaEnv uses of gymnasium_robotics' MujocoRobotEnv."""

    @property
    def dt(self):
        return self.model.opt.timestep * self.n_substeps

    def compute_truncated(self, achieved_goal, desired_goal, info):
        return False

    def _step_callback(self):
        pass


class StubBox:
    def __init__(self):
        self.low, self.high, self.shape = -np.ones(7, np.float32), np.ones(7, np.float32), (7,)


def import_reference_env(m):
    mj, ut = make_stubs(m)
    sys.modules["mujoco"] = mj
    gym = types.ModuleType("gymnasium")
    core = types.ModuleType("gymnasium.core")
    core.ObsType = object
    gym.core = core
    gr = types.ModuleType("gymnasium_robotics")
    gre = types.ModuleType("gymnasium_robotics.envs")
    grr = types.ModuleType("gymnasium_robotics.envs.robot_env")
    grr.MujocoRobotEnv = StubRobotEnv
    gru = types.ModuleType("gymnasium_robotics.utils")
    rot = types.ModuleType("gymnasium_robotics.utils.rotations")
    rot.euler2quat, rot.quat_mul, rot.mat2euler = EO.euler2quat, EO.quat_mul, EO.mat2euler
    gru.rotations = rot
    for name, mod in (("gymnasium", gym), ("gymnasium.core", core), ("gymnasium_robotics", gr),
                      ("gymnasium_robotics.envs", gre), ("gymnasium_robotics.envs.robot_env", grr),
                      ("gymnasium_robotics.utils", gru), ("gymnasium_robotics.utils.rotations", rot)):
        sys.modules[name] = mod
    for name, sub in (("panda_mujoco_gym", ""), ("panda_mujoco_gym.envs", "envs")):
        pkg = types.ModuleType(name)
        pkg.__path__ = [os.path.join(REF, "panda_mujoco_gym", sub)]
        sys.modules[name] = pkg
    mod = importlib.import_module("panda_mujoco_gym.envs.panda_env")
    return mod, mj, ut


def new_env(mod, mj, ut, m, reward_type):
    """FrankaShelfPNPEnv as constructed by shelf_pnp.py / FrankaEnv.__init__ (values only), then
    the reference's own _env_setup + _initialize_multi_object_task."""
    env = mod.FrankaEnv.__new__(mod.FrankaEnv)
    env.task_sequence = ["cube1", "cube2", "cube3"]
    env.current_task_index = 0
    env.current_target_object = "cube1"
    env.goal = None
    env.block_gripper = False
    env.reward_type = reward_type
    env.neutral_joint_values = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00])
    env.orientation_weight, env.orientation_threshold, env.high_pick_z = 0.2, 0.15, 0.35
    env.distance_threshold, env.obj_x_range, env.obj_y_range = 0.05, 0.02, 0.2
    env.n_substeps = N_SUBSTEPS
    env.render_mode = None
    env.action_space = StubBox()
    env._mujoco, env._utils = mj, ut
    env.model, env.data = StubModel(m), StubData(m)
    env.arm_joint_names = [f"joint{i}" for i in range(1, 8)]
    env.gripper_joint_names = ["finger_joint1", "finger_joint2"]
    env.nu, env.nq, env.nv = m.nu, m.nq, m.nv
    env.ctrl_range = env.model.actuator_ctrlrange
    env._env_setup(env.neutral_joint_values)
    env.initial_time = env.data.time
    env.initial_qvel = np.copy(env.data.qvel)
    env._initialize_multi_object_task()
    return env


def philox_reset(env_index, episode, n):
    u = rng.uniform(np.array([env_index]), n, seed=rng.SEED, stream=EO.RESET_STREAM | episode)[0]
    it = iter(u)
    return lambda low, high: low + (high - low) * next(it)


def main():
    m = load_model()
    mod, mj, ut = import_reference_env(m)
    rec = {k: [] for k in ("env_index", "reward_dense", "obj_height0", "init_mocap", "reset_obs", "reset_goal",
                           "actions", "place", "obs", "reward", "success", "terminated", "ctrl", "mocap_pos",
                           "mocap_quat", "task", "goal")}
    nsteps = 6
    scen = []
    for e in range(3):
        scen.append((e, "dense", [False] * nsteps))
    scen.append((0, "sparse", [False] * nsteps))
    scen.append((1, "dense", [True, False, True, True, False, True]))   # object placed before these steps
    real_uniform = np.random.uniform
    for env_index, rtype, place in scen:
        env = new_env(mod, mj, ut, m, rtype)
        rec["obj_height0"].append(float(env.initial_object_height))
        rec["init_mocap"].append(np.concatenate([env.initial_mocap_position, env.grasp_site_pose]))
        np.random.uniform = philox_reset(env_index, 0, 6)
        try:
            env._reset_sim()
        finally:
            np.random.uniform = real_uniform
        env.goal = env._sample_goal().copy()           # BaseRobotEnv.reset after _reset_sim
        o = env._get_obs()
        rec["reset_obs"].append(o["observation"])
        rec["reset_goal"].append(env.goal.copy())
        acts = np.random.default_rng(100 + env_index).uniform(-1, 1, size=(nsteps, 7)).astype(np.float32)
        rows = {k: [] for k in ("obs", "reward", "success", "terminated", "ctrl", "mocap_pos", "mocap_quat", "task",
                                "goal")}
        for k in range(nsteps):
            if place[k]:
                obj = env.current_target_object
                j = m.joint_id(f"{obj}_joint")
                a = int(m.jnt_qposadr[j])
                env.data.st["qpos"][0, a:a + 7] = np.concatenate([env.goal, [1, 0, 0, 0]])
                mj.mj_forward(env.model, env.data)
            obs, r, term, trunc, info = env.step(acts[k])
            rows["obs"].append(obs["observation"])
            rows["reward"].append(float(r))
            rows["success"].append(float(info["is_success"]))
            rows["terminated"].append(bool(term))
            rows["ctrl"].append(env.data.st["ctrl"][0].copy())
            rows["mocap_pos"].append(env.data.st["mocap_pos"][0].copy())
            rows["mocap_quat"].append(env.data.st["mocap_quat"][0].copy())
            rows["task"].append(env.current_task_index)
            rows["goal"].append(np.array(env.goal, np.float64).copy())
        rec["env_index"].append(env_index)
        rec["reward_dense"].append(rtype == "dense")
        rec["actions"].append(acts)
        rec["place"].append(place)
        for k, v in rows.items():
            rec[k].append(v)
    out = {k: np.array(v) for k, v in rec.items()}
    out["n_substeps"] = np.array(N_SUBSTEPS)
    np.savez_compressed(os.path.join(HERE, "env_golden.npz"), **out)
    print(f"wrote {len(scen)} reference env episodes x {nsteps} steps; rewards "
          f"{np.round(out['reward'], 3).tolist()}; success {out['success'].sum()}, terminated {out['terminated'].sum()}")


if __name__ == "__main__":
    main()
