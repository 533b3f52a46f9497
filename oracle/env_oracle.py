"""CPU restatement of the reference's gym env (panda_mujoco_gym/envs/panda_env.py,
envs/shelf_pnp.py) over the fp64 physics oracle (physics.c) — TEST INFRASTRUCTURE ONLY.

Each method follows the reference file:line in its docstring.  MuJoCo's data.site_* semantics
are modelled explicitly: `qpos_kin` is the qpos the last forward ran at (the pre-integration qpos
of the last sub-step of mj_step, or the state after mj_forward), and every site position /
orientation / Jacobian the env reads comes from the kinematics at qpos_kin, while velocities
multiply those Jacobians with the current (integrated) qvel and the finger width reads the
current qpos — exactly what the reference sees through gymnasium_robotics mujoco_utils.

Third-party helpers restated from their published definitions (absent here):
  gymnasium_robotics.utils.rotations.euler2quat / quat_mul / mat2euler (version 1.2.2),
  MuJoCo mju_mat2Quat (oracle.c orc_mat2quat).
The object-placement draws use Philox (pnp_amd/rng.py) instead of the reference's unseeded
global np.random: uniform(env_index, 2 * n_tasks, seed,
stream = 0x40000000 | episode), x then y per object.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from . import oracle as O

RESET_STREAM = 0x40000000
NEUTRAL = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00])   # panda_env.py:64-66
_EPS4 = np.finfo(np.float64).eps * 4.0


# ------------------------------------------------------------------ rotations (gymnasium_robotics)
def euler2quat(euler):
    e = np.asarray(euler, np.float64)
    ai, aj, ak = e[..., 2] / 2, -e[..., 1] / 2, e[..., 0] / 2
    si, sj, sk = np.sin(ai), np.sin(aj), np.sin(ak)
    ci, cj, ck = np.cos(ai), np.cos(aj), np.cos(ak)
    cc, cs, sc, ss = ci * ck, ci * sk, si * ck, si * sk
    q = np.empty(e.shape[:-1] + (4,))
    q[..., 0] = cj * cc + sj * ss
    q[..., 3] = cj * sc - sj * cs
    q[..., 2] = -(cj * ss + sj * cc)
    q[..., 1] = cj * cs - sj * sc
    return q


def quat_mul(a, b):
    w0, x0, y0, z0 = a
    w1, x1, y1, z1 = b
    return np.array([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1,
                     w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                     w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1,
                     w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1])


def mat2euler(mat):
    R = np.asarray(mat, np.float64).reshape(3, 3)
    cy = np.sqrt(R[2, 2] * R[2, 2] + R[1, 2] * R[1, 2])
    ok = cy > _EPS4
    e = np.empty(3)
    e[2] = -np.arctan2(R[0, 1], R[0, 0]) if ok else -np.arctan2(-R[1, 0], R[1, 1])
    e[1] = -np.arctan2(-R[0, 2], cy)
    e[0] = -np.arctan2(R[1, 2], R[2, 2]) if ok else 0.0
    return e


VERTICAL_QUAT = euler2quat(np.zeros(3))                        # panda_env.py:29
HORIZONTAL_QUAT = euler2quat(np.array([-np.pi / 2, 0, 0]))     # panda_env.py:30


@dataclasses.dataclass
class EnvConfig:
    """FrankaShelfPNPEnv constructor values (shelf_pnp.py:11-25, panda_env.py:32-46, 205-277)."""
    reward_type: str = "dense"
    n_substeps: int = 25
    n_calls: int = 10
    max_episode_steps: int = 300
    task_sequence: tuple = ("cube1", "cube2", "cube3")
    distance_threshold: float = 0.05
    obj_x_range: float = 0.02
    obj_y_range: float = 0.2
    high_pick_z: float = 0.35
    grip_width: float = 0.045
    reach_thresh: float = 0.05
    lift_height: float = 0.04
    pos_scale: float = 0.05
    rot_scale: float = 0.1
    finger_scale: float = 0.2
    seed: int = 20250808


class EnvOracle:
    """B independent FrankaShelfPNPEnv instances, fp64, one env at a time."""

    def __init__(self, B, cfg: EnvConfig | None = None, env_index=None, model=None, nthreads=8):
        self.m = m = model or O.load_model()
        self.cfg = cfg or EnvConfig()
        self.B = B
        self.nthreads = nthreads
        self.env_index = np.arange(B) if env_index is None else np.asarray(env_index)
        q = lambda j: int(m.jnt_qposadr[m.joint_id(j)])
        self.ee = m.site_id("ee_center_site")
        self.obj_site = [m.site_id(f"{o}_site") for o in self.cfg.task_sequence]
        self.target_site = [m.site_id(f"target_{o}") for o in self.cfg.task_sequence]
        self.obj_qadr = [q(f"{o}_joint") for o in self.cfg.task_sequence]
        self.finger_qadr = [q("finger_joint1"), q("finger_joint2")]
        self.neutral_qadr = [q(f"joint{i}") for i in range(1, 8)] + self.finger_qadr
        self.height_qadr = q("obj_joint")
        self.st = O.new_state(B, model=m)
        self._env_setup()

    # ---------------------------------------------------------------- helpers
    def _frames(self, b, site, qpos=None):
        """site_xpos / site_xmat (all sites) + jacp / jacr of `site` at qpos_kin[b]."""
        qk = self.qpos_kin[b] if qpos is None else qpos
        sx, sm, jp, jr = O.site_jac2(qk[None], site, self.st["mocap_pos"][b][None], self.st["mocap_quat"][b][None],
                                     model=self.m)
        return sx[0], sm[0], jp[0], jr[0]

    def _advance(self, idx):
        """n_calls x mj_step(nstep=n_substeps) on envs idx; records qpos_kin (panda_env.py:355-358)."""
        n = self.cfg.n_substeps * self.cfg.n_calls
        sub = {k: v[idx].copy() for k, v in self.st.items()}
        O.step(sub, nsub=n - 1, nthreads=self.nthreads, model=self.m)
        qk = sub["qpos"].copy()
        # a bad-state reset inside the last sub-step (mj_checkPos / checkVel / checkAcc ->
        # mj_resetData) means its forward ran at qpos0 (warn bits are sticky: first reset only)
        pre = {k: v.copy() for k, v in sub.items()}
        O.step(sub, nsub=1, nthreads=self.nthreads, model=self.m)
        bad = (sub["warn"] & 7) & ~(pre["warn"] & 7)
        for j in np.nonzero(bad)[0]:
            qk[j] = self.m.qpos0
        for k in self.st:
            self.st[k][idx] = sub[k]
        self.qpos_kin[idx] = qk

    # ---------------------------------------------------------------- init (panda_env.py:106-141, 100-104)
    def _env_setup(self):
        m, cfg, st = self.m, self.cfg, self.st
        B = self.B
        self.qpos_kin = st["qpos"].copy()
        st["qpos"][:, self.neutral_qadr] = NEUTRAL                 # set_joint_neutral (:322-327)
        st["ctrl"][:, :7] = NEUTRAL[:7]                            # :127
        sx, sm, _, _ = self._frames(0, self.ee, qpos=st["qpos"][0])   # reset_mocap_welds -> mj_forward
        mocap_q = O.mat2quat(sm[self.ee])                          # get_ee_orientation (:337-342)
        st["mocap_pos"][:] = sx[self.ee]                           # set_mocap_pose (:137)
        st["mocap_quat"][:] = mocap_q
        self._advance(np.arange(B))                                # _mujoco_step (:138)
        self.obj_height0 = st["qpos"][:, self.height_qadr + 2].copy()   # :139-141
        self.init_time = st["time"].copy()                         # :121
        self.init_qvel = st["qvel"].copy()                         # :122
        self.init_mocap = np.concatenate([st["mocap_pos"], st["mocap_quat"]], 1)
        self.task = np.zeros(B, np.int64)                          # _initialize_multi_object_task
        self.elapsed = np.zeros(B, np.int64)
        self.episode = np.zeros(B, np.int64)
        sxt, _, _, _ = self._frames(0, self.ee)
        self.goal = np.tile(sxt[self.target_site[0]], (B, 1))     # _sample_goal (:360-364)

    # ---------------------------------------------------------------- observation (panda_env.py:279-301)
    def _observe(self, b, task, goal):
        cfg = self.cfg
        ti = min(task, len(self.obj_site) - 1)
        dt = self.m.opt_timestep * cfg.n_substeps                  # MujocoRobotEnv.dt
        qvel = self.st["qvel"][b]
        sx, sm, jp_ee, _ = self._frames(b, self.ee)
        _, _, jp_ob, jr_ob = self._frames(b, self.obj_site[ti])
        ee_pos = sx[self.ee]
        ob_pos = sx[self.obj_site[ti]]
        width = self.st["qpos"][b, self.finger_qadr[0]] + self.st["qpos"][b, self.finger_qadr[1]]
        obs = np.concatenate([ee_pos, (jp_ee @ qvel) * dt, [width], ob_pos, mat2euler(sm[self.obj_site[ti]]),
                              (jp_ob @ qvel) * dt, (jr_ob @ qvel) * dt])
        return dict(observation=obs, achieved_goal=ob_pos.copy(), desired_goal=np.array(goal, np.float64),
                    ee_pos=ee_pos, ee_xmat=sm[self.ee], width=width, sx=sx)

    # ---------------------------------------------------------------- reset (panda_env.py:366-391, 146-158)
    def reset(self, mask=None):
        from pnp_amd import rng
        cfg, st = self.cfg, self.st
        out = {}
        idx = np.arange(self.B) if mask is None else np.nonzero(mask)[0]
        for b in idx:
            sx_old, _, _, _ = self._frames(b, self.ee)             # data.site_xpos before the reset
            st["time"][b] = self.init_time[b]
            st["qvel"][b] = self.init_qvel[b]
            st["qpos"][b, self.neutral_qadr] = NEUTRAL
            st["mocap_pos"][b] = self.init_mocap[b, :3]
            st["mocap_quat"][b] = self.init_mocap[b, 3:]
            u = rng.uniform(np.array([self.env_index[b]]), 2 * len(self.obj_site), seed=cfg.seed,
                            stream=RESET_STREAM | int(self.episode[b]))[0]
            for k, (s, a) in enumerate(zip(self.obj_site, self.obj_qadr)):
                c = sx_old[s]
                x = c[0] + (-cfg.obj_x_range + (cfg.obj_x_range - -cfg.obj_x_range) * u[2 * k])
                y = c[1] + (-cfg.obj_y_range + (cfg.obj_y_range - -cfg.obj_y_range) * u[2 * k + 1])
                st["qpos"][b, a:a + 7] = [x, y, c[2], 1, 0, 0, 0]
            self.task[b] = 0
            self.elapsed[b] = 0
            self.episode[b] += 1
            self.qpos_kin[b] = st["qpos"][b]                       # mj_forward (:383)
            sxn, _, _, _ = self._frames(b, self.ee)
            self.goal[b] = sxn[self.target_site[0]]
            out[b] = self._observe(b, 0, self.goal[b])
        return out

    # ---------------------------------------------------------------- step (panda_env.py:163-277)
    def step(self, actions):
        cfg, st = self.cfg, self.st
        # float32 action space: the clip and the action scalings run in float32 (NumPy promotes
        # float32 array * python float to float32), then meet the float64 state
        f32 = np.float32
        actions = np.clip(np.asarray(actions, f32), f32(-1.0), f32(1.0))
        for b in range(self.B):                                    # _set_action (:250-277)
            a = actions[b]
            sx, sm, _, _ = self._frames(b, self.ee)
            width = (st["qpos"][b, self.finger_qadr[0]] + st["qpos"][b, self.finger_qadr[1]]
                     + np.float64(a[6] * f32(cfg.finger_scale)))
            lo, hi = self.m.actuator_ctrlrange[-1]
            st["ctrl"][b, -2:] = np.clip(width / 2, lo, hi)
            pos = sx[self.ee] + (f32(cfg.pos_scale) * a[:3]).astype(np.float64)
            pos[2] = max(0.0, pos[2])
            dq = euler2quat((np.clip(a[3:6], f32(-1.0), f32(1.0)) * f32(cfg.rot_scale)).astype(np.float64))
            st["mocap_pos"][b] = pos
            st["mocap_quat"][b] = quat_mul(dq, O.mat2quat(sm[self.ee]))
        self._advance(np.arange(self.B))
        res = []
        for b in range(self.B):
            task = int(self.task[b])
            ob = self._observe(b, task, self.goal[b])
            ag, dg = ob["achieved_goal"], ob["desired_goal"]
            d_reach = float(np.linalg.norm(ob["ee_pos"] - ag))     # compute_reward (:205-245)
            d_place = float(np.linalg.norm(ag - dg))
            gripped = ob["width"] < cfg.grip_width and d_reach < cfg.reach_thresh
            lifted = gripped and (ag[2] - self.obj_height0[b] > cfg.lift_height)
            placed = d_place < cfg.distance_threshold
            ee_q = O.mat2quat(ob["ee_xmat"])
            need = HORIZONTAL_QUAT if ag[2] > cfg.high_pick_z else VERTICAL_QUAT
            ori_err = 1.0 - abs(float(np.dot(ee_q, need)))
            if cfg.reward_type == "sparse":
                reward = -float(not placed)
            else:
                reward = -0.003 - min(d_reach, cfg.reach_thresh)
                if gripped:
                    reward += 2.0 + (1.0 - ori_err)
                if lifted:
                    reward += 4.0
                if placed:
                    reward += 10.0
                reward += 0.5 * (task / len(self.obj_site))
            reward = float(np.float32(reward))                     # compute_reward returns np.float32
            terminated = False
            if placed:                                             # task sequencing (:183-193)
                self.task[b] = task + 1
                if self.task[b] < len(self.obj_site):
                    self.goal[b] = ob["sx"][self.target_site[self.task[b]]]
                else:
                    terminated = True
            self.elapsed[b] += 1                                   # TimeLimit (__init__.py:15)
            truncated = cfg.max_episode_steps > 0 and self.elapsed[b] >= cfg.max_episode_steps
            res.append(dict(obs=ob, reward=reward, is_success=float(placed), terminated=terminated,
                            truncated=bool(truncated)))
        return res
