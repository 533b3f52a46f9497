"""Batched FrankaShelfPNP gym envs on the GPU (reference panda_mujoco_gym/envs/panda_env.py,
envs/shelf_pnp.py, __init__.py registration).

``BatchedFrankaShelfPNPEnv``  B envs on one device; one fused HIP launch per gym step
                              (pnp_env_step: _set_action -> 250 mj_step -> obs / reward / success
                              / task sequencing / TimeLimit), vector-env auto-reset.
``FrankaShelfPNPEnv``         the single-env gymnasium surface (reset / step / the helper methods
                              the skills and behaviour tree call), numpy in / out, B = 1 on the
                              device (fp64 by default, like MuJoCo's mjtNum).
``make(env_id)``              gym.make replacement for FrankaShelfPNP{Dense,Sparse}-v0
                              (max_episode_steps = 300).

Everything runs through libpnp.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np
import torch

from . import _lib, rng
from .engine import _ptr, _stream, get_engine

NEUTRAL = (0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00)   # panda_env.py:64-66
ENV_IDS = ("FrankaShelfPNPSparse-v0", "FrankaShelfPNPDense-v0")     # __init__.py:6-18


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
    seed: int = rng.SEED


def env_params(model, cfg: EnvConfig) -> _lib.PnpEnvParams:
    if cfg.reward_type not in ("dense", "sparse"):
        raise ValueError(f"reward_type must be 'dense' or 'sparse', got {cfg.reward_type!r}")
    n = len(cfg.task_sequence)
    if not 1 <= n <= _lib.MAX_TASKS:
        raise ValueError(f"task_sequence must have 1..{_lib.MAX_TASKS} objects")
    q = lambda j: int(model.jnt_qposadr[model.joint_id(j)])
    p = _lib.PnpEnvParams()
    p.n_substeps, p.n_calls = cfg.n_substeps, cfg.n_calls
    p.reward_dense = int(cfg.reward_type == "dense")
    p.max_episode_steps, p.n_tasks = cfg.max_episode_steps, n
    p.ee_site = model.site_id("ee_center_site")
    for k, o in enumerate(cfg.task_sequence):
        p.obj_site[k] = model.site_id(f"{o}_site")
        p.target_site[k] = model.site_id(f"target_{o}")
        p.obj_qadr[k] = q(f"{o}_joint")
    p.finger_qadr[0], p.finger_qadr[1] = q("finger_joint1"), q("finger_joint2")
    for i, j in enumerate([f"joint{i}" for i in range(1, 8)] + ["finger_joint1", "finger_joint2"]):
        p.neutral_qadr[i] = q(j)
        p.neutral[i] = NEUTRAL[i]
    p.height_qadr = q("obj_joint")
    p.arm_ctrl_n = 7
    for f in ("distance_threshold", "high_pick_z", "grip_width", "reach_thresh", "lift_height", "obj_x_range",
              "obj_y_range", "pos_scale", "rot_scale", "finger_scale"):
        setattr(p, f, float(getattr(cfg, f)))
    p.seed_lo, p.seed_hi = cfg.seed & 0xFFFFFFFF, (cfg.seed >> 32) & 0xFFFFFFFF
    return p


class Box:
    """Minimal gymnasium.spaces.Box stand-in (gymnasium is not a dependency)."""

    def __init__(self, low, high, shape, dtype=np.float32, seed=None):
        self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        self.low = np.full(shape, low, dtype=self.dtype)
        self.high = np.full(shape, high, dtype=self.dtype)
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)


class BatchedFrankaShelfPNPEnv:
    """``num_envs`` FrankaShelfPNPEnv instances on one GPU.

    Global env indices ``env_offset + arange(num_envs)`` key the reset draws, so a batch sharded
    over ranks (rank r: env_offset = r * num_envs) reproduces the single-device batch exactly.
    """

    def __init__(self, num_envs, reward_type="dense", device=None, dtype=torch.float32, env_offset=0,
                 autoreset=True, config: EnvConfig | None = None, engine=None):
        self.engine = engine or get_engine(device)
        self.model = m = self.engine.model
        self.cfg = dataclasses.replace(config or EnvConfig(), reward_type=reward_type)
        self.params = env_params(m, self.cfg)
        self.num_envs = B = int(num_envs)
        self.dtype, self.device = dtype, self.engine.device
        self.autoreset = autoreset
        self.task_sequence = list(self.cfg.task_sequence)
        self.action_space = Box(-1.0, 1.0, (7,))
        dev, dt = self.device, dtype
        self.state = self.engine.new_state(B, dtype)
        z = lambda *s, d=dt: torch.zeros(*s, dtype=d, device=dev)
        self.env = dict(goal=z(B, 3), task=z(B, d=torch.int32), elapsed=z(B, d=torch.int32),
                        qpos_kin=z(B, m.nq), obj_height0=z(B), init_mocap=z(B, 7), init_qvel=z(B, m.nv),
                        init_time=z(B), episode=z(B, d=torch.int32),
                        env_index=torch.arange(env_offset, env_offset + B, dtype=torch.int32, device=dev),
                        tier=z(B, d=torch.uint8))   # fp32 routing hint (include/pnp.h pnp_env_state.tier)
        self.out = dict(obs=z(B, _lib.OBS_DIM), achieved_goal=z(B, 3), desired_goal=z(B, 3), reward=z(B),
                        is_success=z(B), terminated=z(B, d=torch.uint8), truncated=z(B, d=torch.uint8))
        self._S, _, _ = self.engine._state_struct(self.state)
        self._E = _lib.PnpEnvState(*[self.env[k].data_ptr() for k in _lib.ENV_STATE_FIELDS])
        self._O = _lib.PnpEnvOut(*[self.out[k].data_ptr() for k in _lib.ENV_OUT_FIELDS])
        f64 = dt == torch.float64
        L = self.engine.lib
        self._eval = L.pnp_env_evaluate_f64 if f64 else L.pnp_env_evaluate
        self.eval_out = dict(obs=z(B, _lib.OBS_DIM), achieved_goal=z(B, 3), desired_goal=z(B, 3), reward=z(B),
                             is_success=z(B))
        self._EO = _lib.PnpEnvOut(*[self.eval_out[k].data_ptr() if k in self.eval_out else None
                                    for k in _lib.ENV_OUT_FIELDS])
        self._init = L.pnp_env_init_f64 if f64 else L.pnp_env_init
        self._reset = L.pnp_env_reset_f64 if f64 else L.pnp_env_reset
        self._step = L.pnp_env_step_f64 if f64 else L.pnp_env_step
        h = self.engine._h
        _lib.check(self._init(h, C.byref(self._S), C.byref(self.params), C.byref(self._E), B, _stream()),
                   "pnp_env_init")

    # ---------------------------------------------------------------- gym surface
    def _obs(self):
        return {"observation": self.out["obs"], "achieved_goal": self.out["achieved_goal"],
                "desired_goal": self.out["desired_goal"]}

    def reset(self, mask=None):
        """Reset every env (mask None) or the envs where mask != 0; returns the obs dict (device
        tensors, views of the output buffers: copy before the next call)."""
        mp = None
        if mask is not None:
            mask = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
            if mask.shape != (self.num_envs,):
                raise ValueError(f"mask must have shape ({self.num_envs},)")
            mp = _ptr(mask)
        _lib.check(self._reset(self.engine._h, C.byref(self._S), C.byref(self.params), C.byref(self._E), mp,
                               C.byref(self._O), self.num_envs, _stream()), "pnp_env_reset")
        self._keep = mask
        return self._obs()

    def step(self, actions):
        """actions [B, 7] -> (obs, reward, terminated, truncated, info).  With autoreset, envs that
        ended are reset in the same call: obs holds their first observation, and
        info["final_observation"] / info["final_achieved_goal"] the terminal ones."""
        a = torch.as_tensor(actions, device=self.device).to(self.dtype).contiguous()
        if a.shape != (self.num_envs, 7):
            raise ValueError("Action dimension mismatch")          # panda_env.py:165-166
        _lib.check(self._step(self.engine._h, C.byref(self._S), C.byref(self.params), C.byref(self._E), _ptr(a),
                              C.byref(self._O), self.num_envs, _stream()), "pnp_env_step")
        reward = self.out["reward"].clone()
        term = self.out["terminated"].bool()
        trunc = self.out["truncated"].bool()
        info = {"is_success": self.out["is_success"].clone()}
        if self.autoreset:
            done = term | trunc
            info["final_observation"] = self.out["obs"].clone()
            info["final_achieved_goal"] = self.out["achieved_goal"].clone()
            info["final_desired_goal"] = self.out["desired_goal"].clone()
            if bool(done.any()):
                self.reset(done)
        obs = {k: v.clone() for k, v in self._obs().items()}
        return obs, reward, term, trunc, info

    def evaluate(self, achieved_goal=None, desired_goal=None):
        """_get_obs + compute_reward / _is_success at the current state, no step (pnp_env_evaluate):
        returns the eval_out dict (obs / achieved_goal / desired_goal observed, reward / is_success
        for the given goals, default the observed ones).  Views: copy before the next call."""
        def goals(g):
            if g is None:
                return None, None
            t = torch.as_tensor(g, device=self.device).to(self.dtype).reshape(self.num_envs, 3).contiguous()
            return t, _ptr(t)
        ag, agp = goals(achieved_goal)
        dg, dgp = goals(desired_goal)
        _lib.check(self._eval(self.engine._h, C.byref(self._S), C.byref(self.params), C.byref(self._E), agp, dgp,
                              C.byref(self._EO), self.num_envs, _stream()), "pnp_env_evaluate")
        return self.eval_out

    def step_subset(self, idx, actions):
        """FrankaEnv.step for the envs ``idx`` only (no auto-reset): their state and episode
        state are gathered into a contiguous sub-batch, stepped by one pnp_env_step launch and
        scattered back; the other envs are untouched.  Per env the result is the full-batch
        step's (envs are independent).  Returns the sub-batch's outputs (device tensors)."""
        idx = torch.as_tensor(idx, dtype=torch.long, device=self.device)
        n = int(idx.numel())
        a = torch.as_tensor(actions, device=self.device).to(self.dtype).reshape(n, 7).contiguous()
        st = {k: v.index_select(0, idx).contiguous() for k, v in self.state.items()}
        ev = {k: v.index_select(0, idx).contiguous() for k, v in self.env.items()}
        z = lambda *sh, d=self.dtype: torch.zeros(*sh, dtype=d, device=self.device)
        out = dict(obs=z(n, _lib.OBS_DIM), achieved_goal=z(n, 3), desired_goal=z(n, 3), reward=z(n),
                   is_success=z(n), terminated=z(n, d=torch.uint8), truncated=z(n, d=torch.uint8))
        S, _, _ = self.engine._state_struct(st)
        E = _lib.PnpEnvState(*[ev[k].data_ptr() for k in _lib.ENV_STATE_FIELDS])
        O = _lib.PnpEnvOut(*[out[k].data_ptr() for k in _lib.ENV_OUT_FIELDS])
        if n:
            _lib.check(self._step(self.engine._h, C.byref(S), C.byref(self.params), C.byref(E), _ptr(a), C.byref(O), n,
                                  _stream()), "pnp_env_step")
        for k, v in st.items():
            self.state[k].index_copy_(0, idx, v)
        for k, v in ev.items():
            self.env[k].index_copy_(0, idx, v)
        return out

    # ---------------------------------------------------------------- helpers (panda_env.py:317-352)
    def _site_frames(self):
        """site_xpos / site_xmat of the last forward (data.site_*)."""
        return self.engine.site_kinematics(self.env["qpos_kin"], self.state["mocap_pos"], self.state["mocap_quat"])

    def get_ee_position(self):
        sx, _ = self._site_frames()
        return sx[:, self.params.ee_site]

    def get_ee_orientation(self):
        """mju_mat2Quat(site_xmat[ee]) per env (wxyz)."""
        _, sm = self._site_frames()
        return mat2quat_batch(sm[:, self.params.ee_site])

    def get_fingers_width(self):
        q = self.state["qpos"]
        return q[:, self.params.finger_qadr[0]] + q[:, self.params.finger_qadr[1]]

    def set_mocap_pose(self, pos, quat):
        self.state["mocap_pos"].copy_(torch.as_tensor(pos, dtype=self.dtype, device=self.device).reshape(-1, 3))
        self.state["mocap_quat"].copy_(torch.as_tensor(quat, dtype=self.dtype, device=self.device).reshape(-1, 4))

    @property
    def current_task_index(self):
        return self.env["task"]

    @property
    def goal(self):
        return self.env["goal"]


def mat2quat_batch(R):
    """mju_mat2Quat on [N, 9] row-major matrices (torch, device): host-side helper for the facade's
    accessors (the kernels carry their own copy)."""
    R = R.reshape(-1, 9)
    q = torch.zeros(R.shape[0], 4, dtype=R.dtype, device=R.device)
    t = R[:, 0] + R[:, 4] + R[:, 8]
    c0 = t > 0
    c1 = ~c0 & (R[:, 0] > R[:, 4]) & (R[:, 0] > R[:, 8])
    c2 = ~c0 & ~c1 & (R[:, 4] > R[:, 8])
    c3 = ~c0 & ~c1 & ~c2
    s = torch.sqrt(torch.clamp(1 + R[:, 0] + R[:, 4] + R[:, 8], min=0)) * 0.5
    q[c0, 0] = s[c0]
    q[c0, 1] = 0.25 * (R[c0, 7] - R[c0, 5]) / s[c0]
    q[c0, 2] = 0.25 * (R[c0, 2] - R[c0, 6]) / s[c0]
    q[c0, 3] = 0.25 * (R[c0, 3] - R[c0, 1]) / s[c0]
    s = torch.sqrt(torch.clamp(1 + R[:, 0] - R[:, 4] - R[:, 8], min=0)) * 0.5
    q[c1, 1] = s[c1]
    q[c1, 0] = 0.25 * (R[c1, 7] - R[c1, 5]) / s[c1]
    q[c1, 2] = 0.25 * (R[c1, 1] + R[c1, 3]) / s[c1]
    q[c1, 3] = 0.25 * (R[c1, 2] + R[c1, 6]) / s[c1]
    s = torch.sqrt(torch.clamp(1 - R[:, 0] + R[:, 4] - R[:, 8], min=0)) * 0.5
    q[c2, 2] = s[c2]
    q[c2, 0] = 0.25 * (R[c2, 2] - R[c2, 6]) / s[c2]
    q[c2, 1] = 0.25 * (R[c2, 1] + R[c2, 3]) / s[c2]
    q[c2, 3] = 0.25 * (R[c2, 5] + R[c2, 7]) / s[c2]
    s = torch.sqrt(torch.clamp(1 - R[:, 0] - R[:, 4] + R[:, 8], min=0)) * 0.5
    q[c3, 3] = s[c3]
    q[c3, 0] = 0.25 * (R[c3, 3] - R[c3, 1]) / s[c3]
    q[c3, 1] = 0.25 * (R[c3, 2] + R[c3, 6]) / s[c3]
    q[c3, 2] = 0.25 * (R[c3, 5] + R[c3, 7]) / s[c3]
    return q / torch.linalg.norm(q, dim=1, keepdim=True)


class FrankaShelfPNPEnv:
    """Single-env gymnasium surface of FrankaShelfPNPEnv (numpy in / out), B = 1 on the device.

    reset(seed=None) -> (obs, {});  step(a) -> (obs, reward, terminated, truncated, info), with
    TimeLimit(max_episode_steps) truncation and no auto-reset (gym semantics).  Also the helper
    methods the skills / behaviour tree use (get_ee_position, get_ee_orientation,
    get_fingers_width, set_mocap_pose, set_joint_neutral, home_pos, task_sequence, action_space)
    and the MuJoCo-binding objects behind ``unwrapped`` (``model``, ``data``, ``_mujoco``,
    ``_utils``: pnp_amd/mjshim.py) that reference code such as skills/base.py:41-44 and
    skills/move.py:79-85 reaches through.

    ``self.data`` (MjData, host) is the state of record between calls, as MjData is for the
    reference: writes to it are seen by the next step / mj_step, and every device call uploads it,
    runs, and downloads the result in place.
    """

    metadata = {"render_modes": [], "render_fps": 20}

    def __init__(self, reward_type="dense", render_mode=None, device=None, dtype=torch.float64,
                 max_episode_steps=300, config: EnvConfig | None = None, env_index: int = 0):
        from .mjshim import MjData, MujocoShim, UtilsShim
        if render_mode not in (None,):
            raise ValueError("rendering is not part of this engine (render_mode must be None)")
        cfg = dataclasses.replace(config or EnvConfig(), max_episode_steps=max_episode_steps)
        # env_index: the Philox counter of this env's reset draws (env i of a batched run)
        self._b = BatchedFrankaShelfPNPEnv(1, reward_type, device=device, dtype=dtype, autoreset=False, config=cfg,
                                           env_offset=int(env_index))
        self.model = self._b.model
        self.data = MjData(self.model)
        self._mujoco = MujocoShim(self._b.engine, dtype)
        self._utils = UtilsShim(self._mujoco)
        self.render_mode = None
        self.reward_type = reward_type
        self.task_sequence = self._b.task_sequence
        self.action_space = Box(-1.0, 1.0, (7,))
        self.home_pos = None
        self.dt = self._b.model.opt_timestep * cfg.n_substeps
        self.neutral_joint_values = np.array(NEUTRAL)
        self._pull()

    @property
    def unwrapped(self):
        return self

    # ---------------------------------------------------------------- mirror <-> device
    def _push(self):
        self._mujoco.upload(self.data, self._b.state)
        self._b.env["qpos_kin"][0].copy_(torch.from_numpy(np.asarray(self.data.qpos_kin, np.float64)))

    def _pull(self):
        self._mujoco.download(self.data, self._b.state)
        self.data.qpos_kin = self._b.env["qpos_kin"][0].double().cpu().numpy()
        self._mujoco.frames(self.data)

    def _np_obs(self, obs):
        return {k: v[0].double().cpu().numpy() for k, v in obs.items()}

    def reset(self, seed=None, options=None):
        if seed is not None:
            self.action_space.seed(seed)
        self._push()
        obs = self._np_obs(self._b.reset())
        self._pull()
        self.home_pos = self.get_ee_position().copy()               # panda_env.py:387-391
        return obs, {}

    def step(self, action):
        a = np.asarray(action)
        if a.shape != self.action_space.shape:
            raise ValueError("Action dimension mismatch")
        self._push()
        obs, r, term, trunc, info = self._b.step(torch.as_tensor(a[None], dtype=self._b.dtype))
        self._pull()
        return (self._np_obs(obs), np.float32(r[0].item()), bool(term[0]), bool(trunc[0]),
                {"is_success": np.float32(info["is_success"][0].item())})

    def close(self):
        pass

    # ---------------------------------------------------------------- reward / observation (panda_env.py:205-315)
    def _evaluate(self, achieved_goal=None, desired_goal=None):
        self._push()
        return self._b.evaluate(achieved_goal, desired_goal)

    def _get_obs(self):
        """FrankaEnv._get_obs (panda_env.py:279-301) at the current data (device: pnp_env_evaluate)."""
        out = self._evaluate()
        return {"observation": out["obs"][0].double().cpu().numpy(),
                "achieved_goal": out["achieved_goal"][0].double().cpu().numpy(),
                "desired_goal": out["desired_goal"][0].double().cpu().numpy()}

    def compute_reward(self, achieved_goal, desired_goal, info):
        """FrankaEnv.compute_reward (panda_env.py:205-245): np.float32 reward for one achieved /
        desired goal pair at the current data (device: pnp_env_evaluate)."""
        out = self._evaluate(np.asarray(achieved_goal, np.float64).reshape(1, 3),
                             np.asarray(desired_goal, np.float64).reshape(1, 3))
        return np.float32(out["reward"][0].item())

    def _is_success(self, achieved_goal, desired_goal):
        """FrankaEnv._is_success (panda_env.py:303-306)."""
        out = self._evaluate(np.asarray(achieved_goal, np.float64).reshape(1, 3),
                             np.asarray(desired_goal, np.float64).reshape(1, 3))
        return np.float32(out["is_success"][0].item())

    def slerp_track(self, start_xyzw, delta_xyzw, steps):
        """RotateSkill's target and slerp trajectory on the device (pnp_slerp_track_f64)."""
        t, trk = self._b.engine.slerp_track(start_xyzw, delta_xyzw, steps)
        return t[0], trk[0]

    @staticmethod
    def goal_distance(a, b):
        """FrankaEnv.goal_distance (panda_env.py:311-315)."""
        return np.linalg.norm(np.array(a) - np.array(b), axis=-1)

    @property
    def initial_object_height(self):
        return float(self._b.env["obj_height0"][0])

    # ---------------------------------------------------------------- helpers (panda_env.py:317-352)
    def get_ee_position(self):
        return self._utils.get_site_xpos(self.model, self.data, "ee_center_site")

    def get_ee_orientation(self):
        q = np.zeros(4)
        self._mujoco.mju_mat2Quat(q, self.data.site_xmat[self.model.site_id("ee_center_site")])
        return q

    def get_fingers_width(self):
        """finger_joint1 + finger_joint2 qpos, a shape-(1,) array like the reference's."""
        return (self._utils.get_joint_qpos(self.model, self.data, "finger_joint1")
                + self._utils.get_joint_qpos(self.model, self.data, "finger_joint2"))

    def set_mocap_pose(self, pos, quat):
        self._utils.set_mocap_pos(self.model, self.data, "panda_mocap", pos)
        self._utils.set_mocap_quat(self.model, self.data, "panda_mocap", quat)

    def set_joint_neutral(self):
        names = [f"joint{i}" for i in range(1, 8)] + ["finger_joint1", "finger_joint2"]
        for name, v in zip(names, self.neutral_joint_values):
            self._utils.set_joint_qpos(self.model, self.data, name, v)

    @property
    def current_task_index(self):
        return int(self._b.env["task"][0])

    @property
    def goal(self):
        return self._b.env["goal"][0].double().cpu().numpy()


def make(env_id, **kwargs):
    """gym.make("FrankaShelfPNP{Dense,Sparse}-v0") replacement (__init__.py:6-18)."""
    if env_id not in ENV_IDS:
        raise KeyError(f"unknown env id {env_id!r}; registered: {ENV_IDS}")
    reward_type = "dense" if env_id == "FrankaShelfPNPDense-v0" else "sparse"
    return FrankaShelfPNPEnv(reward_type=reward_type, **kwargs)
