"""Batched behaviour-tree runs: B copies of the reference's pick-and-place
demo (scripts/execute_pnp.py + behavior_tree/trees/pnp_tree.py:20-42) on B envs of ONE batched
device env, stepped together.

Every env runs the reference's control logic unchanged -- its own behaviour tree (pnp_amd.bt),
skills (pnp_amd.skills) and MoveIK waypoint planner (skills/move.py:95-191) -- in its own host
thread, against a per-env view of the batched env (``EnvView``: the facade's API).  A view never
touches the device: every physics, IK or slerp request a skill makes blocks its thread and goes
to the ``PhysicsServer``, which waits until every live env is blocked (or finished), then serves
all pending requests of a kind with ONE launch over the envs that made them:

  * ``env.step(action)`` (GripperSkill)       pnp_env_step on the gathered sub-batch
  * ``mj_step(model, data, n)`` (_step_sim,   pnp_step on the gathered sub-batch (n - 1, then 1
    execute_pnp's extra sub-steps)            sub-step: data.site_* are the last sub-step's forward)
  * ``JacobianIKController.solve`` (the       pnp_ik_dls over every planner's solve of the round
    MoveIK planners)                          (the C2 hot path, lockstep like BatchedMoveIKPlanner)
  * RotateSkill.reset's slerp                 pnp_slerp_track for every reset of the round

then refreshes the host caches (qpos, site frames) and releases the threads.  Per env the run is
the sequential facade run's (same env index, same Philox reset draws, envs independent in every
kernel): tests/test_bt_gpu.py compares tick counts and success with sequential facade runs.
"""
from __future__ import annotations

import threading
import types

import numpy as np
import torch

from .bt import DEFAULT_SKILLS
from .envs import BatchedFrankaShelfPNPEnv, Box, EnvConfig
from .execute_pnp import run_on
from .ik_solver import IKResult
from .mjshim import BAD_STATE_BITS, MujocoShim
from .skills.move import MoveIKSkill, plan_ik_waypoints


class _Request:
    __slots__ = ("b", "kind", "args", "result", "error", "done")

    def __init__(self, b, kind, args):
        self.b, self.kind, self.args = b, kind, args
        self.result, self.error, self.done = None, None, False


class PhysicsServer:
    """Owns the batched env; serves the views' blocking requests in batched launches."""

    def __init__(self, num_envs, reward_type="dense", env_offset=0, device=None, dtype=torch.float64,
                 config: EnvConfig | None = None):
        self.env = BatchedFrankaShelfPNPEnv(num_envs, reward_type, device=device, dtype=dtype, autoreset=False,
                                            env_offset=env_offset, config=config)
        self.engine, self.model, self.B = self.env.engine, self.env.model, num_envs
        self.shim = MujocoShim(self.engine, dtype)          # mju_mat2Quat: the facade's own code path
        self.ee_site = self.model.site_id("ee_center_site")
        self._cv = threading.Condition()
        self._pending = {}
        self._finished = set()
        self._errors = {}
        self.rounds = 0
        self.launches = {"gym": 0, "mj_step": 0, "ik": 0, "slerp": 0}
        # mocap is host state of record (the views' set_mocap_pose), uploaded before every physics
        # launch and taken back from the device after a gym step (whose _set_action writes it);
        # everything else lives on the device and is mirrored after each physics round
        st = self.env.state
        self.mocap_pos = st["mocap_pos"].double().cpu().numpy()
        self.mocap_quat = st["mocap_quat"].double().cpu().numpy()
        self.refresh()

    # ------------------------------------------------------------------ host mirrors
    def refresh(self):
        st = self.env.state
        self.qpos = st["qpos"].double().cpu().numpy()
        self.qvel = st["qvel"].double().cpu().numpy()
        sx, sm = self.engine.site_kinematics(self.env.env["qpos_kin"], st["mocap_pos"], st["mocap_quat"])
        self.site_xpos = sx.double().cpu().numpy()
        self.site_xmat = sm.double().cpu().numpy()

    def reset(self):
        self.env.reset()
        st = self.env.state
        self.mocap_pos = st["mocap_pos"].double().cpu().numpy()
        self.mocap_quat = st["mocap_quat"].double().cpu().numpy()
        self.refresh()

    def _upload_mocap(self):
        st = self.env.state
        st["mocap_pos"].copy_(torch.as_tensor(self.mocap_pos, dtype=st["mocap_pos"].dtype))
        st["mocap_quat"].copy_(torch.as_tensor(self.mocap_quat, dtype=st["mocap_quat"].dtype))

    # ------------------------------------------------------------------ requests (view threads)
    def request(self, b, kind, *args):
        r = _Request(b, kind, args)
        with self._cv:
            self._pending[b] = r
            self._cv.notify_all()
            while not r.done:
                self._cv.wait()
        if r.error is not None:
            raise r.error
        return r.result

    def _thread_main(self, b, fn):
        try:
            fn()
        except BaseException as e:   # noqa: BLE001 (re-raised by run())
            self._errors[b] = e
        finally:
            with self._cv:
                self._finished.add(b)
                self._cv.notify_all()

    def run(self, programs):
        """Run ``programs[b]()`` for every env in its own thread, serving their requests in
        batched rounds until all have returned."""
        self._finished, self._errors = set(), {}
        threads = [threading.Thread(target=self._thread_main, args=(b, fn), daemon=True) for b, fn in enumerate(programs)]
        for t in threads:
            t.start()
        n = len(threads)
        while True:
            with self._cv:
                while len(self._pending) + len(self._finished) < n:
                    self._cv.wait()
                if len(self._finished) == n:
                    break
                batch, self._pending = self._pending, {}
            try:
                self._serve(batch)
            except BaseException as e:   # noqa: BLE001 (handed to every waiting thread)
                for r in batch.values():
                    r.error = e
            with self._cv:
                for r in batch.values():
                    r.done = True
                self._cv.notify_all()
        for t in threads:
            t.join()
        if self._errors:
            b, e = sorted(self._errors.items())[0]
            raise RuntimeError(f"env {b}: {type(e).__name__}: {e}") from e

    # ------------------------------------------------------------------ serving
    def _serve(self, batch):
        self.rounds += 1
        kinds = {}
        for r in batch.values():
            kinds.setdefault(r.kind, []).append(r)
        physics = False
        for r_list in (kinds.get("slerp", []),):
            by_steps = {}
            for r in r_list:
                by_steps.setdefault(int(r.args[2]), []).append(r)
            for steps, rs in by_steps.items():
                tgt, trk = self.engine.slerp_track([r.args[0] for r in rs], [r.args[1] for r in rs], steps)
                self.launches["slerp"] += 1
                for i, r in enumerate(rs):
                    r.result = (tgt[i], trk[i])
        by_prm = {}
        for r in kinds.get("ik", []):
            by_prm.setdefault(tuple(r.args[2]), []).append(r)
        for prm, rs in by_prm.items():
            dev = self.engine.device
            q0 = torch.as_tensor(np.stack([np.asarray(r.args[1], np.float64).reshape(7) for r in rs]), device=dev)
            tg = torch.as_tensor(np.stack([np.asarray(r.args[0], np.float64).reshape(3) for r in rs]), device=dev)
            out = self.engine.ik_dls(q0.contiguous(), tg.contiguous(), site=self.ee_site, max_iters=prm[0],
                                     pos_thresh=prm[1], damping=prm[2], step_limit=prm[3])
            self.launches["ik"] += 1
            q, fp = out["q"].double().cpu().numpy(), out["final_pos"].double().cpu().numpy()
            err, it, fl = (out["pos_error"].double().cpu().numpy(), out["iterations"].cpu().numpy(),
                           out["flags"].cpu().numpy().astype(np.int64))
            for i, r in enumerate(rs):
                r.result = IKResult(success=bool(fl[i] & 2), q=q[i].copy(), final_pos=fp[i].copy(),
                                    pos_error=float(err[i]), iterations=int(it[i]), converged=bool(fl[i] & 1))
        if "gym" in kinds or "mj_step" in kinds:
            physics = True
            self._upload_mocap()
        if "gym" in kinds:
            rs = kinds["gym"]
            ids = [r.b for r in rs]
            out = self.env.step_subset(ids, np.stack([np.asarray(r.args[0], np.float32) for r in rs]))
            self.launches["gym"] += 1
            # _set_action wrote these envs' mocap pose (the facade downloads it into data.mocap_*)
            self.mocap_pos[ids] = self.env.state["mocap_pos"][ids].double().cpu().numpy()
            self.mocap_quat[ids] = self.env.state["mocap_quat"][ids].double().cpu().numpy()
            host = {k: v.double().cpu().numpy() for k, v in out.items()}
            for i, r in enumerate(rs):
                obs = {"observation": host["obs"][i], "achieved_goal": host["achieved_goal"][i],
                       "desired_goal": host["desired_goal"][i]}
                r.result = (obs, np.float32(host["reward"][i]), bool(host["terminated"][i]), bool(host["truncated"][i]),
                            {"is_success": np.float32(host["is_success"][i])})
        by_n = {}
        for r in kinds.get("mj_step", []):
            by_n.setdefault(int(r.args[0]), []).append(r)
        st, m = self.env.state, self.model
        for n, rs in by_n.items():
            # MujocoShim.mj_step on the sub-batch: n - 1 sub-steps, the last one's pre-integration
            # qpos kept as data.site_*'s (qpos0 after a bad-state reset), then the last sub-step
            idx = torch.as_tensor([r.b for r in rs], dtype=torch.long, device=self.engine.device)
            sub = {k: v.index_select(0, idx).contiguous() for k, v in st.items()}
            if n > 1:
                self.engine.step(sub, n - 1)
            qk = sub["qpos"].clone()
            w0 = sub["warn"].clone()
            self.engine.step(sub, 1)
            self.launches["mj_step"] += 1 + (n > 1)
            newbad = ((sub["warn"] & BAD_STATE_BITS) & ~(w0 & BAD_STATE_BITS)) != 0
            if bool(newbad.any()):
                qk[newbad] = torch.as_tensor(np.asarray(m.qpos0, np.float64), dtype=qk.dtype, device=qk.device)
            for k, v in sub.items():
                st[k].index_copy_(0, idx, v)
            self.env.env["qpos_kin"].index_copy_(0, idx, qk)
            for r in rs:
                r.result = None
        if physics:
            self.refresh()


# ---------------------------------------------------------------------------- per-env view
class _ViewData:
    """The slice of MjData the skills read (qpos / qvel snapshots of the env's row)."""

    def __init__(self, view):
        self._v = view

    @property
    def qpos(self):
        return self._v.server.qpos[self._v.b].copy()

    @property
    def qvel(self):
        return self._v.server.qvel[self._v.b].copy()


class _ViewMujoco:
    def __init__(self, view):
        self._v = view

    def mj_step(self, model, data, nstep=1):
        if int(nstep) >= 1:
            self._v.server.request(self._v.b, "mj_step", int(nstep))


class _ViewUtils:
    def __init__(self, view):
        self._v = view

    def get_site_xpos(self, model, data, name):
        return self._v.server.site_xpos[self._v.b, self._v.model.site_id(name)].copy()

    def get_site_xmat(self, model, data, name):
        return self._v.server.site_xmat[self._v.b, self._v.model.site_id(name)].reshape(3, 3).copy()


class _ServerIK:
    """JacobianIKController.solve through the server (batched with the other envs' solves)."""

    def __init__(self, view):
        self._v = view

    def solve(self, target_pos, q_init, max_iters=100, pos_thresh=1e-3, damping=1e-2, step_limit=0.1):
        return self._v.server.request(self._v.b, "ik", np.asarray(target_pos, np.float64),
                                      np.asarray(q_init, np.float64), (int(max_iters), float(pos_thresh),
                                                                       float(damping), float(step_limit)))


class EnvView:
    """Env b of the server's batch behind the single-env facade's API (the part the behaviour
    tree, the skills and execute_pnp use: reset state, gym step, mocap, site frames, mj_step)."""

    def __init__(self, server: PhysicsServer, b: int, task_sequence):
        self.server, self.b = server, b
        self.model = server.model
        self.data = _ViewData(self)
        self._mujoco = _ViewMujoco(self)
        self._utils = _ViewUtils(self)
        self.ik = _ServerIK(self)
        self.action_space = Box(-1.0, 1.0, (7,))
        self.render_mode = None
        self.task_sequence = list(task_sequence)
        self.home_pos = self.get_ee_position().copy()     # (the facade sets it at reset)

    @property
    def unwrapped(self):
        return self

    def step(self, action):
        a = np.asarray(action)
        if a.shape != self.action_space.shape:
            raise ValueError("Action dimension mismatch")
        return self.server.request(self.b, "gym", a)

    def get_ee_position(self):
        return self.server.site_xpos[self.b, self.server.ee_site].copy()

    def get_ee_orientation(self):
        q = np.zeros(4)
        self.server.shim.mju_mat2Quat(q, self.server.site_xmat[self.b, self.server.ee_site])
        return q

    def get_fingers_width(self):
        m, q = self.model, self.server.qpos[self.b]
        a1 = int(m.jnt_qposadr[m.joint_id("finger_joint1")])
        a2 = int(m.jnt_qposadr[m.joint_id("finger_joint2")])
        return q[a1:a1 + 1] + q[a2:a2 + 1]

    def set_mocap_pose(self, pos, quat):
        self.server.mocap_pos[self.b] = np.asarray(pos, np.float64).reshape(3)
        self.server.mocap_quat[self.b] = np.asarray(quat, np.float64).reshape(4)

    def slerp_track(self, start_xyzw, delta_xyzw, steps):
        return self.server.request(self.b, "slerp", np.asarray(start_xyzw, np.float64),
                                   np.asarray(delta_xyzw, np.float64), int(steps))


class ServerMoveIKSkill(MoveIKSkill):
    """MoveIKSkill whose planner solves through the server (reference skills/move.py:76-191:
    the same planner, plan_ik_waypoints; its scratch MjData copy is not needed)."""

    def reset(self):
        self.i = 0
        self.done = False
        u = self.env.unwrapped
        self.pos_traj, self.quat_traj = plan_ik_waypoints(
            u.ik, self.env.get_ee_position().copy(), self.env.get_ee_orientation().copy(), u.data.qpos[:7].copy(),
            self.target_pos, self.pos_thresh, self.max_traj_points, self.step_size, log=lambda *a: None)


SERVER_SKILLS = types.SimpleNamespace(RotateSkill=DEFAULT_SKILLS.RotateSkill, MoveIKSkill=ServerMoveIKSkill,
                                      MoveSkill=DEFAULT_SKILLS.MoveSkill, GripperSkill=DEFAULT_SKILLS.GripperSkill)


def run_batched(num_envs, env_id="FrankaShelfPNPDense-v0", max_tick=3000, sim_steps=5, task_sequence=None,
                env_offset=0, device=None):
    """scripts/execute_pnp.py for envs env_offset .. env_offset + num_envs - 1 at once.  Returns
    per-env success and tick counts plus the server's round / launch counts."""
    reward_type = "dense" if env_id == "FrankaShelfPNPDense-v0" else "sparse"
    server = PhysicsServer(num_envs, reward_type, env_offset=env_offset, device=device)
    server.reset()
    seq = list(task_sequence) if task_sequence else ["cube1", "cube2", "cube3"]
    views = [EnvView(server, b, seq) for b in range(num_envs)]
    success = np.zeros(num_envs, bool)
    ticks = np.zeros(num_envs, np.int64)

    def program(b):
        def fn():
            s, t, _ = run_on(views[b], max_tick, sim_steps, False, skills=SERVER_SKILLS)
            success[b], ticks[b] = s, t
        return fn

    server.run([program(b) for b in range(num_envs)])
    objects = {n: server.site_xpos[:, server.model.site_id(f"{n}_site")].copy() for n in seq}
    warn = (server.env.state["warn"].to(torch.int64) & 0xFFFF).cpu().numpy()   # sticky warning bits per env
    return {"success": success, "ticks": ticks, "rounds": server.rounds, "launches": dict(server.launches),
            "objects": objects, "warn": warn}
