"""The MuJoCo-binding surface of the single-env facade.

The reference's physics boundary is the MuJoCo Python binding: the env, the
skills and the scripts reach it through ``env.unwrapped._mujoco`` / ``.model`` / ``.data`` and
gymnasium-robotics' ``mujoco_utils`` (``env.unwrapped._utils``).  This module provides those
three objects over libpnp.so, so that code written against them keeps working:

``MjData``      host mirror of one env's mjData fields the reference reads or writes (qpos, qvel,
                ctrl, act, time, mocap_pos, mocap_quat, qacc_warmstart, site_xpos, site_xmat).
                Plain numpy arrays: writes through views stick and ``copy.deepcopy(data)``
                works (reference skills/move.py:83-84).
``MujocoShim``  mj_step / mj_forward / mj_kinematics / mj_jacSite / mju_mat2Quat / mj_resetData
                on ONE env, each a device launch (pnp_step, pnp_site_kinematics,
                pnp_jac_site_full): upload the mirror, run, download.  No host physics.
``UtilsShim``   get_site_xpos / xmat / xvelp / xvelr, get/set_joint_qpos / qvel,
                set_mocap_pos / quat (gymnasium-robotics 1.2.2 mujoco_utils, as called at
                reference envs/panda_env.py:110-158, 285-293, 317-352).

MuJoCo semantics kept: ``data.site_*`` are the frames of the last forward.  After mj_step that is
the pre-integration qpos of its last sub-step (mj_step = mj_forward + integrate), or qpos0 when
that sub-step hit a bad-state reset (mj_checkPos / checkVel / checkAcc -> mj_resetData).
"""
from __future__ import annotations

import numpy as np
import torch

BAD_STATE_BITS = 7    # pnp_state.warn bits 0..2: bad qpos / qvel / qacc reset (include/pnp.h)


class MjData:
    """One env's mjData fields, host-resident (the facade's state of record between calls)."""

    def __init__(self, model):
        m = model
        mb = int((m.body_mocapid >= 0).nonzero()[0][0])
        self.qpos = np.array(m.qpos0, np.float64)
        self.qvel = np.zeros(m.nv)
        self.ctrl = np.zeros(m.nu)
        self.act = np.zeros(0)
        self.qacc_warmstart = np.zeros(m.nv)
        self.mocap_pos = np.tile(np.asarray(m.body_pos[mb], np.float64), (m.nmocap, 1))
        self.mocap_quat = np.tile(np.asarray(m.body_quat[mb], np.float64), (m.nmocap, 1))
        self.time = 0.0
        self.warn = 0                      # sticky bad-state bits (MuJoCo: data.warning counters)
        self.site_xpos = np.zeros((m.nsite, 3))
        self.site_xmat = np.zeros((m.nsite, 9))
        self.qpos_kin = self.qpos.copy()   # qpos the site frames were computed at

    STATE = ("qpos", "qvel", "ctrl", "mocap_pos", "mocap_quat", "qacc_warmstart")


class MujocoShim:
    """``mujoco`` module stand-in bound to one device engine (B = 1 launches)."""

    def __init__(self, engine, dtype=torch.float64):
        self.engine, self.dtype = engine, dtype
        self.model = engine.model
        self._st = engine.new_state(1, dtype)

    # ---------------------------------------------------------------- mirror <-> device
    # One packed host->device copy per upload and one device->host copy per download (each
    # pageable copy is a synchronisation: per-field copies made a BT tick ~20 round trips).
    def upload(self, data, st=None):
        st = self._st if st is None else st
        parts = [np.ascontiguousarray(getattr(data, k), np.float64).reshape(-1) for k in MjData.STATE]
        d = torch.from_numpy(np.concatenate(parts + [np.array([float(data.time)])])).to(self.engine.device)
        o = 0
        for k, p in zip(MjData.STATE, parts):
            st[k][0].copy_(d[o:o + p.size])
            o += p.size
        st["time"][0].copy_(d[o])
        st["warn"][0] = int(data.warn)
        return st

    def _fetch(self, tensors):
        """Device tensors -> float64 numpy arrays, in one transfer."""
        flat = torch.cat([t.reshape(-1).double() for t in tensors]).cpu().numpy()
        out, o = [], 0
        for t in tensors:
            out.append(flat[o:o + t.numel()])
            o += t.numel()
        return out

    def _store(self, data, host):
        for k in MjData.STATE:
            getattr(data, k)[...] = host[k].reshape(getattr(data, k).shape)
        data.time = float(host["time"][0])
        data.warn = int(host["warn"][0])

    def download(self, data, st=None):
        st = self._st if st is None else st
        keys = list(st.keys())
        self._store(data, dict(zip(keys, self._fetch([st[k][0] for k in keys]))))

    def frames(self, data):
        """site_xpos / site_xmat of data.qpos_kin (the last forward)."""
        t = lambda a: torch.as_tensor(np.asarray(a, np.float64).reshape(1, -1), dtype=self.dtype,
                                      device=self.engine.device)
        sx, sm = self.engine.site_kinematics(t(data.qpos_kin), t(data.mocap_pos), t(data.mocap_quat))
        data.site_xpos[...], data.site_xmat[...] = (a.reshape(data.site_xpos.shape[0], -1) for a in self._fetch([sx[0], sm[0]]))

    # ---------------------------------------------------------------- the binding's functions
    def mj_step(self, model, data, nstep=1):
        nstep = int(nstep)
        if nstep < 1:
            return
        st = self.upload(data)
        if nstep > 1:
            self.engine.step(st, nstep - 1)
        qk = st["qpos"][0:1].clone()          # the last sub-step's forward runs at this qpos
        w0 = st["warn"][0].clone()
        self.engine.step(st, 1)
        # data.site_* of the last forward, launched before the one download
        sx, sm = self.engine.site_kinematics(qk, st["mocap_pos"][0:1].contiguous(), st["mocap_quat"][0:1].contiguous())
        keys = list(st.keys())
        got = self._fetch([st[k][0] for k in keys] + [qk[0], w0, sx[0], sm[0]])
        host = dict(zip(keys, got[:len(keys)]))
        self._store(data, host)
        q_kin, w_before = got[len(keys)], int(got[len(keys) + 1][0])
        if (data.warn & BAD_STATE_BITS) & ~(w_before & BAD_STATE_BITS):
            data.qpos_kin = np.array(self.model.qpos0, np.float64)   # bad-state reset: frames at qpos0
            self.frames(data)
            return
        data.qpos_kin = np.array(q_kin, np.float64)
        data.site_xpos[...] = got[len(keys) + 2].reshape(data.site_xpos.shape)
        data.site_xmat[...] = got[len(keys) + 3].reshape(data.site_xmat.shape)

    def mj_forward(self, model, data):
        data.qpos_kin = np.array(data.qpos, np.float64)
        self.frames(data)

    def mj_kinematics(self, model, data):
        self.mj_forward(model, data)

    def mj_jacSite(self, model, data, jacp, jacr, site_id):
        t = lambda a: torch.as_tensor(np.asarray(a, np.float64).reshape(1, -1), dtype=self.dtype,
                                      device=self.engine.device)
        jp, jr = self.engine.jac_site_full(t(data.qpos_kin), int(site_id), t(data.mocap_pos), t(data.mocap_quat),
                                           want_jacp=jacp is not None, want_jacr=jacr is not None)
        if jacp is not None:
            jacp[...] = jp[0].double().cpu().numpy().reshape(np.shape(jacp))
        if jacr is not None:
            jacr[...] = jr[0].double().cpu().numpy().reshape(np.shape(jacr))

    def mju_mat2Quat(self, quat, mat):
        from .envs import mat2quat_batch
        R = torch.as_tensor(np.asarray(mat, np.float64).reshape(1, 9), dtype=torch.float64, device=self.engine.device)
        quat[...] = mat2quat_batch(R)[0].cpu().numpy()

    def mj_resetData(self, model, data):
        fresh = MjData(self.model)
        for k, v in vars(fresh).items():
            if isinstance(v, np.ndarray) and isinstance(getattr(data, k, None), np.ndarray) \
                    and getattr(data, k).shape == v.shape:
                getattr(data, k)[...] = v
            else:
                setattr(data, k, v)


class UtilsShim:
    """gymnasium-robotics ``mujoco_utils`` accessors over an MjData + MujocoShim."""

    def __init__(self, shim: MujocoShim):
        self._mj = shim
        self.model = shim.model

    def _jnt(self, name):
        m = self.model
        j = m.joint_id(name)
        n_q = {0: 7, 1: 4}.get(int(m.jnt_type[j]), 1)
        n_v = {0: 6, 1: 3}.get(int(m.jnt_type[j]), 1)
        return int(m.jnt_qposadr[j]), n_q, int(m.jnt_dofadr[j]), n_v

    def get_site_xpos(self, model, data, name):
        return data.site_xpos[self.model.site_id(name)].copy()

    def get_site_xmat(self, model, data, name):
        return data.site_xmat[self.model.site_id(name)].reshape(3, 3).copy()

    def get_site_xvelp(self, model, data, name):
        jacp = np.zeros((3, self.model.nv))
        self._mj.mj_jacSite(model, data, jacp, None, self.model.site_id(name))
        return jacp @ data.qvel

    def get_site_xvelr(self, model, data, name):
        jacr = np.zeros((3, self.model.nv))
        self._mj.mj_jacSite(model, data, None, jacr, self.model.site_id(name))
        return jacr @ data.qvel

    def get_joint_qpos(self, model, data, name):
        a, n, _, _ = self._jnt(name)
        return data.qpos[a:a + n].copy()

    def set_joint_qpos(self, model, data, name, value):
        a, n, _, _ = self._jnt(name)
        data.qpos[a:a + n] = value

    def get_joint_qvel(self, model, data, name):
        _, _, a, n = self._jnt(name)
        return data.qvel[a:a + n].copy()

    def set_joint_qvel(self, model, data, name, value):
        _, _, a, n = self._jnt(name)
        data.qvel[a:a + n] = value

    def set_mocap_pos(self, model, data, name, value):
        data.mocap_pos[int(self.model.body_mocapid[self.model.body_id(name)])] = value

    def set_mocap_quat(self, model, data, name, value):
        data.mocap_quat[int(self.model.body_mocapid[self.model.body_id(name)])] = value
