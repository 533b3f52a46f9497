"""Model-derived constants (MuJoCo 2.3.3 ``mj_setConst``, run by its compiler at qpos0).

* ``dof_parentid``: parent dof in the kinematic tree (sparsity of M).
* ``dof_invweight0``: diag(M^-1) at qpos0, averaged over the 3 translational / 3 rotational dofs
  of a free joint — the diagonal approximation used for joint-limit rows' regulariser.
* ``body_invweight0``: mean diagonal of J M^-1 J^T for the body's COM (translational and
  rotational 3x3 blocks separately) at qpos0, 0 for static bodies — used for equality and
  contact rows' ``efc_diagApprox`` (reference call sites: every mj_step).
* ``stat_meaninertia``: mjStatistic.meaninertia, the mean of diag(M) at qpos0 (armature
  included), which scales the Newton and no-slip termination tests.

M here is assembled independently of the engine's CRBA, as the Jacobian sum
``M = sum_b Jp_b^T m_b Jp_b + Jr_b^T I_b Jr_b + diag(armature)`` over body COMs, in numpy.
"""
from __future__ import annotations

import numpy as np

from .mjcf import quat2mat


def _quat_mul(a, b):
    return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                     a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                     a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                     a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def forward_frames(m, qpos):
    """Body frames, joint anchors/axes (numpy restatement of mj_kinematics)."""
    nb = int(m["nbody"])
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    nj = int(m["njnt"])
    xanchor = np.zeros((nj, 3))
    xaxis = np.zeros((nj, 3))
    for i in range(1, nb):
        ja, jn = int(m["body_jntadr"][i]), int(m["body_jntnum"][i])
        if jn == 1 and m["jnt_type"][ja] == 0:
            a = int(m["jnt_qposadr"][ja])
            p = qpos[a:a + 3].copy()
            q = qpos[a + 3:a + 7] / np.linalg.norm(qpos[a + 3:a + 7])
            xanchor[ja] = p
            xaxis[ja] = m["jnt_axis"][ja]
        else:
            pid = int(m["body_parentid"][i])
            p = xpos[pid] + quat2mat(xquat[pid]) @ m["body_pos"][i]
            q = _quat_mul(xquat[pid], m["body_quat"][i])
            for j in range(ja, ja + jn):
                R = quat2mat(q)
                ax = R @ m["jnt_axis"][j]
                an = p + R @ m["jnt_pos"][j]
                a = int(m["jnt_qposadr"][j])
                if m["jnt_type"][j] == 2:
                    p = p + ax * (qpos[a] - m["qpos0"][a])
                elif m["jnt_type"][j] == 3:
                    ang = qpos[a] - m["qpos0"][a]
                    ql = np.concatenate([[np.cos(ang / 2)], m["jnt_axis"][j] * np.sin(ang / 2)])
                    q = _quat_mul(q, ql)
                    p = an - quat2mat(q) @ m["jnt_pos"][j]
                xanchor[j] = an
                xaxis[j] = ax
        q = q / np.linalg.norm(q)
        xpos[i], xquat[i] = p, q
    return xpos, xquat, xanchor, xaxis


def body_jacobians(m, qpos, points=None):
    """(Jp [nbody,3,nv], Jr [nbody,3,nv]) of each body's COM (or of given world points)."""
    xpos, xquat, xanchor, xaxis = forward_frames(m, qpos)
    nb, nv = int(m["nbody"]), int(m["nv"])
    Jp = np.zeros((nb, 3, nv))
    Jr = np.zeros((nb, 3, nv))
    for b in range(1, nb):
        pt = xpos[b] + quat2mat(xquat[b]) @ m["body_ipos"][b] if points is None else points[b]
        c = b
        while c > 0:
            ja, jn = int(m["body_jntadr"][c]), int(m["body_jntnum"][c])
            for j in range(ja, ja + jn) if ja >= 0 else []:
                d = int(m["jnt_dofadr"][j])
                t = m["jnt_type"][j]
                if t == 3:
                    Jr[b, :, d] = xaxis[j]
                    Jp[b, :, d] = np.cross(xaxis[j], pt - xanchor[j])
                elif t == 2:
                    Jp[b, :, d] = xaxis[j]
                elif t == 0:
                    R = quat2mat(xquat[c])
                    for k in range(3):
                        Jp[b, k, d + k] = 1.0
                        Jr[b, :, d + 3 + k] = R[:, k]
                        Jp[b, :, d + 3 + k] = np.cross(R[:, k], pt - xanchor[j])
            c = int(m["body_parentid"][c])
    return Jp, Jr, xpos, xquat


def mass_matrix(m, qpos):
    """Joint-space inertia by the Jacobian sum (independent of the engine's CRBA)."""
    Jp, Jr, xpos, xquat = body_jacobians(m, qpos)
    nv = int(m["nv"])
    M = np.zeros((nv, nv))
    for b in range(1, int(m["nbody"])):
        if m["body_mass"][b] == 0:
            continue
        Ri = quat2mat(xquat[b]) @ quat2mat(m["body_iquat"][b])
        Iw = Ri @ np.diag(m["body_inertia"][b]) @ Ri.T
        M += m["body_mass"][b] * Jp[b].T @ Jp[b] + Jr[b].T @ Iw @ Jr[b]
    M[np.diag_indices(nv)] += m["dof_armature"]
    return M


def compute(m):
    """Returns the extra arrays (dof_parentid, dof_invweight0, body_invweight0, body_subtreemass,
    body_treedepth) and the model statistic stat_meaninertia."""
    nv, nb, nj = int(m["nv"]), int(m["nbody"]), int(m["njnt"])
    # dof_parentid: previous dof of the same joint, else last dof of the nearest ancestor body
    dof_parentid = -np.ones(nv, np.int32)
    last_dof = -np.ones(nb, np.int32)
    for b in range(1, nb):
        par = int(m["body_parentid"][b])
        prev = last_dof[par]
        for d in range(int(m["body_dofadr"][b]), int(m["body_dofadr"][b]) + int(m["body_dofnum"][b])) \
                if m["body_dofadr"][b] >= 0 else []:
            dof_parentid[d] = prev
            prev = d
        last_dof[b] = prev
    qpos0 = np.asarray(m["qpos0"], np.float64)
    M = mass_matrix(m, qpos0)
    Minv = np.linalg.inv(M)
    dof_invweight0 = np.zeros(nv)
    for j in range(nj):
        d = int(m["jnt_dofadr"][j])
        t = m["jnt_type"][j]
        if t == 0:
            dof_invweight0[d:d + 3] = np.mean(np.diag(Minv)[d:d + 3])
            dof_invweight0[d + 3:d + 6] = np.mean(np.diag(Minv)[d + 3:d + 6])
        elif t == 1:
            dof_invweight0[d:d + 3] = np.mean(np.diag(Minv)[d:d + 3])
        else:
            dof_invweight0[d] = Minv[d, d]
    Jp, Jr, _, _ = body_jacobians(m, qpos0)
    body_invweight0 = np.zeros((nb, 2))
    for b in range(1, nb):
        if m["body_weldid"][b] == 0:
            continue
        J = np.concatenate([Jp[b], Jr[b]], 0)
        A = J @ Minv @ J.T
        body_invweight0[b] = [np.trace(A[:3, :3]) / 3, np.trace(A[3:, 3:]) / 3]
    subtreemass = np.array(m["body_mass"], np.float64).copy()
    for b in range(nb - 1, 0, -1):
        subtreemass[int(m["body_parentid"][b])] += subtreemass[b]
    depth = np.zeros(nb, np.int32)
    for b in range(1, nb):
        depth[b] = depth[int(m["body_parentid"][b])] + 1
    # mjStatistic.meaninertia: the mean diagonal of M at qpos0 (armature included); mj_solNewton and
    # mj_solNoSlip scale their termination tests by 1 / (meaninertia * max(1, nv))
    stat_meaninertia = float(np.mean(np.diag(M))) if nv else 1.0
    return dict(dof_parentid=dof_parentid, dof_invweight0=dof_invweight0, body_invweight0=body_invweight0,
                body_subtreemass=subtreemass, body_treedepth=depth, stat_meaninertia=stat_meaninertia)
