// kinematics.hip — batched mj_kinematics (site frames) and mj_jacSite (jacp / jacr), one thread per env.
//
// Reference call sites replaced: skills/ik_solver.py:58-59 and 70-72 (mj_kinematics, site_xpos,
// mj_jacSite), envs/panda_env.py:285-293 and 337-346 (site_xpos / site_xmat / jacSite reads of
// _get_obs, get_ee_position, get_ee_orientation).  Formulas follow MuJoCo 2.3.3 mj_kinematics
// (quaternion composition, mocap bodies, free joints) exactly as restated in oracle/oracle.c.
//
// These are the general-tree kernels (any body / site, free joints, mocap).  They are not the
// throughput path — the IK kernel (ik_dls.hip) carries its own specialised chain FK.
#include "pnp_internal.h"

// Full-tree FK into per-thread frames.  Body frames are kept in registers/scratch: the tree
// has 20 bodies, the kernels are one-thread-per-env and not HBM-bound.
template <typename T>
__device__ void d_kinematics(const DevModel<T>& m, const T* qpos, const T* mocap_pos,
                             const T* mocap_quat, T (*xpos)[3], T (*xquat)[4],
                             T (*xanchor)[3], T (*xaxis)[3]) {
  xpos[0][0] = xpos[0][1] = xpos[0][2] = 0;
  xquat[0][0] = 1; xquat[0][1] = xquat[0][2] = xquat[0][3] = 0;
  for (int i = 1; i < m.nbody; i++) {
    T p[3], q[4];
    const int ja = m.body_jntadr[i], jn = m.body_jntnum[i];
    if (jn == 1 && m.jnt_type[ja] == 0) {
      const T* qp = qpos + m.jnt_qposadr[ja];
      p[0] = qp[0]; p[1] = qp[1]; p[2] = qp[2];
      q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
      d_normalize4(q);
      if (xanchor) { xanchor[ja][0] = p[0]; xanchor[ja][1] = p[1]; xanchor[ja][2] = p[2]; }
      if (xaxis) { xaxis[ja][0] = m.jnt_axis[ja][0]; xaxis[ja][1] = m.jnt_axis[ja][1]; xaxis[ja][2] = m.jnt_axis[ja][2]; }
    } else {
      const int pid = m.body_parentid[i];
      T bp[3], bq[4];
      const int mid = m.body_mocapid[i];
      if (mid >= 0 && mocap_pos) {
        bp[0] = mocap_pos[3 * mid]; bp[1] = mocap_pos[3 * mid + 1]; bp[2] = mocap_pos[3 * mid + 2];
      } else {
        bp[0] = m.body_pos[i][0]; bp[1] = m.body_pos[i][1]; bp[2] = m.body_pos[i][2];
      }
      if (mid >= 0 && mocap_quat) {
        bq[0] = mocap_quat[4 * mid]; bq[1] = mocap_quat[4 * mid + 1];
        bq[2] = mocap_quat[4 * mid + 2]; bq[3] = mocap_quat[4 * mid + 3];
        d_normalize4(bq);
      } else {
        bq[0] = m.body_quat[i][0]; bq[1] = m.body_quat[i][1];
        bq[2] = m.body_quat[i][2]; bq[3] = m.body_quat[i][3];
      }
      if (pid) {
        T pm[9];
        d_quat2mat(pm, xquat[pid]);
        d_mulmatvec3(p, pm, bp);
        p[0] += xpos[pid][0]; p[1] += xpos[pid][1]; p[2] += xpos[pid][2];
        d_mulquat(q, xquat[pid], bq);
      } else {
        p[0] = bp[0]; p[1] = bp[1]; p[2] = bp[2];
        q[0] = bq[0]; q[1] = bq[1]; q[2] = bq[2]; q[3] = bq[3];
      }
      for (int j = 0; j < jn; j++) {
        const int jid = ja + j, qa = m.jnt_qposadr[jid], t = m.jnt_type[jid];
        T ax[3], an[3];
        d_rotvecquat(ax, m.jnt_axis[jid], q);
        d_rotvecquat(an, m.jnt_pos[jid], q);
        an[0] += p[0]; an[1] += p[1]; an[2] += p[2];
        if (t == 2) {
          T d = qpos[qa] - m.qpos0[qa];
          p[0] += ax[0] * d; p[1] += ax[1] * d; p[2] += ax[2] * d;
        } else if (t == 3 || t == 1) {
          T ql[4], v[3];
          if (t == 1) {
            ql[0] = qpos[qa]; ql[1] = qpos[qa + 1]; ql[2] = qpos[qa + 2]; ql[3] = qpos[qa + 3];
            d_normalize4(ql);
          } else {
            T ang = qpos[qa] - m.qpos0[qa];
            if (ang == T(0)) {
              ql[0] = 1; ql[1] = ql[2] = ql[3] = 0;
            } else {
              T s, c;
              d_sincos(ang * T(0.5), &s, &c);
              ql[0] = c; ql[1] = m.jnt_axis[jid][0] * s; ql[2] = m.jnt_axis[jid][1] * s;
              ql[3] = m.jnt_axis[jid][2] * s;
            }
          }
          d_mulquat(q, q, ql);
          d_rotvecquat(v, m.jnt_pos[jid], q);
          p[0] = an[0] - v[0]; p[1] = an[1] - v[1]; p[2] = an[2] - v[2];
        }
        if (xanchor) { xanchor[jid][0] = an[0]; xanchor[jid][1] = an[1]; xanchor[jid][2] = an[2]; }
        if (xaxis) { xaxis[jid][0] = ax[0]; xaxis[jid][1] = ax[1]; xaxis[jid][2] = ax[2]; }
      }
    }
    d_normalize4(q);
    xquat[i][0] = q[0]; xquat[i][1] = q[1]; xquat[i][2] = q[2]; xquat[i][3] = q[3];
    xpos[i][0] = p[0]; xpos[i][1] = p[1]; xpos[i][2] = p[2];
  }
}

template <typename T>
__global__ void __launch_bounds__(64) site_kinematics_kernel(
    const DevModel<T>* __restrict__ mp, const T* __restrict__ qpos, const T* __restrict__ mocap_pos,
    const T* __restrict__ mocap_quat, T* __restrict__ site_xpos, T* __restrict__ site_xmat, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const DevModel<T>& m = *mp;
  T xpos[PNP_MAXBODY][3], xquat[PNP_MAXBODY][4];
  d_kinematics<T>(m, qpos + (size_t)b * m.nq, mocap_pos ? mocap_pos + (size_t)b * 3 * m.nmocap : nullptr,
                  mocap_quat ? mocap_quat + (size_t)b * 4 * m.nmocap : nullptr, xpos, xquat,
                  nullptr, nullptr);
  for (int s = 0; s < m.nsite; s++) {
    const int bd = m.site_bodyid[s];
    T bm[9], v[3];
    d_quat2mat(bm, xquat[bd]);
    d_mulmatvec3(v, bm, m.site_pos[s]);
    if (site_xpos) {
      T* o = site_xpos + ((size_t)b * m.nsite + s) * 3;
      o[0] = xpos[bd][0] + v[0]; o[1] = xpos[bd][1] + v[1]; o[2] = xpos[bd][2] + v[2];
    }
    if (site_xmat) {
      T q[4], sm[9];
      d_mulquat(q, xquat[bd], m.site_quat[s]);
      d_quat2mat(sm, q);
      T* o = site_xmat + ((size_t)b * m.nsite + s) * 9;
      for (int k = 0; k < 9; k++) o[k] = sm[k];
    }
  }
}

// mj_jacSite: translational (jacp) and rotational (jacr) Jacobian of `site` over all dofs.  A dof
// moves the site only if its joint is an ancestor of the site's body; free / ball joints turn
// about the body frame's axes (columns of xmat), as cdof does.
template <typename T>
__global__ void __launch_bounds__(64) jac_site_kernel(const DevModel<T>* __restrict__ mp, int site,
                                                     const T* __restrict__ qpos,
                                                     const T* __restrict__ mocap_pos,
                                                     const T* __restrict__ mocap_quat,
                                                     T* __restrict__ jacp, T* __restrict__ jacr, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const DevModel<T>& m = *mp;
  T xpos[PNP_MAXBODY][3], xquat[PNP_MAXBODY][4], xanchor[PNP_MAXJNT][3], xaxis[PNP_MAXJNT][3];
  d_kinematics<T>(m, qpos + (size_t)b * m.nq, mocap_pos ? mocap_pos + (size_t)b * 3 * m.nmocap : nullptr,
                  mocap_quat ? mocap_quat + (size_t)b * 4 * m.nmocap : nullptr, xpos, xquat, xanchor, xaxis);
  const int sb = m.site_bodyid[site];
  T bm[9], v[3], pt[3];
  d_quat2mat(bm, xquat[sb]);
  d_mulmatvec3(v, bm, m.site_pos[site]);
  pt[0] = xpos[sb][0] + v[0]; pt[1] = xpos[sb][1] + v[1]; pt[2] = xpos[sb][2] + v[2];
  const int nv = m.nv;
  T* Jp = jacp ? jacp + (size_t)b * 3 * nv : nullptr;
  T* Jr = jacr ? jacr + (size_t)b * 3 * nv : nullptr;
  for (int k = 0; k < 3 * nv; k++) {
    if (Jp) Jp[k] = 0;
    if (Jr) Jr[k] = 0;
  }
  // one rotational axis a at dof d: jacr column a, jacp column a x (site - anchor)
  auto put = [&](int d, const T* a, const T* r) {
    if (Jp) {
      Jp[0 * nv + d] = a[1] * r[2] - a[2] * r[1];
      Jp[1 * nv + d] = a[2] * r[0] - a[0] * r[2];
      Jp[2 * nv + d] = a[0] * r[1] - a[1] * r[0];
    }
    if (Jr) { Jr[0 * nv + d] = a[0]; Jr[1 * nv + d] = a[1]; Jr[2 * nv + d] = a[2]; }
  };
  for (int bd = sb; bd > 0; bd = m.body_parentid[bd]) {
    for (int j = m.body_jntadr[bd]; j >= 0 && j < m.body_jntadr[bd] + m.body_jntnum[bd]; j++) {
      const int d = m.jnt_dofadr[j], t = m.jnt_type[j];
      const T r[3] = {pt[0] - xanchor[j][0], pt[1] - xanchor[j][1], pt[2] - xanchor[j][2]};
      if (t == 3) {
        put(d, xaxis[j], r);
      } else if (t == 2) {
        if (Jp) { Jp[0 * nv + d] = xaxis[j][0]; Jp[1 * nv + d] = xaxis[j][1]; Jp[2 * nv + d] = xaxis[j][2]; }
      } else {   // free (3 translational + 3 rotational dofs) or ball (3 rotational)
        T R[9];
        d_quat2mat(R, xquat[bd]);
        const int dr = t == 0 ? d + 3 : d;
        if (t == 0 && Jp)
          for (int k = 0; k < 3; k++) Jp[k * nv + d + k] = 1;
        for (int k = 0; k < 3; k++) {
          const T a[3] = {R[0 + k], R[3 + k], R[6 + k]};
          put(dr + k, a, r);
        }
      }
    }
  }
}

template <typename T>
static int32_t launch_site_kinematics(pnp_model* model, const T* qpos, const T* mocap_pos,
                                      const T* mocap_quat, T* site_xpos, T* site_xmat, int32_t B,
                                      void* stream, const DevModel<T>* dm) {
  if (!model || !qpos || B < 0) { pnp_set_error("pnp_site_kinematics: bad argument"); return PNP_ERR_ARG; }
  if (B == 0) return PNP_OK;
  hipLaunchKernelGGL(site_kinematics_kernel<T>, dim3((B + 63) / 64), dim3(64), 0,
                     (hipStream_t)stream, dm, qpos, mocap_pos, mocap_quat, site_xpos, site_xmat, B);
  return pnp_check_launch("site_kinematics_kernel");
}

template <typename T>
static int32_t launch_jac_site(pnp_model* model, int32_t site, const T* qpos, T* jacp, int32_t B,
                               void* stream, const DevModel<T>* dm) {
  if (!model || !qpos || !jacp || B < 0 || site < 0 || site >= model->h.nsite) {
    pnp_set_error("pnp_jac_site: bad argument");
    return PNP_ERR_ARG;
  }
  if (B == 0) return PNP_OK;
  hipLaunchKernelGGL(jac_site_kernel<T>, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, dm,
                     site, qpos, (const T*)nullptr, (const T*)nullptr, jacp, (T*)nullptr, B);
  return pnp_check_launch("jac_site_kernel");
}

template <typename T>
static int32_t launch_jac_site_full(pnp_model* model, int32_t site, const T* qpos, const T* mocap_pos,
                                    const T* mocap_quat, T* jacp, T* jacr, int32_t B, void* stream,
                                    const DevModel<T>* dm) {
  if (!model || !qpos || (!jacp && !jacr) || B < 0 || site < 0 || site >= model->h.nsite) {
    pnp_set_error("pnp_jac_site_full: bad argument");
    return PNP_ERR_ARG;
  }
  if (B == 0) return PNP_OK;
  hipLaunchKernelGGL(jac_site_kernel<T>, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, dm,
                     site, qpos, mocap_pos, mocap_quat, jacp, jacr, B);
  return pnp_check_launch("jac_site_kernel");
}

extern "C" int32_t pnp_site_kinematics(pnp_model* model, const float* qpos, const float* mocap_pos,
                                       const float* mocap_quat, float* site_xpos, float* site_xmat,
                                       int32_t B, void* stream) {
  return launch_site_kinematics<float>(model, qpos, mocap_pos, mocap_quat, site_xpos, site_xmat, B,
                                       stream, model ? model->d_f32 : nullptr);
}

extern "C" int32_t pnp_site_kinematics_f64(pnp_model* model, const double* qpos,
                                           const double* mocap_pos, const double* mocap_quat,
                                           double* site_xpos, double* site_xmat, int32_t B,
                                           void* stream) {
  return launch_site_kinematics<double>(model, qpos, mocap_pos, mocap_quat, site_xpos, site_xmat,
                                        B, stream, model ? model->d_f64 : nullptr);
}

extern "C" int32_t pnp_jac_site(pnp_model* model, int32_t site_id, const float* qpos, float* jacp,
                                int32_t B, void* stream) {
  return launch_jac_site<float>(model, site_id, qpos, jacp, B, stream, model ? model->d_f32 : nullptr);
}

extern "C" int32_t pnp_jac_site_f64(pnp_model* model, int32_t site_id, const double* qpos,
                                    double* jacp, int32_t B, void* stream) {
  return launch_jac_site<double>(model, site_id, qpos, jacp, B, stream, model ? model->d_f64 : nullptr);
}

extern "C" int32_t pnp_jac_site_full(pnp_model* model, int32_t site_id, const float* qpos,
                                     const float* mocap_pos, const float* mocap_quat, float* jacp,
                                     float* jacr, int32_t B, void* stream) {
  return launch_jac_site_full<float>(model, site_id, qpos, mocap_pos, mocap_quat, jacp, jacr, B, stream,
                                     model ? model->d_f32 : nullptr);
}

extern "C" int32_t pnp_jac_site_full_f64(pnp_model* model, int32_t site_id, const double* qpos,
                                         const double* mocap_pos, const double* mocap_quat,
                                         double* jacp, double* jacr, int32_t B, void* stream) {
  return launch_jac_site_full<double>(model, site_id, qpos, mocap_pos, mocap_quat, jacp, jacr, B, stream,
                                      model ? model->d_f64 : nullptr);
}
