/*
 * oracle.c — CPU fp64 restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product path (libpnp.so) never links,
 * loads or falls back to it.
 *
 * What it restates:
 *   - MuJoCo 2.3.3 mj_kinematics (tree FK incl. mocap and free joints, body/site frames) and
 *     mj_jacSite's translational Jacobian.  MuJoCo is a third-party dependency absent from
 *     /root/reference (requirements.txt:1 pins mujoco==2.3.3); the algorithm is restated from
 *     its published engine (engine_core_smooth.c mj_kinematics, engine_util_spatial.c
 *     mju_mulQuat / mju_rotVecQuat / mju_quat2Mat / mju_mat2Quat / mju_axisAngle2Quat) and
 *     pinned by the reference's own known answer: FK(ee_center_site, neutral q) =
 *     [1.23843967, 0, 0.49740014] (scripts/execute_pnp.py:38, test/reward_test.py:47 with the
 *     neutral pose of envs/panda_env.py:64-66).
 *   - JacobianIKController.solve, reference skills/ik_solver.py:35-101, control flow verbatim:
 *     convergence test before the update (:63-67), DLS step J^T (J J^T + damping I)^-1 e
 *     (:78-79, numpy.linalg.solve = LU with partial pivoting), per-joint clip to +-step_limit
 *     then to jnt_range (:80-81), iterations = i+1 (:66,85), final position measured after the
 *     last update (:88-89), success = converged && err < 2 thr (:92).
 *     Pinned by golden vectors produced by running that very function (tests/golden/).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pnp.h"

#define MINVAL 1e-15

/* ------------------------------------------------------------------ spatial helpers (MuJoCo) */
static void mulquat(double r[4], const double a[4], const double b[4]) {
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}

static void normalize4(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - 1) > MINVAL) {
    double s = 1.0 / n;
    q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
  }
}

static void rotvecquat(double r[3], const double v[3], const double q[4]) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) {
    r[0] = r[1] = r[2] = 0;
    return;
  }
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2];
    return;
  }
  double t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
  double t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
  double t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
  r[0] = v[0] + 2 * (q[2] * t2 - q[3] * t1);
  r[1] = v[1] + 2 * (q[3] * t0 - q[1] * t2);
  r[2] = v[2] + 2 * (q[1] * t1 - q[2] * t0);
}

static void quat2mat(double m[9], const double q[4]) {
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    memset(m, 0, 9 * sizeof(double));
    m[0] = m[4] = m[8] = 1;
    return;
  }
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33;
  m[4] = q00 - q11 + q22 - q33;
  m[8] = q00 - q11 - q22 + q33;
  m[1] = 2 * (q12 - q03);
  m[2] = 2 * (q13 + q02);
  m[3] = 2 * (q12 + q03);
  m[5] = 2 * (q23 - q01);
  m[6] = 2 * (q13 - q02);
  m[7] = 2 * (q23 + q01);
}

static void axisangle2quat(double r[4], const double ax[3], double ang) {
  if (ang == 0) {
    r[0] = 1; r[1] = r[2] = r[3] = 0;
    return;
  }
  double s = sin(ang * 0.5);
  r[0] = cos(ang * 0.5);
  r[1] = ax[0] * s; r[2] = ax[1] * s; r[3] = ax[2] * s;
}

static void mulmatvec3(double r[3], const double m[9], const double v[3]) {
  double t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

/* mju_mat2Quat (trace / largest-diagonal branch, then normalise); reference call site
 * envs/panda_env.py:337-342 (get_ee_orientation). */
void orc_mat2quat(double q[4], const double m[9]) {
  if (m[0] + m[4] + m[8] > 0) {
    q[0] = 0.5 * sqrt(1 + m[0] + m[4] + m[8]);
    q[1] = 0.25 * (m[7] - m[5]) / q[0];
    q[2] = 0.25 * (m[2] - m[6]) / q[0];
    q[3] = 0.25 * (m[3] - m[1]) / q[0];
  } else if (m[0] > m[4] && m[0] > m[8]) {
    q[1] = 0.5 * sqrt(1 + m[0] - m[4] - m[8]);
    q[0] = 0.25 * (m[7] - m[5]) / q[1];
    q[2] = 0.25 * (m[1] + m[3]) / q[1];
    q[3] = 0.25 * (m[2] + m[6]) / q[1];
  } else if (m[4] > m[8]) {
    q[2] = 0.5 * sqrt(1 - m[0] + m[4] - m[8]);
    q[0] = 0.25 * (m[2] - m[6]) / q[2];
    q[1] = 0.25 * (m[1] + m[3]) / q[2];
    q[3] = 0.25 * (m[5] + m[7]) / q[2];
  } else {
    q[3] = 0.5 * sqrt(1 - m[0] - m[4] + m[8]);
    q[0] = 0.25 * (m[3] - m[1]) / q[3];
    q[1] = 0.25 * (m[2] + m[6]) / q[3];
    q[2] = 0.25 * (m[5] + m[7]) / q[3];
  }
  normalize4(q);
}

/* ------------------------------------------------------------------ kinematics */
/* mj_kinematics (bodies, joint anchors/axes, sites).  Outputs may be NULL except the body
 * frame scratch: xpos[nbody*3], xquat[nbody*4], xmat[nbody*9]. */
void orc_kinematics(const pnp_model_desc* m, const double* qpos, const double* mocap_pos,
                    const double* mocap_quat, double* xpos, double* xquat, double* xmat,
                    double* xanchor, double* xaxis, double* site_xpos, double* site_xmat) {
  xpos[0] = xpos[1] = xpos[2] = 0;
  xquat[0] = 1; xquat[1] = xquat[2] = xquat[3] = 0;
  quat2mat(xmat, xquat);
  for (int i = 1; i < m->nbody; i++) {
    double p[3], q[4];
    int ja = m->body_jntadr[i], jn = m->body_jntnum[i];
    if (jn == 1 && m->jnt_type[ja] == 0) {
      const double* qp = qpos + m->jnt_qposadr[ja];
      p[0] = qp[0]; p[1] = qp[1]; p[2] = qp[2];
      q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
      normalize4(q);
      if (xanchor) memcpy(xanchor + 3 * ja, p, sizeof(p));
      if (xaxis) memcpy(xaxis + 3 * ja, m->jnt_axis + 3 * ja, 3 * sizeof(double));
    } else {
      int pid = m->body_parentid[i];
      const double *bp, *bq;
      double mq[4];
      if (m->body_mocapid[i] >= 0) {
        int k = m->body_mocapid[i];
        bp = mocap_pos ? mocap_pos + 3 * k : m->body_pos + 3 * i;
        if (mocap_quat) memcpy(mq, mocap_quat + 4 * k, sizeof(mq));
        else memcpy(mq, m->body_quat + 4 * i, sizeof(mq));
        normalize4(mq);
        bq = mq;
      } else {
        bp = m->body_pos + 3 * i;
        bq = m->body_quat + 4 * i;
      }
      if (pid) {
        mulmatvec3(p, xmat + 9 * pid, bp);
        p[0] += xpos[3 * pid]; p[1] += xpos[3 * pid + 1]; p[2] += xpos[3 * pid + 2];
        mulquat(q, xquat + 4 * pid, bq);
      } else {
        memcpy(p, bp, sizeof(p));
        memcpy(q, bq, sizeof(q));
      }
      for (int j = 0; j < jn; j++) {
        int jid = ja + j, qa = m->jnt_qposadr[jid], t = m->jnt_type[jid];
        double ax[3], an[3];
        rotvecquat(ax, m->jnt_axis + 3 * jid, q);
        rotvecquat(an, m->jnt_pos + 3 * jid, q);
        an[0] += p[0]; an[1] += p[1]; an[2] += p[2];
        if (t == 2) {
          double d = qpos[qa] - m->qpos0[qa];
          p[0] += ax[0] * d; p[1] += ax[1] * d; p[2] += ax[2] * d;
        } else if (t == 3 || t == 1) {
          double ql[4], v[3];
          if (t == 1) {
            memcpy(ql, qpos + qa, sizeof(ql));
            normalize4(ql);
          } else {
            axisangle2quat(ql, m->jnt_axis + 3 * jid, qpos[qa] - m->qpos0[qa]);
          }
          mulquat(q, q, ql);
          rotvecquat(v, m->jnt_pos + 3 * jid, q);
          p[0] = an[0] - v[0]; p[1] = an[1] - v[1]; p[2] = an[2] - v[2];
        }
        if (xanchor) memcpy(xanchor + 3 * jid, an, sizeof(an));
        if (xaxis) memcpy(xaxis + 3 * jid, ax, sizeof(ax));
      }
    }
    normalize4(q);
    memcpy(xquat + 4 * i, q, sizeof(q));
    memcpy(xpos + 3 * i, p, sizeof(p));
    quat2mat(xmat + 9 * i, q);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double v[3], q[4];
    mulmatvec3(v, xmat + 9 * b, m->site_pos + 3 * s);
    if (site_xpos) {
      site_xpos[3 * s] = xpos[3 * b] + v[0];
      site_xpos[3 * s + 1] = xpos[3 * b + 1] + v[1];
      site_xpos[3 * s + 2] = xpos[3 * b + 2] + v[2];
    }
    if (site_xmat) {
      mulquat(q, xquat + 4 * b, m->site_quat + 4 * s);
      quat2mat(site_xmat + 9 * s, q);
    }
  }
}

/* mj_jacSite translational part: column of dof d on the site's ancestor chain =
 * xaxis x (point - xanchor) for hinge, xaxis for slide, unit vectors / cross(e_k, ...) for free.
 * jacp is 3 x nv row-major. */
void orc_jac_site(const pnp_model_desc* m, const double* xanchor, const double* xaxis,
                  const double* xmat, const double* site_xpos, int site, double* jacp) {
  int nv = m->nv;
  memset(jacp, 0, 3 * nv * sizeof(double));
  const double* pt = site_xpos + 3 * site;
  for (int b = m->site_bodyid[site]; b > 0; b = m->body_parentid[b]) {
    for (int j = m->body_jntadr[b]; j >= 0 && j < m->body_jntadr[b] + m->body_jntnum[b]; j++) {
      int d = m->jnt_dofadr[j], t = m->jnt_type[j];
      const double* ax = xaxis + 3 * j;
      const double* an = xanchor + 3 * j;
      if (t == 3) {
        double r[3] = {pt[0] - an[0], pt[1] - an[1], pt[2] - an[2]};
        jacp[0 * nv + d] = ax[1] * r[2] - ax[2] * r[1];
        jacp[1 * nv + d] = ax[2] * r[0] - ax[0] * r[2];
        jacp[2 * nv + d] = ax[0] * r[1] - ax[1] * r[0];
      } else if (t == 2) {
        jacp[0 * nv + d] = ax[0];
        jacp[1 * nv + d] = ax[1];
        jacp[2 * nv + d] = ax[2];
      } else if (t == 0) {
        const double* R = xmat + 9 * b;
        double r[3] = {pt[0] - an[0], pt[1] - an[1], pt[2] - an[2]};
        for (int k = 0; k < 3; k++) jacp[k * nv + d + k] = 1;
        /* rotational dofs are in the body frame: column = (R e_k) x r */
        for (int k = 0; k < 3; k++) {
          double a[3] = {R[0 + k], R[3 + k], R[6 + k]};
          jacp[0 * nv + d + 3 + k] = a[1] * r[2] - a[2] * r[1];
          jacp[1 * nv + d + 3 + k] = a[2] * r[0] - a[0] * r[2];
          jacp[2 * nv + d + 3 + k] = a[0] * r[1] - a[1] * r[0];
        }
      }
    }
  }
}

/* mj_jacSite rotational part (jacr, 3 x nv row-major): hinge -> xaxis, slide -> 0, free joint ->
 * 0 for the translational dofs and the body-frame axes (columns of xmat) for the rotational ones */
void orc_jac_site_rot(const pnp_model_desc* m, const double* xaxis, const double* xmat, int site, double* jacr) {
  int nv = m->nv;
  memset(jacr, 0, 3 * nv * sizeof(double));
  for (int b = m->site_bodyid[site]; b > 0; b = m->body_parentid[b]) {
    for (int j = m->body_jntadr[b]; j >= 0 && j < m->body_jntadr[b] + m->body_jntnum[b]; j++) {
      int d = m->jnt_dofadr[j], t = m->jnt_type[j];
      if (t == 3) {
        for (int k = 0; k < 3; k++) jacr[k * nv + d] = xaxis[3 * j + k];
      } else if (t == 0) {
        const double* R = xmat + 9 * b;
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 3; r++) jacr[r * nv + d + 3 + k] = R[3 * r + k];
      }
    }
  }
}

/* ------------------------------------------------------------------ DLS IK */
typedef struct {
  double* xpos; double* xquat; double* xmat; double* xanchor; double* xaxis;
  double* site_xpos; double* site_xmat; double* jacp; double* qpos;
} orc_scratch;

static int scratch_alloc(const pnp_model_desc* m, orc_scratch* s) {
  s->xpos = (double*)calloc((size_t)m->nbody * 3, sizeof(double));
  s->xquat = (double*)calloc((size_t)m->nbody * 4, sizeof(double));
  s->xmat = (double*)calloc((size_t)m->nbody * 9, sizeof(double));
  s->xanchor = (double*)calloc((size_t)m->njnt * 3, sizeof(double));
  s->xaxis = (double*)calloc((size_t)m->njnt * 3, sizeof(double));
  s->site_xpos = (double*)calloc((size_t)m->nsite * 3, sizeof(double));
  s->site_xmat = (double*)calloc((size_t)m->nsite * 9, sizeof(double));
  s->jacp = (double*)calloc((size_t)m->nv * 3, sizeof(double));
  s->qpos = (double*)calloc((size_t)m->nq, sizeof(double));
  return s->xpos && s->xquat && s->xmat && s->xanchor && s->xaxis && s->site_xpos &&
         s->site_xmat && s->jacp && s->qpos ? 0 : -1;
}

static void scratch_free(orc_scratch* s) {
  free(s->xpos); free(s->xquat); free(s->xmat); free(s->xanchor); free(s->xaxis);
  free(s->site_xpos); free(s->site_xmat); free(s->jacp); free(s->qpos);
}

/* LAPACK dgesv-style LU with partial pivoting for the 3x3 system (numpy.linalg.solve). */
static void solve3_lu(double A[9], double b[3]) {
  int piv[3] = {0, 1, 2};
  for (int k = 0; k < 3; k++) {
    int p = k;
    double mx = fabs(A[3 * k + k]);
    for (int i = k + 1; i < 3; i++)
      if (fabs(A[3 * i + k]) > mx) { mx = fabs(A[3 * i + k]); p = i; }
    if (p != k) {
      for (int c = 0; c < 3; c++) { double t = A[3 * k + c]; A[3 * k + c] = A[3 * p + c]; A[3 * p + c] = t; }
      double t = b[k]; b[k] = b[p]; b[p] = t;
      int ti = piv[k]; piv[k] = piv[p]; piv[p] = ti;
    }
    double r = 1.0 / A[3 * k + k];
    for (int i = k + 1; i < 3; i++) {
      double l = A[3 * i + k] * r;
      A[3 * i + k] = l;
      for (int c = k + 1; c < 3; c++) A[3 * i + c] -= l * A[3 * k + c];
      b[i] -= l * b[k];
    }
  }
  for (int i = 2; i >= 0; i--) {
    double s = b[i];
    for (int c = i + 1; c < 3; c++) s -= A[3 * i + c] * b[c];
    b[i] = s / A[3 * i + i];
  }
}

static void site_fk(const pnp_model_desc* m, orc_scratch* s) {
  orc_kinematics(m, s->qpos, NULL, NULL, s->xpos, s->xquat, s->xmat, s->xanchor, s->xaxis,
                 s->site_xpos, NULL);
}

/* One solve; qpos_base (length nq) supplies the non-arm coordinates (NULL -> qpos0). */
static void ik_one(const pnp_model_desc* m, orc_scratch* s, int site, pnp_ik_params prm,
                   const double* q_init, const double* target, double* q_out, double* final_pos,
                   double* pos_error, int32_t* iterations, uint8_t* flags) {
  double q[7];
  int nv = m->nv;
  memcpy(q, q_init, sizeof(q));
  memcpy(s->qpos, q, sizeof(q));
  site_fk(m, s);
  int converged = 0, iters = 0;
  for (int i = 0; i < prm.max_iters; i++) {
    const double* p = s->site_xpos + 3 * site;
    double e[3] = {target[0] - p[0], target[1] - p[1], target[2] - p[2]};
    double n = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
    if (n < prm.pos_thresh) {
      converged = 1;
      iters = i + 1;
      break;
    }
    orc_jac_site(m, s->xanchor, s->xaxis, s->xmat, s->site_xpos, site, s->jacp);
    const double* J = s->jacp;
    double A[9];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        double acc = 0;
        for (int k = 0; k < nv; k++) acc += J[r * nv + k] * J[c * nv + k];
        A[3 * r + c] = acc + (r == c ? prm.damping : 0.0);
      }
    double y[3] = {e[0], e[1], e[2]};
    solve3_lu(A, y);
    for (int k = 0; k < 7; k++) {
      double dq = J[0 * nv + k] * y[0] + J[1 * nv + k] * y[1] + J[2 * nv + k] * y[2];
      dq = fmin(fmax(dq, -prm.step_limit), prm.step_limit);
      double lo = m->jnt_range[2 * k], hi = m->jnt_range[2 * k + 1];
      q[k] = fmin(fmax(q[k] + dq, lo), hi);
    }
    memcpy(s->qpos, q, sizeof(q));
    site_fk(m, s);
    iters = i + 1;
  }
  const double* fp = s->site_xpos + 3 * site;
  double d[3] = {fp[0] - target[0], fp[1] - target[1], fp[2] - target[2]};
  double err = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  memcpy(q_out, q, sizeof(q));
  memcpy(final_pos, fp, 3 * sizeof(double));
  *pos_error = err;
  *iterations = iters;
  *flags = (uint8_t)((converged ? PNP_IK_CONVERGED : 0u) |
                     ((converged && err < prm.pos_thresh * 2) ? PNP_IK_SUCCESS : 0u));
}

typedef struct {
  const pnp_model_desc* m; int site; pnp_ik_params prm;
  const double *q_init, *target; double *q_out, *final_pos, *pos_error;
  int32_t* iterations; uint8_t* flags; int b0, b1; const double* qpos_base; int rc;
} ik_job;

static void* ik_worker(void* arg) {
  ik_job* j = (ik_job*)arg;
  orc_scratch s;
  if (scratch_alloc(j->m, &s)) { j->rc = -1; return NULL; }
  for (int b = j->b0; b < j->b1; b++) {
    if (j->qpos_base) memcpy(s.qpos, j->qpos_base, j->m->nq * sizeof(double));
    else memcpy(s.qpos, j->m->qpos0, j->m->nq * sizeof(double));
    ik_one(j->m, &s, j->site, j->prm, j->q_init + 7 * b, j->target + 3 * b, j->q_out + 7 * b,
           j->final_pos + 3 * b, j->pos_error + b, j->iterations + b, j->flags + b);
  }
  scratch_free(&s);
  j->rc = 0;
  return NULL;
}

/* Batched solve over `nthreads` host threads (the CPU baseline of bench.py). */
int orc_ik_dls_batch(const pnp_model_desc* m, int site, pnp_ik_params prm, const double* q_init,
                     const double* target, double* q_out, double* final_pos, double* pos_error,
                     int32_t* iterations, uint8_t* flags, int B, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B > 0 ? B : 1;
  ik_job* jobs = (ik_job*)calloc((size_t)nthreads, sizeof(ik_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return -1; }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    ik_job j = {m, site, prm, q_init, target, q_out, final_pos, pos_error, iterations, flags,
                (int)((long)B * t / nthreads), (int)((long)B * (t + 1) / nthreads), NULL, 0};
    jobs[t] = j;
    if (nthreads == 1) ik_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, ik_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  free(jobs); free(th);
  return rc;
}

/* Batched site frames (kinematics of every body) for parity tests of pnp_site_kinematics. */
int orc_site_kinematics_batch(const pnp_model_desc* m, const double* qpos, const double* mocap_pos,
                              const double* mocap_quat, double* site_xpos, double* site_xmat,
                              int B) {
  orc_scratch s;
  if (scratch_alloc(m, &s)) return -1;
  for (int b = 0; b < B; b++) {
    orc_kinematics(m, qpos + (size_t)b * m->nq, mocap_pos ? mocap_pos + (size_t)b * 3 * m->nmocap : NULL,
                   mocap_quat ? mocap_quat + (size_t)b * 4 * m->nmocap : NULL, s.xpos, s.xquat,
                   s.xmat, s.xanchor, s.xaxis, site_xpos + (size_t)b * 3 * m->nsite,
                   site_xmat + (size_t)b * 9 * m->nsite);
  }
  scratch_free(&s);
  return 0;
}

/* Batched site Jacobian (jacp 3 x nv per env). */
int orc_jac_site_batch(const pnp_model_desc* m, int site, const double* qpos, double* jacp, int B) {
  orc_scratch s;
  if (scratch_alloc(m, &s)) return -1;
  for (int b = 0; b < B; b++) {
    orc_kinematics(m, qpos + (size_t)b * m->nq, NULL, NULL, s.xpos, s.xquat, s.xmat, s.xanchor,
                   s.xaxis, s.site_xpos, NULL);
    orc_jac_site(m, s.xanchor, s.xaxis, s.xmat, s.site_xpos, site, jacp + (size_t)b * 3 * m->nv);
  }
  scratch_free(&s);
  return 0;
}

/* Batched site frames + full site Jacobian (jacp, jacr: 3 x nv per env) at qpos (mocap pose
 * from mocap_pos / mocap_quat when given). */
int orc_site_jac2_batch(const pnp_model_desc* m, int site, const double* qpos, const double* mocap_pos,
                        const double* mocap_quat, double* site_xpos, double* site_xmat, double* jacp,
                        double* jacr, int B) {
  orc_scratch s;
  if (scratch_alloc(m, &s)) return -1;
  for (int b = 0; b < B; b++) {
    orc_kinematics(m, qpos + (size_t)b * m->nq, mocap_pos ? mocap_pos + (size_t)b * 3 * m->nmocap : NULL,
                   mocap_quat ? mocap_quat + (size_t)b * 4 * m->nmocap : NULL, s.xpos, s.xquat, s.xmat,
                   s.xanchor, s.xaxis, site_xpos + (size_t)b * 3 * m->nsite, site_xmat + (size_t)b * 9 * m->nsite);
    orc_jac_site(m, s.xanchor, s.xaxis, s.xmat, site_xpos + (size_t)b * 3 * m->nsite, site, jacp + (size_t)b * 3 * m->nv);
    orc_jac_site_rot(m, s.xaxis, s.xmat, site, jacr + (size_t)b * 3 * m->nv);
  }
  scratch_free(&s);
  return 0;
}
