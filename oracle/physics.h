/* physics.h — fp64 CPU restatement of MuJoCo 2.3.3 mj_step for the shelf_pnp scene.
 * TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline) — see oracle.c header. */
#ifndef ORC_PHYSICS_H
#define ORC_PHYSICS_H

#include <stdint.h>

#include "../include/pnp.h"

#define ORC_MAXB 24
#define ORC_MAXJ 16
#define ORC_MAXQ 40
#define ORC_MAXV 36
#define ORC_MAXU 12
#define ORC_MAXG 112
#define ORC_MAXS 12
#define ORC_MAXCON 192
#define ORC_MAXEFC 784

/* constraint types (mjtConstraint) */
#define ORC_CNSTR_EQUALITY 0
#define ORC_CNSTR_LIMIT_JOINT 3
#define ORC_CNSTR_CONTACT_PYRAMIDAL 6

/* warning bits (mjtWarning subset) — set per env, reset to model defaults like mj_resetData */
#define ORC_WARN_BADQPOS 1u
#define ORC_WARN_BADQVEL 2u
#define ORC_WARN_BADQACC 4u
#define ORC_WARN_CONTACTFULL 8u
#define ORC_WARN_CNSTRFULL 16u

typedef struct {
  double pos[3];
  double frame[9];
  double dist, includemargin;
  double friction[5];
  double solref[2], solimp[5];
  int dim, geom1, geom2, efc_address;
} orc_contact;

typedef struct {
  /* state */
  double qpos[ORC_MAXQ], qvel[ORC_MAXV], ctrl[ORC_MAXU];
  double mocap_pos[6], mocap_quat[8];
  double qacc_warmstart[ORC_MAXV];
  double time;
  uint32_t warn;
  /* position-dependent */
  double xpos[ORC_MAXB * 3], xquat[ORC_MAXB * 4], xmat[ORC_MAXB * 9];
  double xipos[ORC_MAXB * 3], ximat[ORC_MAXB * 9];
  double xanchor[ORC_MAXJ * 3], xaxis[ORC_MAXJ * 3];
  double geom_xpos[ORC_MAXG * 3], geom_xmat[ORC_MAXG * 9];
  double site_xpos[ORC_MAXS * 3], site_xmat[ORC_MAXS * 9];
  double subtree_com[ORC_MAXB * 3], cinert[ORC_MAXB * 10], cdof[ORC_MAXV * 6];
  double crb[ORC_MAXB * 10];
  double qM[ORC_MAXV * ORC_MAXV];     /* dense, symmetric, incl. armature */
  double qLD[ORC_MAXV * ORC_MAXV];    /* dense Cholesky factor (lower) of qM */
  int ncon;
  orc_contact contact[ORC_MAXCON];
  int nefc, ne;
  int efc_type[ORC_MAXEFC], efc_id[ORC_MAXEFC];
  double efc_J[ORC_MAXEFC * ORC_MAXV];
  double efc_pos[ORC_MAXEFC], efc_margin[ORC_MAXEFC], efc_diagApprox[ORC_MAXEFC];
  double efc_R[ORC_MAXEFC], efc_D[ORC_MAXEFC], efc_KBIP[ORC_MAXEFC * 4];
  /* velocity-dependent */
  double cvel[ORC_MAXB * 6], cdof_dot[ORC_MAXV * 6];
  double qfrc_bias[ORC_MAXV], qfrc_passive[ORC_MAXV];
  double efc_vel[ORC_MAXEFC], efc_aref[ORC_MAXEFC];
  /* actuation / acceleration */
  double actuator_force[ORC_MAXU], qfrc_actuator[ORC_MAXV];
  double qfrc_smooth[ORC_MAXV], qacc_smooth[ORC_MAXV];
  double efc_force[ORC_MAXEFC], efc_b[ORC_MAXEFC];
  double qfrc_constraint[ORC_MAXV], qacc[ORC_MAXV], qacc_newton[ORC_MAXV];
  int solver_iter;
  double solver_improvement, solver_gradient;
  double noslip_improvement[8];   /* MuJoCo's scaled noslip improvement of sweep k (-1: not run) */
  int noslip_iter;                /* noslip sweeps run (mj_solNoSlip's early exit) */
} orc_data;

#endif
