// phys_model.h — device image of the compiled model for the mj_step kernel (step.hip).
//
// Everything the step needs that does not change per env, precomputed on the host from
// pnp_model_desc (phys_host.cpp): MuJoCo's model arrays (MjModel names) plus derived index
// tables that let every stage run lane-parallel without tree-level barriers:
//   body_path      root->body chain, so each lane composes its own body's world frame
//   body_dofmask   dofs that move the body (cvel / cacc / Jacobian supports)
//   body_subtree   bodies below the body (composite inertia, force accumulation)
//   dof_velmask    dofs whose velocity enters the cvel used for the dof's cdof_dot (MuJoCo's
//                  free/ball convention: rotational dofs of one joint share one cvel)
//   trees          independent kinematic trees (arm, cube1..3, dummy) = dof ranges; M is
//                  block diagonal over trees, constraint rows touch <= 2 trees
//   pairs          geom pairs surviving MuJoCo's static collision filters, in oracle order
#pragma once

#include <stdint.h>

#define PH_MAXB 24
#define PH_MAXJ 16
#define PH_MAXV 36
#define PH_MAXQ 40
#define PH_MAXU 12
#define PH_MAXDEPTH 12
#define PH_MAXT 8
#define PH_MAXTDOF 16     // dofs per tree (arm 9)
#define PH_MAXG 48        // collidable geoms
#define PH_MAXS 12        // sites
#define PH_MAXPAIR 1024
#define PH_PAIR_PRIM 0     // primitive collider, sphere test only
#define PH_PAIR_CONVEX 1   // MPR pair: + oriented bounding boxes overlap
#define PH_PAIR_PLANE 2    // plane vs geom: + the geom's box reaches the plane
#define PH_PAIR_BOX 3      // box vs box: + the boxes (inflated by margin + 1 um) overlap
#define PH_MAXBP 256        // body pairs with at least one candidate geom pair
#define PH_MAXMESHV 1400
#define PH_MAXMESH 16
#ifndef PH_MAXCON
// The full build's capacities.  64 contacts (round 5; 48 before): the random-action gym workload's
// closed grippers peak at 57-64 contacts (tools/gym_queue_census.py: ~97 % of the envs the 48-contact
// full tier handed to the wide tier, 465-574 per 4096-env step), and the wide tier holds one env per
// CU against the full tier's 3 (Env 51.9 KB; 40.4 KB and 4 per CU at 48).
#define PH_MAXCON 64      // contacts per env (lane per contact: <= 64)
#endif
#ifndef PH_MAXEFC
#define PH_MAXEFC 272     // 6 weld + 9 limit + 4 x 64 contact rows
#endif
#ifndef PH_MAXJSLOT
#define PH_MAXJSLOT 2688  // packed constraint-Jacobian slots (sum of row widths)
#endif
#ifndef PH_JTCAP
#define PH_JTCAP 2560    // dense island Jacobian entries (sum over islands of rows x dofs; larger: slot path)
#endif
#define PH_ROWW 16        // sparse row width: dofs of <= 2 trees (arm 9 + cube 6)
#define PH_MAXMENTRY 160  // (i, j in ancestors(i)) entries of M
#define PH_MAXMBLK 256    // sum over trees of tree_dofnum^2

template <typename T>
struct DevPhys {
  int nq, nv, nu, nbody, njnt, ngeom, npair, nmocap, neq, ntree, nmentry;
  T timestep, gravity[3];
  int noslip_iterations, iterations;
  // termination of mj_solNewton / mj_solNoSlip: mjOption tolerance / noslip_tolerance, both tested
  // on values scaled by 1 / (stat.meaninertia * max(1, nv))
  T tolerance, noslip_tolerance, meaninertia;
  // bodies
  int body_parentid[PH_MAXB], body_rootid[PH_MAXB], body_weldid[PH_MAXB], body_mocapid[PH_MAXB];
  int body_jntadr[PH_MAXB], body_jntnum[PH_MAXB], body_dofadr[PH_MAXB], body_dofnum[PH_MAXB];
  int body_tree[PH_MAXB];
  int body_pathlen[PH_MAXB];
  int body_path[PH_MAXB][PH_MAXDEPTH];
  uint32_t body_subtree[PH_MAXB];
  uint64_t body_dofmask[PH_MAXB];
  T body_pos[PH_MAXB][3], body_quat[PH_MAXB][4], body_ipos[PH_MAXB][3], body_iquat[PH_MAXB][4];
  T body_mass[PH_MAXB], body_inertia[PH_MAXB][3], body_invweight0[PH_MAXB][2], body_subtreemass[PH_MAXB];
  // joints
  int jnt_type[PH_MAXJ], jnt_qposadr[PH_MAXJ], jnt_dofadr[PH_MAXJ], jnt_bodyid[PH_MAXJ], jnt_limited[PH_MAXJ];
  T jnt_pos[PH_MAXJ][3], jnt_axis[PH_MAXJ][3], jnt_range[PH_MAXJ][2], jnt_solref[PH_MAXJ][2];
  T jnt_solimp[PH_MAXJ][5], jnt_margin[PH_MAXJ];
  // dofs
  int dof_bodyid[PH_MAXV], dof_jntid[PH_MAXV], dof_parentid[PH_MAXV], dof_tree[PH_MAXV];
  uint64_t dof_velmask[PH_MAXV];
  T dof_armature[PH_MAXV], dof_damping[PH_MAXV], dof_invweight0[PH_MAXV];
  T qpos0[PH_MAXQ];
  // M sparsity: entries (i, j) with j an ancestor-or-self of i
  int mentry_i[PH_MAXMENTRY], mentry_j[PH_MAXMENTRY];
  // trees
  int tree_dofadr[PH_MAXT], tree_dofnum[PH_MAXT], tree_moff[PH_MAXT];   // M stored as per-tree dense blocks
  int nmblock;                                                         // sum of tree_dofnum^2
  // collidable geoms (compact ids 0..ngeom-1; geom_id = index in the full model)
  int geom_id[PH_MAXG], geom_type[PH_MAXG], geom_bodyid[PH_MAXG], geom_dataid[PH_MAXG];
  int geom_condim[PH_MAXG], geom_priority[PH_MAXG];
  T geom_size[PH_MAXG][3], geom_pos[PH_MAXG][3], geom_quat[PH_MAXG][4], geom_friction[PH_MAXG][3];
  T geom_solref[PH_MAXG][2], geom_solimp[PH_MAXG][5], geom_margin[PH_MAXG], geom_gap[PH_MAXG];
  T geom_solmix[PH_MAXG], geom_rbound[PH_MAXG];
  T geom_aabb[PH_MAXG][6];   // geom-frame bounding box: centre (3), half extents (3) (OBB pre-test)
  int pair_g1[PH_MAXPAIR], pair_g2[PH_MAXPAIR];   // compact geom ids, g1 has the lower type
  // broadphase table: bounding-sphere reach r1 + r2 + margin (< 0: a geom has no bounding sphere,
  // i.e. a plane), the pair margin, and the exact box test the pair gets (PH_PAIR_*)
  T pair_reach[PH_MAXPAIR], pair_margin[PH_MAXPAIR];
  unsigned char pair_kind[PH_MAXPAIR];
  // the broadphase's per-pair word: g1 | g2 << 8 | kind << 16 | body pair << 24 (one load per lane)
  uint32_t pair_pack[PH_MAXPAIR];
  // body-pair pre-cull: the candidate geom pairs grouped by their (body, body) pair; a body's
  // bounding sphere (body-frame centre body_bcen, radius body_brad covering every collidable geom's
  // bounding sphere) and the group reach R1 + R2 + max margin (< 0: a body with a plane, always
  // tested).  Result-neutral: a body pair out of reach has every geom pair out of reach.
  int nbpair;
  short bp_b1[PH_MAXBP], bp_b2[PH_MAXBP];
  T bp_reach[PH_MAXBP];
  T body_bcen[PH_MAXB][3], body_brad[PH_MAXB];
  // meshes (convex hulls)
  int mesh_vertadr[PH_MAXMESH], mesh_vertnum[PH_MAXMESH];
  T mesh_vert[PH_MAXMESHV][3];
  // actuators (joint transmission)
  int act_trnid[PH_MAXU], act_biastype[PH_MAXU], act_ctrllimited[PH_MAXU], act_forcelimited[PH_MAXU];
  int act_dof[PH_MAXU], act_qadr[PH_MAXU];
  T act_gear[PH_MAXU], act_gainprm[PH_MAXU][3], act_biasprm[PH_MAXU][3];
  T act_ctrlrange[PH_MAXU][2], act_forcerange[PH_MAXU][2];
  int dof_act[PH_MAXV];   // the one actuator driving the dof, -1 none, -2 several (summed in order)
  // equality (weld)
  int eq_type[4], eq_obj1id[4], eq_obj2id[4];
  T eq_solref[4][2], eq_solimp[4][5], eq_data[4][11];
  // mocap defaults (mj_resetData)
  int mocap_body[4];
  // sites (gym observation / action frames)
  int nsite;
  int site_bodyid[PH_MAXS];
  T site_pos[PH_MAXS][3], site_quat[PH_MAXS][4];
  // fp64 copies of the kinematic chain's constants (per body: offset, its one joint) and of the
  // first weld's data.  The fp32 build carries the weld bodies' poses in fp64 as well
  // (st_kinematics -> weld_pose_f64, st_constraints): the weld (solref 0.01) turns a 1e-7 m
  // position rounding of fp32 kinematics into a 2e-3 m/s^2 error of its reference acceleration,
  // the dominant fp32 error of the arm's constrained acceleration (DESIGN.md §2, fp32 precision).
  double kd_body_pos[PH_MAXB][3], kd_body_quat[PH_MAXB][4];
  double kd_jnt_pos[PH_MAXB][3], kd_jnt_axis[PH_MAXB][3], kd_qpos0[PH_MAXB];
  double kd_eq_data[11];
  int weld_eq, weld_body[2];   // the first weld equality and its bodies (-1: none)
  int multiccd;   // mjENBL_MULTICCD (mjc_Convex's perturbed contacts)
};
