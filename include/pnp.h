/*
 * pnp.h — C ABI of libpnp.so, the MI355X-native batched kinematics / DLS-IK / env-step engine
 * for the panda_mujoco_gym shelf pick-and-place scene.
 *
 * The reference crosses one boundary for all of its hot-path arithmetic: the MuJoCo Python
 * binding (mj_step / mj_forward / mj_kinematics / mj_jacSite / mju_mat2Quat, MjModel, MjData).
 * Each entry point below replaces one of those call sites, batched over B independent envs
 * (SURVEY.md §8b).  Conventions:
 *   - every call returns int32 status: 0 ok, <0 error; pnp_last_error() gives a thread-local
 *     message.  No C++ exception crosses the ABI.
 *   - all batch buffers are CALLER-OWNED DEVICE pointers (e.g. torch.Tensor.data_ptr()),
 *     structure-of-arrays, row-major [B, n], fp32 (the _f64 variants: fp64, for debugging and
 *     bit-level parity against the CPU oracle).
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream);
 *     every call is asynchronous and stream-ordered; no host synchronisation inside.
 *   - model descriptions are HOST pointers read once by pnp_model_create.
 *   - quaternions are MuJoCo wxyz; matrices row-major 3x3.
 */
#ifndef PNP_H
#define PNP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNP_ABI_VERSION 14

#define PNP_OK 0
#define PNP_ERR_ARG -1
#define PNP_ERR_HIP -2
#define PNP_ERR_MODEL -3
#define PNP_ERR_UNSUPPORTED -4

/* Compiled model, MjModel field names (subset the scene needs).  Produced by the host MJCF
 * compiler (mujoco-panda-pnp_amd/pnp_amd/mjcf.py) from assets/shelf_pnp.xml; replaces
 * MjModel.from_xml_path (reference envs/panda_env.py:108).  All reals are float64. */
typedef struct pnp_model_desc {
  int32_t nq, nv, nu, nbody, njnt, ngeom, nsite, nmocap, neq, nmesh, nmeshvert;
  /* <option> (assets/shelf_pnp.xml:4-6) */
  double timestep;
  double gravity[3];
  int32_t noslip_iterations, iterations;
  double tolerance;
  int32_t cone_pyramidal, multiccd, warmstart, integrator_euler;
  /* mjOption noslip_tolerance (default 1e-6) and mjStatistic meaninertia (mj_setConst: mean of
   * diag(M) at qpos0, armature included): mj_solNewton / mj_solNoSlip scale their improvement and
   * gradient tests by 1 / (meaninertia * max(1, nv)) */
  double noslip_tolerance, stat_meaninertia;
  /* bodies [nbody] */
  const int32_t* body_parentid;
  const int32_t* body_rootid;
  const int32_t* body_weldid;
  const int32_t* body_mocapid;
  const int32_t* body_jntadr;
  const int32_t* body_jntnum;
  const int32_t* body_dofadr;
  const int32_t* body_dofnum;
  const double* body_pos;     /* [nbody*3] */
  const double* body_quat;    /* [nbody*4] */
  const double* body_ipos;    /* [nbody*3] */
  const double* body_iquat;   /* [nbody*4] */
  const double* body_mass;    /* [nbody]   */
  const double* body_inertia; /* [nbody*3] */
  const double* body_invweight0;   /* [nbody*2] mj_setConst: mean diag of J M^-1 J^T (tran, rot) */
  const double* body_subtreemass;  /* [nbody] */
  const int32_t* body_treedepth;   /* [nbody] depth below the world (world = 0) */
  /* joints [njnt]: type 0 free, 1 ball, 2 slide, 3 hinge (mjtJoint) */
  const int32_t* jnt_type;
  const int32_t* jnt_qposadr;
  const int32_t* jnt_dofadr;
  const int32_t* jnt_bodyid;
  const int32_t* jnt_limited;
  const double* jnt_pos;      /* [njnt*3] */
  const double* jnt_axis;     /* [njnt*3] */
  const double* jnt_range;    /* [njnt*2] */
  const double* jnt_solref;   /* [njnt*2] solreflimit */
  const double* jnt_solimp;   /* [njnt*5] solimplimit */
  const double* jnt_margin;   /* [njnt]   */
  /* dofs [nv] */
  const int32_t* dof_jntid;
  const int32_t* dof_bodyid;
  const double* dof_armature;
  const double* dof_damping;
  const int32_t* dof_parentid;  /* [nv] parent dof in the tree, -1 at a tree root */
  const double* dof_invweight0; /* [nv] mj_setConst: diag(M^-1) at qpos0 (free joints averaged) */
  const double* qpos0;        /* [nq] */
  /* geoms [ngeom]: type 0 plane, 2 sphere, 6 box, 7 mesh (mjtGeom) */
  const int32_t* geom_type;
  const int32_t* geom_bodyid;
  const int32_t* geom_contype;
  const int32_t* geom_conaffinity;
  const int32_t* geom_condim;
  const int32_t* geom_priority;
  const int32_t* geom_dataid;  /* mesh id or -1 */
  const double* geom_size;     /* [ngeom*3] */
  const double* geom_pos;      /* [ngeom*3] */
  const double* geom_quat;     /* [ngeom*4] */
  const double* geom_friction; /* [ngeom*3] */
  const double* geom_solref;   /* [ngeom*2] */
  const double* geom_solimp;   /* [ngeom*5] */
  const double* geom_margin;
  const double* geom_gap;
  const double* geom_solmix;
  const double* geom_rbound;   /* bounding-sphere radius (0 for planes) */
  /* convex-hull meshes */
  const int32_t* mesh_vertadr; /* [nmesh] */
  const int32_t* mesh_vertnum; /* [nmesh] */
  const double* mesh_vert;     /* [nmeshvert*3], in the geom frame */
  /* sites [nsite] */
  const int32_t* site_bodyid;
  const double* site_pos;      /* [nsite*3] */
  const double* site_quat;     /* [nsite*4] */
  /* actuators [nu]: general, joint transmission, affine bias */
  const int32_t* actuator_trnid;
  const int32_t* actuator_biastype;
  const int32_t* actuator_ctrllimited;
  const int32_t* actuator_forcelimited;
  const double* actuator_gear;       /* [nu]   (gear[0]) */
  const double* actuator_gainprm;    /* [nu*3] */
  const double* actuator_biasprm;    /* [nu*3] */
  const double* actuator_ctrlrange;  /* [nu*2] */
  const double* actuator_forcerange; /* [nu*2] */
  /* equality [neq]: type 1 = weld */
  const int32_t* eq_type;
  const int32_t* eq_obj1id;
  const int32_t* eq_obj2id;
  const double* eq_solref;     /* [neq*2]  */
  const double* eq_solimp;     /* [neq*5]  */
  const double* eq_data;       /* [neq*11] anchor(3) relpos(3) relquat(4) torquescale(1) */
} pnp_model_desc;

/* Parameters of JacobianIKController.solve (reference skills/ik_solver.py:35-37). */
typedef struct pnp_ik_params {
  int32_t max_iters;   /* default 100  */
  double pos_thresh;   /* default 1e-3 */
  double damping;      /* default 1e-2 (added as damping*I3, ik_solver.py:79) */
  double step_limit;   /* default 0.1  */
} pnp_ik_params;

/* flags[b] bits written by pnp_ik_dls* (IKResult.converged / IKResult.success,
 * reference skills/ik_solver.py:16-24, 88-92) */
#define PNP_IK_CONVERGED 1u
#define PNP_IK_SUCCESS 2u

typedef struct pnp_model pnp_model;  /* opaque device-resident model */

int32_t pnp_abi_version(void);
/* sizeof(pnp_model_desc) as compiled into the library: lets bindings check their struct layout. */
int32_t pnp_model_desc_size(void);
const char* pnp_last_error(void);

/* Replaces MjModel.from_xml_path + JacobianIKController.__init__ constants (reference
 * envs/panda_env.py:108-109, skills/ik_solver.py:27-33): copies the model constants to the
 * current HIP device (fp32 and fp64 images). */
int32_t pnp_model_create(const pnp_model_desc* desc, pnp_model** out);
int32_t pnp_model_destroy(pnp_model* model);
/* Host-only validation of a model description (no HIP call): builds every host-side image
 * pnp_model_create would upload (kinematics tables, both precisions' physics images) and reports
 * the first capacity / consistency error.  0 = the step kernel accepts the model. */
int32_t pnp_model_check(const pnp_model_desc* desc);

/* Batched mj_kinematics restricted to what the hot path reads (site frames), reference
 * skills/ik_solver.py:58-59, envs/panda_env.py:285-291,344-346, 337-342 (site_xpos / site_xmat).
 *   qpos[B*nq], mocap_pos[B*nmocap*3] (may be NULL), mocap_quat[B*nmocap*4] (may be NULL)
 *   -> site_xpos[B*nsite*3], site_xmat[B*nsite*9] (either may be NULL). */
int32_t pnp_site_kinematics(pnp_model* model, const float* qpos, const float* mocap_pos,
                            const float* mocap_quat, float* site_xpos, float* site_xmat,
                            int32_t B, void* stream);
int32_t pnp_site_kinematics_f64(pnp_model* model, const double* qpos, const double* mocap_pos,
                                const double* mocap_quat, double* site_xpos, double* site_xmat,
                                int32_t B, void* stream);

/* Batched position Jacobian of a site (mj_jacSite jacp, reference skills/ik_solver.py:70-72):
 *   qpos[B*nq] -> jacp[B*3*nv] (row-major 3 x nv per env). */
int32_t pnp_jac_site(pnp_model* model, int32_t site_id, const float* qpos, float* jacp,
                     int32_t B, void* stream);
int32_t pnp_jac_site_f64(pnp_model* model, int32_t site_id, const double* qpos, double* jacp,
                         int32_t B, void* stream);

/* Full mj_jacSite (reference skills/ik_solver.py:70-72, and gymnasium-robotics get_site_xvelp /
 * get_site_xvelr behind envs/panda_env.py:285-293): translational and rotational Jacobians of a
 * site, mocap bodies placed from mocap_pos / mocap_quat (either may be NULL: model pose).
 *   qpos[B*nq] -> jacp[B*3*nv], jacr[B*3*nv] (row-major 3 x nv per env; either may be NULL). */
int32_t pnp_jac_site_full(pnp_model* model, int32_t site_id, const float* qpos, const float* mocap_pos,
                          const float* mocap_quat, float* jacp, float* jacr, int32_t B, void* stream);
int32_t pnp_jac_site_full_f64(pnp_model* model, int32_t site_id, const double* qpos,
                              const double* mocap_pos, const double* mocap_quat, double* jacp,
                              double* jacr, int32_t B, void* stream);

/* Batched JacobianIKController.solve (reference skills/ik_solver.py:35-101), one solve per env:
 *   q_init[B*7], target[B*3] -> q_out[B*7], final_pos[B*3], pos_error[B], iterations[B],
 *   flags[B] (PNP_IK_CONVERGED | PNP_IK_SUCCESS).
 * The site must hang below the 7 arm hinges (ee_center_site); joints 0..6 are the ones solved,
 * limits are jnt_range[0..6].  Other qpos entries do not affect the site and are not read. */
int32_t pnp_ik_dls(pnp_model* model, int32_t site_id, pnp_ik_params params, const float* q_init,
                   const float* target, float* q_out, float* final_pos, float* pos_error,
                   int32_t* iterations, uint8_t* flags, int32_t B, void* stream);
int32_t pnp_ik_dls_f64(pnp_model* model, int32_t site_id, pnp_ik_params params,
                       const double* q_init, const double* target, double* q_out,
                       double* final_pos, double* pos_error, int32_t* iterations, uint8_t* flags,
                       int32_t B, void* stream);


/* ------------------------------------------------------------------ physics step (mj_step) */
/* Per-env simulation state, SoA device arrays [B, n] (MjData fields of the same names). */
typedef struct pnp_state {
  float* qpos;            /* [B*nq] */
  float* qvel;            /* [B*nv] */
  float* ctrl;            /* [B*nu] */
  float* mocap_pos;       /* [B*nmocap*3] */
  float* mocap_quat;      /* [B*nmocap*4] wxyz */
  float* qacc_warmstart;  /* [B*nv] */
  float* time;            /* [B] */
  uint32_t* warn;         /* [B] PNP_WARN_* bits, sticky */
} pnp_state;
typedef struct pnp_state_f64 {
  double* qpos; double* qvel; double* ctrl; double* mocap_pos; double* mocap_quat;
  double* qacc_warmstart; double* time; uint32_t* warn;
} pnp_state_f64;

/* warn bits (mjtWarning subset); bad state triggers mj_resetData semantics for that env */
#define PNP_WARN_BADQPOS 1u
#define PNP_WARN_BADQVEL 2u
#define PNP_WARN_BADQACC 4u
#define PNP_WARN_CONTACTFULL 8u
#define PNP_WARN_CNSTRFULL 16u
/* bits 16..31 are reserved: inside one fp32 pnp_step / pnp_env_step call they carry a
 * capacity tier's hand-over to the next tier (flag + sub-step); they are clear when a call
 * returns and are ignored on input */

/* nsub x mj_step on every env, in place (reference envs/panda_env.py:355-358 calls this with
 * nsub = 25, ten times; skills/base.py:43 and scripts/execute_pnp.py:103 with nsub = 1).
 * ctrl and mocap are held constant over the nsub sub-steps, as in the reference.
 * fp32: three capacity tiers of one kernel source -- compact (20 contacts, 8 envs per CU), full
 * (64 contacts, 3 per CU), wide (192 contacts, 1 per CU).  Each runs the envs the previous tier
 * handed over, from the sub-step that would have overflowed its capacities, so results equal the
 * wide kernel's bit for bit; only the wide tier truncates (PNP_WARN_CONTACTFULL / CNSTRFULL).
 * fp64 (the single-env facade, the batched behaviour trees, debugging): the full kernel, whose
 * overflowing sub-steps the fp64 wide tier resumes (96 contacts, 400 rows, 1 per CU), truncating
 * past that.  Solver exits: MuJoCo 2.3.3's (Newton: one line search per iteration, stop on scaled
 * improvement or gradient < tolerance; noslip: stop on scaled sweep improvement < noslip_tolerance;
 * scale = 1 / (stat_meaninertia * nv)); the fp32 tiers solve each constraint island to its
 * minimiser (fp32 cannot resolve the 1e-8 scaled tolerance) and share the noslip exit.
 * Environment variables (A/B runs and tests): PNP_STEP_COMPACT=0 starts at the full tier,
 * 3 runs the wide kernel alone, 2 the compact kernel alone (a test diagnostic that leaves
 * handed-over envs mid-call); PNP_STEP_WIDE=0 drops the wide tier (the full kernel truncates). */
int32_t pnp_step(pnp_model* model, const pnp_state* state, int32_t B, int32_t nsub, void* stream);
int32_t pnp_step_f64(pnp_model* model, const pnp_state_f64* state, int32_t B, int32_t nsub, void* stream);

/* Debug/parity: one mj_forward per env (state not advanced), dumping intermediates into
 * dbg[B * PNP_DBG_SIZE] (float64, device, zero-initialised by the caller) at the offsets below.
 * The forward runs through the step's tiers: the full kernel, and for the envs whose forward
 * outgrows it the wide kernel (fp32: 192 contacts / 784 rows; fp64: 96 / 400), truncating past
 * that like pnp_step (PNP_STEP_WIDE=0: the full kernel alone, truncating at 64 / 272).  ABI 14:
 * the record holds the wide tier's capacities (ABI 13's held 48 contacts / 208 rows, less than the
 * full tier's 64 / 272 since round 5: larger forwards wrote past their record). */
#define PNP_DBG_QM 0            /* nv*nv dense joint-space inertia (incl. armature) */
#define PNP_DBG_BIAS 1296       /* qfrc_bias[nv] */
#define PNP_DBG_ACT 1332        /* qfrc_actuator[nv] */
#define PNP_DBG_QACC_SMOOTH 1368
#define PNP_DBG_QACC 1404
#define PNP_DBG_COUNTS 1440     /* ncon, nefc, solver iterations, warn */
#define PNP_DBG_CON 1444        /* ncon (<= 192) x 16: pos3 frame9 dist geom1 geom2 dim */
#define PNP_DBG_CON_STRIDE 16
#define PNP_DBG_EFC_FORCE 4516  /* nefc (<= 784) */
#define PNP_DBG_EFC_POS 5300
#define PNP_DBG_EFC_D 6084
#define PNP_DBG_EFC_AREF 6868
#define PNP_DBG_EFC_TYPE 7652
#define PNP_DBG_EFC_J 8436      /* nefc x nv dense */
#define PNP_DBG_QACC_NEWTON 36660 /* Newton result before no-slip */
#define PNP_DBG_NOSLIP_ITER 36696 /* no-slip sweeps run (mj_solNoSlip's early exit) */
#define PNP_DBG_SIZE 36700
#define PNP_DBG_MAXCON 192
#define PNP_DBG_MAXEFC 784
int32_t pnp_forward_debug(pnp_model* model, const pnp_state* state, int32_t B, double* dbg, void* stream);
int32_t pnp_forward_debug_f64(pnp_model* model, const pnp_state_f64* state, int32_t B, double* dbg,
                              void* stream);
/* Diagnostic: pnp_step with per-stage shader-clock cycles accumulated into
 * stage_cycles[B * PNP_NSTAGE] (uint64, device, caller zeroes).  Stages: check, kinematics,
 * comPos+CRB, factor M, collision, constraints, velocity+RNE, actuation+smooth, Newton setup
 * (islands, warm start), Newton gradient+Hessian, Newton direction (island Cholesky), Newton line
 * search, Newton update+convergence, noslip, finish accel, Euler; then sub-stages (cycles
 * also counted in their parent): broadphase, primitive narrowphase, convex (MPR) pairs, noslip
 * W = M^-1 J^T, noslip pair lists, kinematics per-body prologue, kinematics tree levels,
 * kinematics inertial/geom frames, Newton gradient, Newton convergence test, Newton Hessian; then per-sub-step counts summed over the sub-steps (not
 * cycles): ncon, nefc, Newton iterations, live convex pairs, islands, noslip sweep length,
 * broadphase survivors; then 8 ad-hoc sub-stage timers (aux0..aux7, cycles; what each brackets is
 * stated at its sub_lap call in csrc/step.hip); then three more counts: noslip sub-steps on the
 * dense long-list path and on the streaming path, noslip sweeps run.  Separate instantiation: the
 * product kernel carries no timers. */
#define PNP_NSTAGE 45
#define PNP_NSTAGE_CYCLES 27
int32_t pnp_step_profile(pnp_model* model, const pnp_state* state, int32_t B, int32_t nsub,
                         unsigned long long* stage_cycles, void* stream);
/* LDS bytes one env occupies in the step kernel (fp64 != 0: the debug instantiation). */
int32_t pnp_step_lds_bytes(int32_t fp64);

/* ------------------------------------------------------------------ gym env (FrankaEnv) */
/* Batched FrankaShelfPNPEnv: the reference's gym surface (envs/panda_env.py, envs/shelf_pnp.py)
 * with the whole gym step fused into one launch per batch.  Replaces, per env:
 *   pnp_env_init   FrankaEnv.__init__ -> _initialize_simulation / _env_setup (panda_env.py:106-141)
 *                  + _initialize_multi_object_task (:100-104)
 *   pnp_env_reset  FrankaEnv.reset -> _reset_sim (:366-391), _sample_object (:146-158),
 *                  _sample_goal (:360-364), then _get_obs (:279-301)
 *   pnp_env_step   FrankaEnv.step (:163-196): clip, _set_action (:250-277), _mujoco_step (10 x
 *                  mj_step(nstep=25), :355-358), _get_obs, _is_success (:303-306),
 *                  compute_reward (:205-245), task sequencing, TimeLimit(300) truncation
 *                  (__init__.py:15).
 * "data.site_*" semantics are kept: the observation's positions / Jacobians come from the
 * kinematics of the last forward (the pre-integration qpos of the last sub-step, or the reset
 * state), velocities are J * qvel with the integrated qvel, finger width reads integrated qpos. */
#define PNP_MAX_TASKS 4
#define PNP_OBS_DIM 19
typedef struct pnp_env_params {
  int32_t n_substeps;          /* 25 (shelf_pnp.py:19) */
  int32_t n_calls;             /* 10 mj_step calls per gym step (panda_env.py:357) */
  int32_t reward_dense;        /* 1: dense reward, 0: sparse */
  int32_t max_episode_steps;   /* TimeLimit (300); <= 0: never truncate */
  int32_t n_tasks;             /* len(task_sequence) (3) */
  int32_t ee_site;             /* ee_center_site */
  int32_t obj_site[PNP_MAX_TASKS];     /* "<obj>_site" per task */
  int32_t target_site[PNP_MAX_TASKS];  /* "target_<obj>" per task */
  int32_t obj_qadr[PNP_MAX_TASKS];     /* qpos address of "<obj>_joint" (free joint) */
  int32_t finger_qadr[2];      /* finger_joint1 / finger_joint2 qpos addresses */
  int32_t neutral_qadr[9];     /* arm + gripper joint qpos addresses (set_joint_neutral) */
  int32_t height_qadr;         /* qpos address of obj_joint (initial_object_height = z) */
  int32_t arm_ctrl_n;          /* ctrl[0:arm_ctrl_n] = neutral at setup (7) */
  double neutral[9];           /* neutral_joint_values (panda_env.py:64-66) */
  double distance_threshold;   /* 0.05 */
  double high_pick_z;          /* 0.35 */
  double grip_width;           /* 0.045 */
  double reach_thresh;         /* 0.05: gripped needs d_reach < this; reach penalty cap */
  double lift_height;          /* 0.04 */
  double obj_x_range, obj_y_range;   /* 0.02, 0.2 (shelf_pnp.py:23-24) */
  double pos_scale;            /* 0.05 (ee target = ee_pos + pos_scale * a[0:3]) */
  double rot_scale;            /* 0.1 (delta euler) */
  double finger_scale;         /* 0.2 (finger width += finger_scale * a[6]) */
  uint32_t seed_lo, seed_hi;   /* Philox key of the reset draws */
} pnp_env_params;
/* sizeof(pnp_env_params) (binding layout check) */
int32_t pnp_env_params_size(void);
/* Per-env episode state, device SoA (float or double like the sim state; ints as given). */
typedef struct pnp_env_state {
  void* goal;            /* [B*3] desired goal */
  int32_t* task;         /* [B] current_task_index */
  int32_t* elapsed;      /* [B] TimeLimit step counter */
  void* qpos_kin;        /* [B*nq] qpos of the last forward (what data.site_* were computed at) */
  void* obj_height0;     /* [B] initial_object_height */
  void* init_mocap;      /* [B*7] initial mocap pos (3) + grasp quat (4) */
  void* init_qvel;       /* [B*nv] */
  void* init_time;       /* [B] */
  uint32_t* episode;     /* [B] resets so far: Philox counter of the reset draws */
  uint32_t* env_index;   /* [B] global env index: Philox counter (shard-invariant) */
  uint8_t* tier;         /* [B] optional (NULL: off): fp32 routing hint, the tier (0 compact, 1 full,
                          * 2 wide) the env's next gym step starts in; written by init / reset (0)
                          * and by the full / wide passes of pnp_env_step.  Routing changes where
                          * an env's step runs, never its results (the tiers' arithmetic is
                          * identical); PNP_GYM_ROUTE=0 disables it. */
} pnp_env_state;
/* Outputs (any pointer may be NULL to skip it). */
typedef struct pnp_env_out {
  void* obs;             /* [B*19] observation */
  void* achieved_goal;   /* [B*3] */
  void* desired_goal;    /* [B*3] (goal before this step's task update) */
  void* reward;          /* [B] */
  void* is_success;      /* [B] 1.0 / 0.0 */
  uint8_t* terminated;   /* [B] */
  uint8_t* truncated;    /* [B] */
} pnp_env_out;
int32_t pnp_env_init(pnp_model* model, const pnp_state* state, const pnp_env_params* params,
                     const pnp_env_state* env, int32_t B, void* stream);
int32_t pnp_env_init_f64(pnp_model* model, const pnp_state_f64* state, const pnp_env_params* params,
                         const pnp_env_state* env, int32_t B, void* stream);
/* mask[B] (uint8, NULL = every env): envs to reset; obs / achieved_goal / desired_goal of the
 * reset envs are written to out (other envs' outputs untouched). */
int32_t pnp_env_reset(pnp_model* model, const pnp_state* state, const pnp_env_params* params,
                      const pnp_env_state* env, const uint8_t* mask, const pnp_env_out* out, int32_t B,
                      void* stream);
int32_t pnp_env_reset_f64(pnp_model* model, const pnp_state_f64* state, const pnp_env_params* params,
                          const pnp_env_state* env, const uint8_t* mask, const pnp_env_out* out, int32_t B,
                          void* stream);
/* action[B*7] (same dtype as the state), clipped to [-1, 1] like the action space.
 * fp32: the full-capacity kernel runs the gym step; an env whose physics sub-step outgrows it is
 * finished (remaining sub-steps + observation / reward) by the wide tier's resume pass. */
int32_t pnp_env_step(pnp_model* model, const pnp_state* state, const pnp_env_params* params,
                     const pnp_env_state* env, const float* action, const pnp_env_out* out, int32_t B,
                     void* stream);
int32_t pnp_env_step_f64(pnp_model* model, const pnp_state_f64* state, const pnp_env_params* params,
                         const pnp_env_state* env, const double* action, const pnp_env_out* out, int32_t B,
                         void* stream);
/* Hand-over queue of the routed fp32 gym step (csrc/env_dev.h PNP_HQ_*), after the last such step
 * on the current device; synchronises the device.  out5: [0] envs the full-tier passes handed to
 * the wide tier through the queue, [1] producer workgroups done, [2] consumer claims, [3] consumers
 * that gave up waiting (PNP_GYM_QUEUE_TIMEOUT_US, default 20 s), [4] envs the fallback wide resume
 * pass finished after the join (the envs such consumers left).  Diagnostic: an env is never left
 * mid-step ([3] > 0 costs time, not results). */
int32_t pnp_env_queue_status(int32_t* out5);

/* ------------------------------------------------------------------ TQC learner (C5) */
/* One TQC gradient step (sb3-contrib tqc.py train(): entropy coefficient, critics against the
 * truncated target quantiles, actor, Polyak; the reference's learner, scripts/train.py:74-93) on
 * the matrix cores (csrc/tqc_fused.hip): per 16-row slab of the batch and per network a workgroup
 * runs the forward and backward chains; the weight gradients are whole-batch tile GEMMs with Adam
 * applied in place (no per-slab partial gradients).
 * Parameters in PyTorch's layouts -- actor: latent Linear 25->256->256->256 (weight [out][in],
 * bias [out]) W0 b0 W1 b1 W2 b2, heads mu / log_std 256->7 Wmu bmu Wls bls; critics (and their
 * target copies): n_critics stacked MLPs 32->256->256->256->25, weight [n_critics][in][out], bias
 * [n_critics][1][out], w0 b0 .. w3 b3 -- updated in place, with torch.optim.Adam's fused state
 * (exp_avg, exp_avg_sq, the per-parameter step scalars).  Supported: obs 25, action 7, hidden 256,
 * 2 critics x 25 quantiles, 2 dropped per net, batch a multiple of 16 (PNP_ERR_UNSUPPORTED
 * otherwise).  All pointers are device fp32. */
typedef struct pnp_tqc_desc {
  int32_t batch, obs_dim, act_dim, hidden, n_critics, n_quantiles, n_drop_per_net;
  float gamma, tau, target_entropy, beta1, beta2, adam_eps;
  float* actor[10]; float* actor_m[10]; float* actor_v[10]; float* actor_step[10];
  float* critic[8]; float* critic_m[8]; float* critic_v[8]; float* critic_step[8];
  float* target[8];
  float* log_ent_coef; float* ent_m; float* ent_v; float* ent_step;
  const float* lr;             /* learning rate (device scalar: the linear schedule writes it) */
  float* workspace;            /* pnp_tqc_workspace_floats() floats */
  int64_t workspace_floats;
  float* logs;                 /* [4] out: ent_coef (before the step), critic loss, actor loss, ent-coef loss */
  int64_t* draw_counter;       /* optional: pnp_tqc_sample_draw's counter, advanced by one per step (NULL: none) */
} pnp_tqc_desc;
/* One sampled, normalised batch: obs / next_obs [batch*25], act [batch*7], done / reward [batch],
 * and the two N(0, 1) draws of the step's squashed-Gaussian samples (actor on obs, on next_obs)
 * [batch*7] each -- drawn by the caller in sb3's order so the step is the PyTorch step's. */
typedef struct pnp_tqc_batch {
  const float* obs; const float* act; const float* next_obs; const float* done; const float* reward;
  const float* eps_pi; const float* eps_next;
} pnp_tqc_batch;
/* The replay buffer and the observation normaliser a batch is drawn from: sb3 DictReplayBuffer
 * (optimize_memory_usage=False) rows [rows][n_envs][dim] of obs / next_obs (the dict keys
 * flattened in sorted key order), actions, rewards, dones; `upper` the device scalar count of
 * filled rows; VecNormalize's per-key running mean / var (fp64, key_dim[k] each, same key order),
 * its clip_obs and epsilon. */
typedef struct pnp_tqc_replay {
  const float* obs; const float* next_obs; const float* actions; const float* rewards; const float* dones;
  const float* upper;
  int32_t rows, n_envs, obs_dim, act_dim, n_keys;
  int32_t key_dim[4];
  const double* mean[4]; const double* var[4];
  double clip_obs, norm_eps;
} pnp_tqc_replay;
/* DictReplayBuffer.sample + VecNormalize.normalize (pnp_amd/tqc.py TQC._sample_norm) for one
 * gradient step in one launch: u [2*batch] U[0, 1) draws (the caller's generator, sb3's order) ->
 * row = min(trunc(u[b] * upper), rows - 1), env = min(trunc(u[batch + b] * n_envs), n_envs - 1);
 * obs / next_obs normalised in fp64, clipped and rounded to fp32 ([batch*obs_dim]), act
 * [batch*act_dim], done / reward [batch] -- bit-identical to the PyTorch expressions.  Device
 * pointers, stream-ordered, capturable. */
int32_t pnp_tqc_sample(const pnp_tqc_replay* rb, const float* u, int32_t batch, float* obs, float* act, float* next_obs,
                       float* done, float* reward, void* stream);
/* pnp_tqc_sample with the step's random numbers drawn on the device (TQC.train's default): the two
 * U[0, 1) replay draws per row and the actor's two N(0, 1) draws (eps_pi, eps_next [batch*act_dim],
 * the inputs pnp_tqc_update takes) from Philox4x32-10 keyed by `seed`, counter = (counter[0], row,
 * lane).  counter: device int64[2], zero-initialised -- [0] the draw index, read here and advanced
 * by one on the device by the gradient step whose pnp_tqc_desc.draw_counter is this counter (so a
 * captured graph draws a fresh batch per replay), [1] reserved.  u_out
 * [2*batch] (optional) receives the uniform draws: pnp_tqc_sample with them gives the same batch
 * bit for bit.  Same distributions as the caller's torch generator, not its numbers.  act_dim
 * <= 63.  Stream-ordered, capturable. */
int32_t pnp_tqc_sample_draw(const pnp_tqc_replay* rb, uint64_t seed, int64_t* counter, int32_t batch, float* u_out,
                            float* eps_pi, float* eps_next, float* obs, float* act, float* next_obs, float* done,
                            float* reward, void* stream);
int64_t pnp_tqc_workspace_floats(const pnp_tqc_desc* d);
/* flat gradient sizes (actor, critics) of grads_out below */
int32_t pnp_tqc_param_counts(int32_t* actor_params, int32_t* critic_params);
/* grads_out (optional, tests): the step's reduced gradients, actor then critics, in the
 * parameters' own layouts and order.  Stream-ordered, no host sync; capturable in a HIP graph. */
int32_t pnp_tqc_update(const pnp_tqc_desc* d, const pnp_tqc_batch* b, float* grads_out, void* stream);
/* pnp_tqc_update split for a data-parallel learner (one process per GPU; the reference's learner is
 * single-process, scripts/train.py:67-93 -- this is its multi-GPU form): the caller averages the
 * gradients over ranks between the phases, as sb3 would with a DDP optimiser.  grads: device fp32
 * [actor_params + critic_params + 1] (pnp_tqc_param_counts; the last float is the entropy
 * coefficient's gradient).  The same batch (b) for all three calls of one step.
 *   phase 0: forward chains, critic backward, critic weight gradients -> grads[actor_params ..]
 *            (+ the entropy coefficient's), logs[0, 1, 3]; no parameter changes;
 *   phase 1: Adam on the critics and the entropy coefficient and the Polyak update from
 *            grads[actor_params ..] (all-reduced by the caller), then the actor's chains against
 *            the updated critics, actor weight gradients -> grads[0 .. actor_params), logs[2];
 *   phase 2: Adam on the actor from grads[0 .. actor_params).
 * With no collective in between the three phases equal pnp_tqc_update bit for bit.  Stream-
 * ordered, no host sync. */
int32_t pnp_tqc_update_phase(const pnp_tqc_desc* d, const pnp_tqc_batch* b, float* grads, int32_t phase, void* stream);

/* ------------------------------------------------------------------ skills */
/* RotateSkill.reset's trajectory (reference skills/rotate.py:39-46) for B skills: target =
 * R(start) * R(delta) and scipy Slerp([0, 1], [start, target]) at np.linspace(0, 1, steps).
 * Quaternions scalar-last (scipy's x, y, z, w: the skill hands MuJoCo's w, x, y, z to scipy
 * unchanged), device fp64 arrays: start[B*4], delta[B*4] -> target[B*4]
 * (may be NULL), track[B*steps*4]. */
int32_t pnp_slerp_track_f64(const double* start_xyzw, const double* delta_xyzw, int32_t steps,
                            double* target_xyzw, double* track_xyzw, int32_t B, void* stream);

/* FrankaEnv._get_obs (panda_env.py:279-301) + compute_reward / _is_success (:205-245, :303-306)
 * at the current state, without stepping: data.site_* of the last forward (env->qpos_kin), the
 * current qvel / finger qpos, current_task_index, initial_object_height.  ag / dg ([B*3], same
 * dtype, device; NULL = the observed achieved goal / the env's goal) are compute_reward's
 * achieved_goal / desired_goal arguments.  Writes obs / achieved_goal / desired_goal (observed)
 * and reward / is_success (for ag, dg) to out; terminated / truncated untouched.  The state and
 * the env state are read only (reference test/reward_test.py:69-74 calls _get_obs and
 * compute_reward between physics steps this way). */
int32_t pnp_env_evaluate(pnp_model* model, const pnp_state* state, const pnp_env_params* params,
                         const pnp_env_state* env, const float* ag, const float* dg, const pnp_env_out* out,
                         int32_t B, void* stream);
int32_t pnp_env_evaluate_f64(pnp_model* model, const pnp_state_f64* state, const pnp_env_params* params,
                             const pnp_env_state* env, const double* ag, const double* dg, const pnp_env_out* out,
                             int32_t B, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PNP_H */
