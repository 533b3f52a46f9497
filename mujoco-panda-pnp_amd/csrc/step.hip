// step.hip — batched mj_step for the shelf_pnp scene: one 64-lane wave per env, K sub-steps
// fused per launch with the whole per-env state resident in LDS.
//
// Reference: envs/panda_env.py:355-358 (_mujoco_step: 10 x mj_step(nstep=25)),
// skills/base.py:39-46 (_step_sim), scripts/execute_pnp.py:102-107; MuJoCo 2.3.3 mj_step with
// the options of assets/shelf_pnp.xml:4-6 (Euler, dt 0.002, noslip 3, pyramidal, warmstart).
// Stage for stage the same algorithms as oracle/physics.c (which documents them):
//   kinematics -> comPos -> CRBA(+armature) -> per-tree Cholesky of M -> collision ->
//   constraints (weld, joint limits, pyramidal contacts; impedance) -> comVel -> passive ->
//   RNE -> reference accel -> actuation -> qacc_smooth -> Newton (primal, exact line search) ->
//   noslip (pyramidal pairs) -> checkAcc -> Euler (implicit damping, quaternion integration).
//
// Lane mapping (no tree-level barriers anywhere):
//   bodies  : lane b composes its own root->b chain (body_path); cvel/cacc/crb/forces by masks
//   dofs    : lane d (cdof, cdof_dot, bias projection, gradients)
//   trees   : lane t factorises / solves its dense tree block of M (arm 9x9, cubes 6x6)
//   islands : lane i factorises its island block of the Newton Hessian (trees joined by rows)
//   pairs   : lane p runs broadphase + narrowphase of one candidate geom pair
//   rows    : lane r (impedance, reference acceleration, J.x); rows are stored sparsely over
//             the dofs of the <= 2 trees they touch (PH_ROWW slots)
#include <atomic>

#include "phys_model.h"
#include "pnp_internal.h"

// Three builds of this file, three capacity tiers of the same device code (fp32):
//   step_compact.hip  pnp_compact  20 contacts / 96 rows: 20 KB of LDS per env, 8 envs per CU
//   step.hip          pnp_full     64 contacts / 272 rows: 51 KB, 3 envs per CU; also the fp64
//                                  debugging instantiation, the debug kernels and the C ABI
//   step_wide.hip     pnp_wide     192 contacts / 784 rows: 1 env per CU
// A sub-step that would overflow a tier's capacity is abandoned before it changes the state and
// re-run from that sub-step by the next tier's resume pass (protocol: PNP_RESUME_* below), so an
// fp32 result is that of the widest tier, bit for bit, whichever tier finished each sub-step.  The
// widest tier, and the full tier when it runs alone (fp64, diagnostics), truncate like MuJoCo at a
// full buffer (warning bits CONTACTFULL / CNSTRFULL).  Closed fingers pressed together make 50-150
// contacts (box-box pad pairs, multiccd mesh pairs), so the gym workload needs the wide tier.
#ifndef PNP_COMPACT
#define PNP_COMPACT 0
#endif
#ifndef PNP_WIDE
#define PNP_WIDE 0
#endif
#ifndef PNP_GYM
#define PNP_GYM 0   // env_compact.hip: the compact tier's gym kernel (own namespace and image)
#endif
#ifndef PNP_WIDE64
#define PNP_WIDE64 0   // step_wide64.hip: the fp64 instantiation's wide tier (facade / batched BT)
#endif
#ifdef PNP_NS_NAME
#define PNP_NS PNP_NS_NAME
#elif PNP_COMPACT
#define PNP_NS pnp_compact
#elif PNP_WIDE
#define PNP_NS pnp_wide
#else
#define PNP_NS pnp_full
#endif
// PNP_HANDS: this build can hand an overflowing sub-step to the next tier (the full build only
// when its kernel is launched with hand = 1); PNP_LEAN: no debug-only fields outside the unions
#define PNP_HANDS (!PNP_WIDE)
// PNP_MW: the fp32 gym kernels of this build run several waves per env (helper waves for the convex
// pass): the wide build (4 waves, 1 env per CU) and the full build (2 waves, 3 envs per CU)
#define PNP_MW ((PNP_WIDE || (!PNP_COMPACT && !PNP_GYM)) && !PNP_WIDE64)
// MPR's portal support points in per-wave LDS slots (collide_dev.h SVertL): the full and wide
// builds (the compact builds run no MPR; the fp64 wide build keeps registers)
#define PNP_MPR_SLOTS (!PNP_COMPACT && !PNP_WIDE64)
// PNP_MPR_G: lanes per MPR run in the fp32 full / wide builds' convex pass (collide_dev.h CGrp): 16 =
// four runs per wave, and every fp32 full / wide kernel takes the multi-wave pass (one wave or
// more); 64 (A/B builds) = one run per wave, single-wave kernels on the serial pass
#ifndef PNP_MPR_G
#define PNP_MPR_G 16
#endif
// waves with MPR portal slots: the wide build's four; the full build's two (its opt-in two-wave
// gym kernel, PNP_GYM_FULL_MW), one with eight-lane groups (the slots of 8 groups per wave would
// cost the full tier its third env per CU)
#define PNP_MPR_SV_WAVES (PNP_WIDE ? 4 : (PNP_MPR_G < 16 ? 1 : 2))
// PNP_XLO: the fp32 builds keep each body's world position and quaternion as fp32 pairs (xpos /
// xquat + the remainders of the fp64 kinematic chain, Env::xlo / xqlo); MPR's geom frames and the
// box-box collider's centre offset are formed from them in fp64 (collide_dev.h c_geom_frame64,
// c_rel_pos): the relative geometry of two bodies then matches the fp64 chain's, not its per-body
// rounding to fp32 at world scale (~3e-8 m at 1 m, ~6e-8 rad).  The position remainder in every
// fp32 tier alike (box-box runs in all of them, and the hand-overs are exact only if every tier
// does the same arithmetic); the quaternion remainder (PNP_XQLO) where MPR runs (it does not fit
// the compact tier's 20 KB).
#define PNP_XLO (!PNP_WIDE64)
// Round 6 fp32 precision fixes (on; A/B builds: -DPNP_F32_SNAP=0 -DPNP_F32_NS_NEWTON=0): unresolved
// tangent rows snapped to zero (st_constraints), no-slip from Newton's iterate (st_noslip /
// st_finish_accel)
#ifndef PNP_F32_SNAP
#define PNP_F32_SNAP 1
#endif
#ifndef PNP_F32_NS_NEWTON
#define PNP_F32_NS_NEWTON 1
#endif
#define PNP_XQLO (!PNP_COMPACT && !PNP_WIDE64)
#define PNP_LEAN (PNP_COMPACT || PNP_WIDE || PNP_WIDE64)
// PNP_BIG_ISLANDS: the solver's whole-wave paths for islands with more rows than a wave (line
// search, gradient, MFMA Hessian).  Compiled out of the compact build, which hands such islands
// over instead (build_islands), so its common case pays nothing for them.
#define PNP_BIG_ISLANDS (!PNP_COMPACT)
#define PNP_BIG_ROWS 32   // = 8 lanes x the line search's 4 cached rows per lane
namespace PNP_NS {

// The physics image lives in the device's constant segment, one resident image per precision
// and device (ResidentLease, resident.cpp, copies a model's image in, stream-ordered, when a
// launch uses another model than the last one).  Every stage reads it through phys<T>(), a known global
// address: wave-uniform reads become scalar loads and per-lane reads global loads off a scalar
// base, in out-of-line stage functions as well.  Passed down by reference instead, the image
// reached the out-of-line stages as a generic pointer and every model read was a flat load that
// waits on the vector-memory and the LDS counters together.
__constant__ DevPhys<float> g_phys_f32;
__constant__ DevPhys<double> g_phys_f64;
template <typename T> __device__ __forceinline__ const DevPhys<T>& phys();
template <> __device__ __forceinline__ const DevPhys<float>& phys<float>() { return g_phys_f32; }
template <> __device__ __forceinline__ const DevPhys<double>& phys<double>() { return g_phys_f64; }

#define NT 64
#define EJ(r, k) s.efc_Jv[s.efc_off[r] + (k)]
#define EW(r, k) s.efc_Wv[s.efc_off[r] + (k)]

template <typename T> struct PM;
template <> struct PM<float> {
  static __device__ __forceinline__ float sqrt_(float x) { return __builtin_sqrtf(x); }
  static __device__ __forceinline__ float eps() { return 1.1920929e-07f; }
};
template <> struct PM<double> {
  static __device__ __forceinline__ double sqrt_(double x) { return __builtin_sqrt(x); }
  static __device__ __forceinline__ double eps() { return 2.220446049250313e-16; }
};

template <typename T>
struct Con {
  T pos[3], frame[9], dist, includemargin, friction[5], solref[2], solimp[5];
  int dim, g1, g2;
};

// env_lds_note: every kernel declares its Env as a static __shared__ variable and hands stage
// functions a reference to it.  The stages then address LDS off that pointer (ds_* with a VGPR
// base).  With a dynamic `extern __shared__` buffer instead, out-of-line stages reached the
// buffer through the per-kernel dynamic-LDS offset table: an s_load + lgkmcnt(0) drain that
// the compiler re-issued after every wave fence (once per no-slip pair update, for example).
// Per-env LDS working set, budgeted by lifetime (the compact build must fit 8 envs per CU:
// sizeof(Env<float>) <= 20 KB).  Stage order: kinematics -> comPos / CRB -> factor M ->
// collision -> constraint rows -> velocity / RNE -> actuation -> Newton -> noslip -> Euler.
//   * pos.*  : kinematics through RNE.  Frames, subtree COM, cdof and cinert persist through the
//              velocity stage; the kinematics -> CRB scratch (inertial frames, joint axes, crb)
//              is dead once M is built and makes room for the contact list (collision ->
//              constraint rows); geom frames die with the collision stage, the contact list with
//              the constraint rows, and the velocity stage's RNE vectors reuse both.
//   * sol.*  : Newton and noslip (dense island Jacobian blocks + either the packed island
//              Hessians and factors, or the noslip W = M^-1 J^T and pair lists).  The two
//              members of the outer union never live at the same time: the solver starts once the
//              rows and qacc_smooth exist.
// (The full build keeps the generalised forces of the velocity / actuation stages and the row
// positions outside the unions: its debug kernel dumps them after the whole forward.)
#ifndef PH_HCAP
#define PH_HCAP (PH_MAXV * (PH_MAXV + 1) / 2)   // packed island Hessian entries (sum over islands of n (n + 1) / 2)
#endif
#ifndef PH_MAXLIVE
#define PH_MAXLIVE PH_MAXPAIR   // broadphase survivors (the full build: every candidate pair)
#endif
static_assert(PH_HCAP >= PH_MAXMBLK, "the Euler stage's generic damped-block scratch lives in the Hessian store");
template <typename T>
struct Env {
  // ---- small model tables read in every inner loop (copied from the global model image once
  // per launch; global loads there would be latency-bound)
  int c_tree_dofadr[PH_MAXT], c_tree_dofnum[PH_MAXT], c_tree_moff[PH_MAXT], c_dof_tree[PH_MAXV];
  // ---- state
  T qpos[PH_MAXQ], qvel[PH_MAXV], ctrl[PH_MAXU], mocap_pos[6], mocap_quat[8], qacc_ws[PH_MAXV];
  T time;
  uint32_t warn;
  int ncon, nefc, ne, nisland, solver_iter, noslip_iter;
  int nlive, ncon_raw;     // collision: broadphase survivors, contacts before the capacity cap
  int nconvex;             // collision: live convex (MPR) pairs
  double wpose[2][7];      // fp32 builds: the first weld's two body poses in fp64 (pos, quat)
  union {
    struct {
      // kinematics -> velocity stage (and the gym epilogue's site frames / Jacobians)
      T xpos[PH_MAXB][3], xquat[PH_MAXB][4], xmat[PH_MAXB][9];
      T subcom[PH_MAXB][3], cdof[PH_MAXV][6], cinert[PH_MAXB][10];
      union {
        struct {
          T gpos[PH_MAXG][3], gmat[PH_MAXG][9];   // kinematics -> collision
#if PNP_XQLO
          // the remainder of the fp64 kinematic chain's body quaternion past xquat (fp32 builds
          // that run MPR; with xlo below, collide_dev.h c_geom_frame64)
          float xqlo[PH_MAXB][4];
#endif
          union {
            struct {                              // kinematics -> CRB
              T xipos[PH_MAXB][3], xanchor[PH_MAXJ][3], xaxis[PH_MAXJ][3];
              T crb[PH_MAXB][10], scr6a[PH_MAXV][6];
            };
            Con<T> con[PH_MAXCON];                // collision -> constraint rows
          };
        };
        struct {                                  // velocity stage -> actuation
          T cvel[PH_MAXB][6], cdofdot[PH_MAXV][6];
          T scr6[PH_MAXB > PH_MAXV ? PH_MAXB : PH_MAXV][6];   // per-body / per-dof 6-vector scratch
          T scr6b[PH_MAXB][6];
#if PNP_LEAN
          T qfrc_bias[PH_MAXV], qfrc_passive[PH_MAXV], qfrc_act[PH_MAXV];
#endif
        };
      };
    };
    struct {
      // solver stages: the constraint Jacobian once more, as dense island blocks (rows of island I
      // in island row order x its dofs in island order, row-major at isl_joff[I]; zeros where a
      // row does not touch a dof).  The dof-side sums (gradient, Hessian, J^T f) then stream
      // contiguous rows with no per-row slot lookup.  Built by build_islands when it fits (jt_ok).
      T jt[PH_JTCAP];
      union {
        struct {               // Newton: packed island Hessian blocks + per-row scratch
          // island I's block, lower triangle in island dof order: entry (a, b), a >= b, at
          // isl_eoff[I] + a (a + 1) / 2 + b (HI below)
          T Hp[PH_HCAP];
          T ntmp[PH_MAXEFC];
          T rr_f[PH_MAXEFC], rr_d[PH_MAXEFC];   // island row order: D jar, D (active rows; else 0)
          T NL[7][9][9];       // island Hessian factors of the group-parallel path (GCH_*), kept while isl_hvalid
        };
        struct {               // no-slip: W = M^-1 J^T and the per-group pair lists
          // packed like efc_Jv (+ 8: unmasked 8-slot reads past the last row, zeroed), or dense
          // island blocks laid out like jt (st_noslip's dense long-list path)
          T efc_Wv[PH_MAXJSLOT + 8 > PH_JTCAP ? PH_MAXJSLOT + 8 : PH_JTCAP];
          short ns_list[4][PH_MAXEFC / 2];
          int ns_len[4];
          T rr_g[PH_MAXEFC];   // island row order: forces
        };
      };
    };
  };
  T M[PH_MAXMBLK];    // per-tree dense blocks
  T L[PH_MAXMBLK];    // Cholesky factors of the blocks
  // ---- vectors
#if !PNP_LEAN
  T qfrc_bias[PH_MAXV], qfrc_passive[PH_MAXV], qfrc_act[PH_MAXV];
#endif
  T qfrc_smooth[PH_MAXV];
  T qacc_smooth[PH_MAXV], qacc[PH_MAXV], x[PH_MAXV], grad[PH_MAXV], p[PH_MAXV], v1[PH_MAXV], v2[PH_MAXV];
  // ---- constraints (sparse rows over <= 2 trees; t1 = -1 for single-tree rows)
  signed char efc_t0[PH_MAXEFC], efc_t1[PH_MAXEFC], efc_type[PH_MAXEFC];
  unsigned char efc_id[PH_MAXEFC], efc_act[PH_MAXEFC];
  int efc_off[PH_MAXEFC + 1];   // packed rows: slots [efc_off[r], efc_off[r+1])
  union {
    T efc_Jv[PH_MAXJSLOT + 8];   // + 8: room for unmasked 8-slot reads past the last row
    struct {                   // collision: single-pass contact staging (rows are rebuilt after it)
      T cst_val[NT][7];        // dist, pos[3], normal[3]
      unsigned short cst_key[NT];   // producing lane * 16 + its contact number
      int cst_n;
      short live[PH_MAXLIVE];  // broadphase survivors
    };
  };
#if !PNP_LEAN
  T efc_pos[PH_MAXEFC];        // debug record only
#endif
  T efc_D[PH_MAXEFC], efc_aref[PH_MAXEFC], efc_bb[PH_MAXEFC];
  T efc_force[PH_MAXEFC], efc_jar[PH_MAXEFC], efc_Jp[PH_MAXEFC];
  int con_rbase[PH_MAXCON], con_sbase[PH_MAXCON], con_t[PH_MAXCON][2];
  unsigned char con_dim[PH_MAXCON];
  T con_b[PH_MAXCON];          // contact: the reference acceleration's damping b (st_noslip's pair rows)
  int tree_island[PH_MAXT], isl_n[PH_MAXT];
  union {
    unsigned char isl_dof[PH_MAXT][PH_MAXV];   // build_islands -> the solver stages (Newton, noslip)
#if PNP_XLO
    // fp32 builds, kinematics -> collision: the remainder of the fp64 kinematic chain's body
    // position past xpos (collide_dev.h c_geom_frame64 / c_rel_pos).  Dead before build_islands
    // writes isl_dof; shares its bytes (the compact Env has no 288 B to spare for 8 envs per CU)
    float xlo[PH_MAXB][3];
#endif
  };
  int isl_eoff[PH_MAXT + 1], isl_roff[PH_MAXT + 1];
  int isl_joff[PH_MAXT + 1], tree_ipos[PH_MAXT], jt_ok;   // dense island Jacobian blocks (jt)
  unsigned char dof_ipos[PH_MAXV];                         // a dof's position in its island
  short isl_row[PH_MAXEFC];
  T isl_alpha[PH_MAXT];        // per-island line-search step (also the warm-start choice)
  T isl_cost[PH_MAXT], isl_val[PH_MAXT];   // per-island reductions (cost, |grad|^2 ...)
  int isl_flag[PH_MAXT];       // per-island: done (Newton), active set changed
  int isl_hvalid[PH_MAXT];     // per-island: H block is current for the island's active set
#if !PNP_COMPACT || PNP_GYM
  T qpos_pre[PH_MAXQ];         // gym env: qpos of the last forward (pre-integration)
#endif
  int ovf;                     // a capacity overflowed in this sub-step (hand-over builds)
  int hand;                    // full build: overflows hand over (1) or truncate with a warning (0)
#if PNP_MW
  int mw;                      // waves of the env's workgroup (the wide gym kernel: helper waves, mw_helper)
  int mw_cmd;                  // helper command (MW_*), posted by wave 0 before a workgroup barrier
  int mw_next;                 // the convex pass's next pair (LDS counter)
  unsigned char mw_hit[NT];    // the convex pass: staging slot holds a contact
  unsigned char mw_fan[NT];    // the convex pass: round-local pairs whose multiccd trials run
#endif
#if PNP_MPR_SLOTS
  double mpr_sv[PNP_MPR_SV_WAVES][64 / PNP_MPR_G][4][6];   // per wave and lane group: MPR's portal support points (collide_dev.h SVertL)
#endif
};
static_assert(sizeof(((Env<float>*)0)->efc_Jv) >= 7 * 4 * NT + 2 * NT + 4 + 2 * PH_MAXLIVE,
              "collision staging + broadphase survivors must fit the efc_Jv union");
// island I's packed Hessian entry (a, b), a >= b (island dof positions)
#define HI(I, a, b) s.Hp[s.isl_eoff[I] + (a) * ((a) + 1) / 2 + (b)]

// capacity overflow.  Wide build (and the full build launched with hand = 0): MuJoCo's behaviour
// (a warning bit, the list truncated).  Compact build (and full with hand = 1): flag the env; the
// stages return at the next check and the kernel hands the sub-step to the next tier
// (mj_step_dev, step_kernel).
#if PNP_COMPACT
#define CAP_FULL(bit) (s.ovf |= (bit) == 8u ? PNP_OVF_CONTACTS : PNP_OVF_ROWS)
#elif PNP_WIDE
#define CAP_FULL(bit) (s.warn |= (bit))
#else
#define CAP_FULL(bit) \
  (s.hand ? (void)(s.ovf |= (bit) == 8u ? PNP_OVF_CONTACTS : PNP_OVF_ROWS) : (void)(s.warn |= (bit)))
#endif
// resume protocol between a tier's kernel and the next tier's resume pass: the env's warn
// word carries the flag (bit 31), the capacity that overflowed (bits 28..30, diagnostic) and the
// sub-step to resume from (bits 16..27); the warning bits are 0..4
#define PNP_RESUME_FLAG 0x80000000u
#define PNP_RESUME_SHIFT 16
#define PNP_RESUME_MAXSUB 0xFFF
#define PNP_RESUME_WHY_SHIFT 28
#define PNP_OVF_CONTACTS 1   // collision: > PH_MAXCON contacts or > PH_MAXLIVE broadphase survivors
#define PNP_OVF_ROWS 2       // > PH_MAXEFC rows or > PH_MAXJSLOT Jacobian slots
#define PNP_OVF_JT 4         // dense island blocks: Jacobian > PH_JTCAP or Hessian > PH_HCAP

// stage timer (diagnostic instantiation only: TIMED = true); cycles accumulate in prof[stage]
// Sub-stage timers (sub_start / sub_lap) run inside a parent stage without resetting its lap;
// count() accumulates per-sub-step sizes (contacts, rows, iterations ...) into the count slots.
struct StageClock {
  unsigned long long* prof;
  unsigned long long t, ts, ta;
  __device__ void start() { if (prof) t = __builtin_amdgcn_s_memtime(); }
  __device__ void lap(int k) {
    if (!prof) return;
    __syncthreads();
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) prof[k] += n - t;
    t = n;
  }
  __device__ void sub_start() {
    if (!prof) return;
    __syncthreads();
    ts = __builtin_amdgcn_s_memtime();
  }
  __device__ void sub_lap(int k) {
    if (!prof) return;
    __syncthreads();
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) prof[k] += n - ts;
    ts = n;
  }
  __device__ void count(int k, int v) {
    if (prof && threadIdx.x == 0) prof[k] += (unsigned long long)v;
  }
  // ad-hoc timers (SC_AUX0 ..): a third clock, independent of the stage and sub-stage laps
  __device__ void aux_start() {
    if (!prof) return;
    __syncthreads();
    ta = __builtin_amdgcn_s_memtime();
  }
  __device__ void aux_lap(int k) {
    if (!prof) return;
    __syncthreads();
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) prof[k] += n - ta;
    ta = n;
  }
};
// the product kernels' clock: every call compiles to nothing (no prof pointer to test at run time)
struct NoClock {
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void lap(int) {}
  __device__ __forceinline__ void sub_start() {}
  __device__ __forceinline__ void sub_lap(int) {}
  __device__ __forceinline__ void count(int, int) {}
  __device__ __forceinline__ void aux_start() {}
  __device__ __forceinline__ void aux_lap(int) {}
};
// stage slots (include/pnp.h PNP_NSTAGE): sub-stages and per-step counts after the 16 stages
enum {
  SC_BROAD = 16, SC_NARROW, SC_CONVEX, SC_NS_W, SC_NS_LISTS, SC_K_PRE, SC_K_LEVELS, SC_K_FRAMES, SC_N_GRAD,
  SC_N_CONV, SC_N_HESS,
  SN_CON = 27, SN_EFC, SN_ITER, SN_CONVEX, SN_ISLAND, SN_NS_SWEEP, SN_LIVE,
  SC_AUX0 = 34,  // 8 ad-hoc sub-stage timers, SC_AUX0 .. SC_AUX0 + 7
  SN_NS_DENSE = 42, SN_NS_STREAM, SN_NS_ITER
};

// ============================================================================ small helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & (NT - 1); }   // (the wide gym kernel runs 4 waves)
// Lane hand-off through LDS inside the env's single wave.  The DS instructions of one wave execute
// in issue order, so a store by one lane is seen by a later load of any lane of the same wave
// without an s_waitcnt drain: a wavefront-scope fence (no instruction, a compiler ordering point)
// is all a hand-off needs.  __syncthreads() would also drain every outstanding LDS load at each
// of the step's ~60 hand-offs, serialising loads the scheduler could otherwise overlap.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- wave reductions on the DPP crossbar (no LDS round trips): butterfly inside each row of
// 16 lanes (quad_perm 1032, quad_perm 2301, row_half_mirror, row_mirror), then the four row
// sums are read with v_readlane.  gfx9 DPP controls: quad_perm 0x00-0xFF, row_mirror 0x140,
// row_half_mirror 0x141.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double rdlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// a sum's DPP operand: bound_ctrl set, so that fp32 `v += dpp_s<C>(v)` folds into one
// v_add_f32_dpp (0 is the identity of the add; every source lane of these in-row patterns is
// valid); fp64 adds take no DPP operand and keep the move
template <int CTRL>
__device__ __forceinline__ float dpp_s(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double dpp_s(double v) { return dpp_f<CTRL>(v); }
// lane K of each row of 16 to the whole row (gfx90a+ DPP row_newbcast)
template <int K>
__device__ __forceinline__ float rowbcast(float v) { return dpp_f<0x150 + K>(v); }
template <int K>
__device__ __forceinline__ double rowbcast(double v) { return dpp_f<0x150 + K>(v); }
// sum over each row of 16 lanes, result in every lane of the row
template <typename T>
__device__ __forceinline__ T rowsum16(T v) {
  v += dpp_s<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_s<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_s<0x141>(v);   // row_half_mirror
  v += dpp_s<0x140>(v);   // row_mirror
  return v;
}
// max over each row of 16 lanes, result in every lane of the row
template <typename T>
__device__ __forceinline__ T rowmax16(T v) {
  v = fmax(v, dpp_f<0xB1>(v));
  v = fmax(v, dpp_f<0x4E>(v));
  v = fmax(v, dpp_f<0x141>(v));
  v = fmax(v, dpp_f<0x140>(v));
  return v;
}
// sum over the wave, result (wave-uniform) in every lane
template <typename T>
__device__ __forceinline__ T wsum(T v) {
  v = rowsum16(v);
  return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
}

template <typename T>
__device__ __forceinline__ void t_normalize4(T q[4]) {
  T n = PM<T>::sqrt_(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < T(1e-15)) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else if (fabs(n - T(1)) > T(1e-15)) { T s = T(1) / n; q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s; }
}
template <typename T>
__device__ __forceinline__ T t_normalize3(T v[3]) {
  T n = PM<T>::sqrt_(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < T(1e-15)) { v[0] = 1; v[1] = v[2] = 0; return 0; }
  T s = T(1) / n;
  v[0] *= s; v[1] *= s; v[2] *= s;
  return n;
}
template <typename T>
__device__ __forceinline__ void t_cross(T r[3], const T a[3], const T b[3]) {
  T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T>
__device__ __forceinline__ T t_dot3(const T a[3], const T b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T>
__device__ __forceinline__ void t_mulmattvec3(T r[3], const T m[9], const T v[3]) {
  T t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  T t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  T t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T>
__device__ __forceinline__ void t_mulinertvec(T r[6], const T* i, const T v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
template <typename T>
__device__ __forceinline__ void t_crossmotion(T r[6], const T vel[6], const T v[6]) {
  r[0] = -vel[2] * v[1] + vel[1] * v[2];
  r[1] = vel[2] * v[0] - vel[0] * v[2];
  r[2] = -vel[1] * v[0] + vel[0] * v[1];
  r[3] = -vel[2] * v[4] + vel[1] * v[5];
  r[4] = vel[2] * v[3] - vel[0] * v[5];
  r[5] = -vel[1] * v[3] + vel[0] * v[4];
  r[3] += -vel[5] * v[1] + vel[4] * v[2];
  r[4] += vel[5] * v[0] - vel[3] * v[2];
  r[5] += -vel[4] * v[0] + vel[3] * v[1];
}
template <typename T>
__device__ __forceinline__ void t_crossforce(T r[6], const T vel[6], const T f[6]) {
  r[0] = -vel[2] * f[1] + vel[1] * f[2];
  r[1] = vel[2] * f[0] - vel[0] * f[2];
  r[2] = -vel[1] * f[0] + vel[0] * f[1];
  r[3] = -vel[2] * f[4] + vel[1] * f[5];
  r[4] = vel[2] * f[3] - vel[0] * f[5];
  r[5] = -vel[1] * f[3] + vel[0] * f[4];
  r[0] += -vel[5] * f[4] + vel[4] * f[5];
  r[1] += vel[5] * f[3] - vel[3] * f[5];
  r[2] += -vel[4] * f[3] + vel[3] * f[4];
}
template <typename T>
__device__ __forceinline__ void t_rotvecquat_mj(T r[3], const T v[3], const T q[4]) {
  // MuJoCo shortcut semantics (zero vector / identity quaternion)
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) { r[0] = r[1] = r[2] = 0; return; }
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) { r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; return; }
  d_rotvecquat(r, v, q);
}

// slot s of a sparse row -> dof index
// tree tables come from the env's LDS copy (Env::c_*); the DevPhys argument is kept for
// signature symmetry with the model-side helpers
template <typename T>
__device__ __forceinline__ int slot_dof_(const Env<T>& s, int t0, int t1, int k) {
  if (t0 < 0) return -1;
  const int n0 = s.c_tree_dofnum[t0];
  if (k < n0) return s.c_tree_dofadr[t0] + k;
  if (t1 < 0) return -1;
  k -= n0;
  return k < s.c_tree_dofnum[t1] ? s.c_tree_dofadr[t1] + k : -1;
}
template <typename T>
__device__ __forceinline__ int row_width_(const Env<T>& s, int t0, int t1) {
  return (t0 >= 0 ? s.c_tree_dofnum[t0] : 0) + (t1 >= 0 ? s.c_tree_dofnum[t1] : 0);
}
template <typename T>
__device__ __forceinline__ int mblk_(const Env<T>& s, int i, int j) {
  const int t = s.c_dof_tree[i];
  const int a = s.c_tree_dofadr[t], n = s.c_tree_dofnum[t];
  return s.c_tree_moff[t] + (i - a) * n + (j - a);
}
#define slot_dof(m, t0, t1, k) slot_dof_(s, t0, t1, k)
#define row_width(m, t0, t1) row_width_(s, t0, t1)

// v + J_r . x in slot order (the order of the slot_dof loop it replaces), with the row's tree
// table entries read once and every product's loads independent of the running sum
template <typename T>
__device__ __forceinline__ T row_dot(const Env<T>& s, int r, const T* x, T v) {
  const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], off = s.efc_off[r];
  const int n0 = s.c_tree_dofnum[t0], a0 = s.c_tree_dofadr[t0];
  const int t1c = t1 >= 0 ? t1 : 0;
  const int n1 = t1 >= 0 ? s.c_tree_dofnum[t1c] : 0, a1 = s.c_tree_dofadr[t1c];
  const T* J = s.efc_Jv + off;
#pragma unroll 3
  for (int q = 0; q < n0; q++) v += J[q] * x[a0 + q];
#pragma unroll 3
  for (int q = 0; q < n1; q++) v += J[n0 + q] * x[a1 + q];
  return v;
}
#define mblk(m, i, j) mblk_(s, i, j)

// ============================================================================ position stage
// sin / cos of an fp64 half joint angle: Taylor series to x^23 / x^24 for |x| <= 2 (truncation
// below 3e-16; every hinge of the arm stays within +-3.75 rad of qpos0), the math library's
// sincos otherwise (wave-uniform test: that branch only runs in states outside the joint range)
__device__ __forceinline__ void half_angle_sincos(double x, double* sn, double* cs) {
  if (__ballot(!(fabs(x) <= 2.0)) == 0) {
    const double x2 = x * x;
    // sin x = x sum_k (-1)^k x^2k / (2k+1)!, cos x = sum_k (-1)^k x^2k / (2k)!, Horner in x^2
    const double s0 = 1.0, s1 = -1.0 / 6, s2 = 1.0 / 120, s3 = -1.0 / 5040, s4 = 1.0 / 362880,
                 s5 = -1.0 / 39916800, s6 = 1.0 / 6227020800.0, s7 = -1.0 / 1307674368000.0,
                 s8 = 1.0 / 355687428096000.0, s9 = -1.0 / 121645100408832000.0,
                 s10 = 1.0 / 51090942171709440000.0, s11 = -1.0 / 25852016738884976640000.0;
    const double c0 = 1.0, c1 = -0.5, c2 = 1.0 / 24, c3 = -1.0 / 720, c4 = 1.0 / 40320, c5 = -1.0 / 3628800,
                 c6 = 1.0 / 479001600, c7 = -1.0 / 87178291200.0, c8 = 1.0 / 20922789888000.0,
                 c9 = -1.0 / 6402373705728000.0, c10 = 1.0 / 2432902008176640000.0,
                 c11 = -1.0 / 1124000727777607680000.0, c12 = 1.0 / 620448401733239439360000.0;
    double a = s11;
    a = fma(a, x2, s10); a = fma(a, x2, s9); a = fma(a, x2, s8); a = fma(a, x2, s7); a = fma(a, x2, s6);
    a = fma(a, x2, s5); a = fma(a, x2, s4); a = fma(a, x2, s3); a = fma(a, x2, s2); a = fma(a, x2, s1);
    a = fma(a, x2, s0);
    double c = c12;
    c = fma(c, x2, c11); c = fma(c, x2, c10); c = fma(c, x2, c9); c = fma(c, x2, c8); c = fma(c, x2, c7);
    c = fma(c, x2, c6); c = fma(c, x2, c5); c = fma(c, x2, c4); c = fma(c, x2, c3); c = fma(c, x2, c2);
    c = fma(c, x2, c1); c = fma(c, x2, c0);
    *sn = a * x;
    *cs = c;
  } else {
    sincos(x, sn, cs);
  }
}

template <typename T, class CLK>
__device__ void st_kinematics(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  clk.sub_start();
  // Bodies with at most one joint (this scene): pointer jumping over parent-relative transforms,
  // in fp64 (below).  Otherwise a level-synchronous tree pass in T (mj_kinematics order): a
  // body's frame is its parent's composed with its own offset and joints, the parent's read from
  // LDS one level earlier.  Either way the per-body work that does not need the parent -- the
  // model constants and a single hinge's rotation (sincos) -- is done by every lane at once up
  // front.
  const int b = lane_id();
  const bool mine = b > 0 && b < m.nbody;
  const int bb = mine ? b : 1;
  const int depth = mine ? m.body_pathlen[bb] : 0;
  const int pid = m.body_parentid[bb], ja = m.body_jntadr[bb], jn = m.body_jntnum[bb];
  const int jt = jn > 0 ? m.jnt_type[ja] : -1;
  const int mid = m.body_mocapid[bb];
  const bool one = jn == 1;
  const int qa1 = one ? m.jnt_qposadr[ja] : 0;
  if (!__ballot(mine && jn > 1)) {
    // Pointer jumping, every frame in fp64 and rounded once to T: every body's frame relative to
    // its parent (offset, then its one joint) is formed by all lanes at once from the model's fp64
    // chain constants (DevPhys::kd_*) and the state's exact values, then each lane composes with
    // its ancestor's accumulated transform and jumps to that ancestor's ancestor --
    // ceil(log2(depth)) = 4 register exchanges (ds_bpermute) for the arm's 11 levels instead of
    // one LDS round trip per level.  Rigid transforms compose associatively, so the frames are
    // MuJoCo's up to fp64 rounding (the order of the compositions differs).  Free-joint and mocap
    // bodies hang off the world.  Why fp64: an fp32 chain accumulates ~1e-7 m of rounding at the
    // hand, which the weld (solref 0.01) turns into a 2e-3 m/s^2 error of its reference
    // acceleration and the contact stiffness into a 1e-5-relative one; in fp64
    // every frame is within half an fp32 ulp of MuJoCo's, and the first weld's two body poses are
    // kept in fp64 (s.wpose) for its residual rows (st_constraints).
    double p[3] = {0, 0, 0}, q[4] = {1, 0, 0, 0}, jax[3] = {0, 0, 0}, jpos[3] = {0, 0, 0}, sl = 0;
    int anc = 0;
    if (mine) {
      if (mid >= 0) {
        for (int t = 0; t < 3; t++) p[t] = (double)s.mocap_pos[3 * mid + t];
        for (int t = 0; t < 4; t++) q[t] = (double)s.mocap_quat[4 * mid + t];
        t_normalize4(q);
        anc = pid;
      } else if (one && jt == 0) {
        for (int t = 0; t < 3; t++) p[t] = (double)s.qpos[qa1 + t];
        for (int t = 0; t < 4; t++) q[t] = (double)s.qpos[qa1 + 3 + t];
        t_normalize4(q);
      } else {
        double bq[4];
        for (int t = 0; t < 3; t++) p[t] = m.kd_body_pos[bb][t];
        for (int t = 0; t < 4; t++) q[t] = bq[t] = m.kd_body_quat[bb][t];
        if (one) {
          for (int t = 0; t < 3; t++) { jax[t] = m.kd_jnt_axis[bb][t]; jpos[t] = m.kd_jnt_pos[bb][t]; }
          sl = (double)s.qpos[qa1] - m.kd_qpos0[bb];
          if (jt == 2) {
            double ax[3];
            t_rotvecquat_mj(ax, jax, bq);
            for (int t = 0; t < 3; t++) p[t] += ax[t] * sl;
          } else if (jt == 3 && sl != 0.0) {
            // rotation qh about the axis through jpos: p += R(bq) (jpos - R(qh) jpos), q = bq qh
            double sn, cs, qh[4], v[3], u[3], wv[3];
            half_angle_sincos(sl * 0.5, &sn, &cs);
            qh[0] = cs; qh[1] = jax[0] * sn; qh[2] = jax[1] * sn; qh[3] = jax[2] * sn;
            t_rotvecquat_mj(v, jpos, qh);
            for (int t = 0; t < 3; t++) wv[t] = jpos[t] - v[t];
            t_rotvecquat_mj(u, wv, bq);
            for (int t = 0; t < 3; t++) p[t] += u[t];
            d_mulquat(q, bq, qh);
          }
        }
        anc = pid;
      }
    }
    clk.sub_lap(SC_K_PRE);
    while (__ballot(anc > 0)) {
      const int a = anc > 0 ? anc : 0;
      double pa[3], qa[4];
      for (int t = 0; t < 3; t++) pa[t] = __shfl(p[t], a);
      for (int t = 0; t < 4; t++) qa[t] = __shfl(q[t], a);
      const int a2 = __shfl(anc, a);
      if (anc > 0) {
        double r[3];
        t_rotvecquat_mj(r, p, qa);
        for (int t = 0; t < 3; t++) p[t] = pa[t] + r[t];
        d_mulquat(q, qa, q);
        anc = a2;
      }
    }
    if (mine) {
      t_normalize4(q);
      double R[9];
      d_quat2mat(R, q);
      for (int t = 0; t < 3; t++) s.xpos[b][t] = (T)p[t];
      for (int t = 0; t < 4; t++) s.xquat[b][t] = (T)q[t];
#if PNP_XLO
      for (int t = 0; t < 3; t++) s.xlo[b][t] = (float)(p[t] - (double)s.xpos[b][t]);
#endif
#if PNP_XQLO
      for (int t = 0; t < 4; t++) s.xqlo[b][t] = (float)(q[t] - (double)s.xquat[b][t]);
#endif
      for (int t = 0; t < 9; t++) s.xmat[b][t] = (T)R[t];
      if (one && jt == 0) {
        for (int t = 0; t < 3; t++) { s.xanchor[ja][t] = (T)p[t]; s.xaxis[ja][t] = m.jnt_axis[ja][t]; }
      } else if (one) {
        // the joint's axis and anchor in the body's final frame: a hinge leaves its axis and the
        // point jpos fixed; a slide moved the frame by axis * sl
        double ax[3], an[3];
        t_rotvecquat_mj(ax, jax, q);
        t_rotvecquat_mj(an, jpos, q);
        for (int t = 0; t < 3; t++) {
          s.xanchor[ja][t] = (T)(an[t] + p[t] - (jt == 2 ? ax[t] * sl : 0.0));
          s.xaxis[ja][t] = (T)ax[t];
        }
      }
      if (sizeof(T) == 4 && m.weld_eq >= 0)
        for (int k = 0; k < 2; k++)
          if (b == m.weld_body[k]) {
            for (int t = 0; t < 3; t++) s.wpose[k][t] = p[t];
            for (int t = 0; t < 4; t++) s.wpose[k][3 + t] = q[t];
          }
    }
  } else {
  // the body's own constants and joint, loaded up front: offset, a single joint's constants and
  // qpos, and a single hinge's local rotation (sincos)
  T bp[3], bq[4];
  for (int t = 0; t < 3; t++) bp[t] = m.body_pos[bb][t];
  for (int t = 0; t < 4; t++) bq[t] = m.body_quat[bb][t];
  if (mid >= 0) {
    for (int t = 0; t < 3; t++) bp[t] = s.mocap_pos[3 * mid + t];
    for (int t = 0; t < 4; t++) bq[t] = s.mocap_quat[4 * mid + t];
    t_normalize4(bq);
  }
  T jax[3] = {0, 0, 0}, jpos[3] = {0, 0, 0}, fq[7] = {0, 0, 0, 1, 0, 0, 0}, sl = 0;
  if (one) {
    for (int t = 0; t < 3; t++) { jax[t] = m.jnt_axis[ja][t]; jpos[t] = m.jnt_pos[ja][t]; }
    if (jt == 0)
      for (int t = 0; t < 7; t++) fq[t] = s.qpos[qa1 + t];
    else
      sl = s.qpos[qa1] - m.qpos0[qa1];
  }
  T qh[4] = {1, 0, 0, 0};
  if (one && jt == 3 && sl != T(0)) {
    T sn, cs;
    d_sincos(sl * T(0.5), &sn, &cs);
    qh[0] = cs; qh[1] = jax[0] * sn; qh[2] = jax[1] * sn; qh[3] = jax[2] * sn;
  }
  clk.sub_lap(SC_K_PRE);
  for (int d = 1; __ballot(mine && depth >= d); d++) {
    if (mine && depth == d) {
      T p[3], q[4];
      if (one && jt == 0) {
        p[0] = fq[0]; p[1] = fq[1]; p[2] = fq[2];
        q[0] = fq[3]; q[1] = fq[4]; q[2] = fq[5]; q[3] = fq[6];
        t_normalize4(q);
        for (int t = 0; t < 3; t++) { s.xanchor[ja][t] = p[t]; s.xaxis[ja][t] = jax[t]; }
      } else {
        if (pid > 0) {
          T pm[9], pp[3], dv[3];
          for (int t = 0; t < 9; t++) pm[t] = s.xmat[pid][t];
          for (int t = 0; t < 3; t++) pp[t] = s.xpos[pid][t];
          for (int t = 0; t < 4; t++) q[t] = s.xquat[pid][t];
          d_mulmatvec3(dv, pm, bp);
          for (int t = 0; t < 3; t++) p[t] = pp[t] + dv[t];
          d_mulquat(q, q, bq);
        } else {
          for (int t = 0; t < 3; t++) p[t] = bp[t];
          for (int t = 0; t < 4; t++) q[t] = bq[t];
        }
        if (one) {
          T ax[3], an[3];
          t_rotvecquat_mj(ax, jax, q);
          t_rotvecquat_mj(an, jpos, q);
          an[0] += p[0]; an[1] += p[1]; an[2] += p[2];
          if (jt == 2) {
            p[0] += ax[0] * sl; p[1] += ax[1] * sl; p[2] += ax[2] * sl;
          } else if (jt == 3) {
            T v[3];
            d_mulquat(q, q, qh);
            t_rotvecquat_mj(v, jpos, q);
            p[0] = an[0] - v[0]; p[1] = an[1] - v[1]; p[2] = an[2] - v[2];
          }
          for (int t = 0; t < 3; t++) { s.xanchor[ja][t] = an[t]; s.xaxis[ja][t] = ax[t]; }
        } else {
          for (int j = 0; j < jn; j++) {
            const int jid = ja + j, qa = m.jnt_qposadr[jid], ty = m.jnt_type[jid];
            T ax[3], an[3];
            t_rotvecquat_mj(ax, m.jnt_axis[jid], q);
            t_rotvecquat_mj(an, m.jnt_pos[jid], q);
            an[0] += p[0]; an[1] += p[1]; an[2] += p[2];
            if (ty == 2) {
              const T dd = s.qpos[qa] - m.qpos0[qa];
              p[0] += ax[0] * dd; p[1] += ax[1] * dd; p[2] += ax[2] * dd;
            } else if (ty == 3) {
              const T ang = s.qpos[qa] - m.qpos0[qa];
              T ql[4] = {1, 0, 0, 0}, v[3];
              if (ang != T(0)) {
                T sn, cs;
                d_sincos(ang * T(0.5), &sn, &cs);
                ql[0] = cs; ql[1] = m.jnt_axis[jid][0] * sn; ql[2] = m.jnt_axis[jid][1] * sn; ql[3] = m.jnt_axis[jid][2] * sn;
              }
              d_mulquat(q, q, ql);
              t_rotvecquat_mj(v, m.jnt_pos[jid], q);
              p[0] = an[0] - v[0]; p[1] = an[1] - v[1]; p[2] = an[2] - v[2];
            }
            for (int t = 0; t < 3; t++) { s.xanchor[jid][t] = an[t]; s.xaxis[jid][t] = ax[t]; }
          }
        }
      }
      t_normalize4(q);
      T R[9];
      d_quat2mat(R, q);
      for (int t = 0; t < 3; t++) s.xpos[b][t] = p[t];
#if PNP_XLO
      for (int t = 0; t < 3; t++) s.xlo[b][t] = 0.0f;   // (the T chain: no remainder)
#endif
#if PNP_XQLO
      for (int t = 0; t < 4; t++) s.xqlo[b][t] = 0.0f;
#endif
      for (int t = 0; t < 4; t++) s.xquat[b][t] = q[t];
      for (int t = 0; t < 9; t++) s.xmat[b][t] = R[t];
    }
    wsync();
  }
  if (sizeof(T) == 4 && m.weld_eq >= 0 && b < 2) {   // (multi-joint bodies: the T frames)
    const int wb = m.weld_body[b];
    for (int t = 0; t < 3; t++) s.wpose[b][t] = s.xpos[wb][t];
    for (int t = 0; t < 4; t++) s.wpose[b][3 + t] = s.xquat[wb][t];
  }
  }
  if (b == 0) {
    if (sizeof(T) == 4 && m.weld_eq >= 0)
      for (int k = 0; k < 2; k++)
        if (m.weld_body[k] == 0)
          for (int t = 0; t < 7; t++) s.wpose[k][t] = t == 3 ? 1.0 : 0.0;
    for (int t = 0; t < 3; t++) s.xpos[0][t] = 0;
#if PNP_XLO
    for (int t = 0; t < 3; t++) s.xlo[0][t] = 0.0f;
#endif
#if PNP_XQLO
    for (int t = 0; t < 4; t++) s.xqlo[0][t] = 0.0f;
#endif
    s.xquat[0][0] = 1; s.xquat[0][1] = s.xquat[0][2] = s.xquat[0][3] = 0;
    for (int t = 0; t < 9; t++) s.xmat[0][t] = (t % 4 == 0) ? T(1) : T(0);
  }
  wsync();
  clk.sub_lap(SC_K_LEVELS);
  // inertial frames (bodies) and geom frames (collidable geoms)
  for (int i = lane_id(); i < m.nbody + m.ngeom; i += NT) {
    if (i < m.nbody) {
      T v[3];
      d_mulmatvec3(v, s.xmat[i], m.body_ipos[i]);
      for (int t = 0; t < 3; t++) s.xipos[i][t] = s.xpos[i][t] + v[t];
    } else {
      const int g = i - m.nbody, b = m.geom_bodyid[g];
      T v[3], q[4], R[9];
      d_mulmatvec3(v, s.xmat[b], m.geom_pos[g]);
      d_mulquat(q, s.xquat[b], m.geom_quat[g]);
      d_quat2mat(R, q);
      for (int t = 0; t < 3; t++) s.gpos[g][t] = s.xpos[b][t] + v[t];
      for (int t = 0; t < 9; t++) s.gmat[g][t] = R[t];
    }
  }
  wsync();
  clk.sub_lap(SC_K_FRAMES);
}
template <typename T>
__device__ void st_kinematics(const DevPhys<T>& m, Env<T>& s) {
  NoClock clk;
  st_kinematics(m, s, clk);
}

template <typename T>
__device__ void st_compos_crb(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  // subtree COM of each root body (only roots are read: cinert and cdof are rooted there)
  // Lane i holds body i's mass, position and root; a uniform walk over the bodies reads them by
  // v_readlane (no memory round trip per body -- the walk used to wait on a scalar load of the
  // body's root and mass, then an LDS read, for every one of the nbody bodies) and the root
  // lanes accumulate in body order, as before.
  const bool lb = l < m.nbody;
  const T bm = lb ? m.body_mass[l] : T(0);
  const int br = lb ? m.body_rootid[l] : -1;
  const T bx0 = lb ? s.xipos[l][0] : T(0), bx1 = lb ? s.xipos[l][1] : T(0), bx2 = lb ? s.xipos[l][2] : T(0);
  T acc[3] = {0, 0, 0};
  for (int i = 1; i < m.nbody; i++) {
    const int ri = __builtin_amdgcn_readlane(br, i);
    const T mi = rdlane(bm, i), x0 = rdlane(bx0, i), x1 = rdlane(bx1, i), x2 = rdlane(bx2, i);
    if (ri == l) {
      acc[0] += x0 * mi;
      acc[1] += x1 * mi;
      acc[2] += x2 * mi;
    }
  }
  if (l > 0 && lb && br == l) {
    if (m.body_subtreemass[l] < T(1e-15)) for (int t = 0; t < 3; t++) s.subcom[l][t] = s.xipos[l][t];
    else for (int t = 0; t < 3; t++) s.subcom[l][t] = acc[t] / m.body_subtreemass[l];
  }
  wsync();
  // cinert (bodies), cdof (joints)
  if (l < m.nbody) {
    if (l == 0) {
      for (int t = 0; t < 10; t++) s.cinert[0][t] = 0;
    } else {
      const T* c = s.subcom[m.body_rootid[l]];
      T dif[3] = {s.xipos[l][0] - c[0], s.xipos[l][1] - c[1], s.xipos[l][2] - c[2]};
      const T* I = m.body_inertia[l];
      T R[9], iq[4];
      d_mulquat(iq, s.xquat[l], m.body_iquat[l]);
      d_quat2mat(R, iq);
      const T ms = m.body_mass[l];
      T tmp[9];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
          tmp[3 * i + j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] + R[3 * i + 2] * I[2] * R[3 * j + 2];
      T* o = s.cinert[l];
      o[0] = tmp[0] + ms * (dif[1] * dif[1] + dif[2] * dif[2]);
      o[1] = tmp[4] + ms * (dif[0] * dif[0] + dif[2] * dif[2]);
      o[2] = tmp[8] + ms * (dif[0] * dif[0] + dif[1] * dif[1]);
      o[3] = tmp[1] - ms * dif[0] * dif[1];
      o[4] = tmp[2] - ms * dif[0] * dif[2];
      o[5] = tmp[5] - ms * dif[1] * dif[2];
      o[6] = ms * dif[0]; o[7] = ms * dif[1]; o[8] = ms * dif[2];
      o[9] = ms;
    }
  }
  if (l < m.njnt) {
    const int da = m.jnt_dofadr[l], bi = m.jnt_bodyid[l];
    const T* c = s.subcom[m.body_rootid[bi]];
    T off[3] = {c[0] - s.xanchor[l][0], c[1] - s.xanchor[l][1], c[2] - s.xanchor[l][2]};
    switch (m.jnt_type[l]) {
      case 0:
        for (int i = 0; i < 3; i++) {
          for (int t = 0; t < 6; t++) s.cdof[da + i][t] = 0;
          s.cdof[da + i][3 + i] = 1;
        }
        for (int i = 0; i < 3; i++) {
          T ax[3] = {s.xmat[bi][i], s.xmat[bi][i + 3], s.xmat[bi][i + 6]};
          T* cd = s.cdof[da + 3 + i];
          cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
          t_cross(cd + 3, ax, off);
        }
        break;
      case 2: {
        T* cd = s.cdof[da];
        cd[0] = cd[1] = cd[2] = 0;
        cd[3] = s.xaxis[l][0]; cd[4] = s.xaxis[l][1]; cd[5] = s.xaxis[l][2];
        break;
      }
      case 3: {
        T* cd = s.cdof[da];
        T ax[3] = {s.xaxis[l][0], s.xaxis[l][1], s.xaxis[l][2]};
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        t_cross(cd + 3, ax, off);
        break;
      }
      default:
        break;
    }
  }
  wsync();
  // composite inertia: crb[b] = sum of cinert over the subtree of b
  if (l > 0 && l < m.nbody) {
    T acc[10];
    for (int t = 0; t < 10; t++) acc[t] = 0;
    uint32_t st = m.body_subtree[l];
    while (st) {
      const int c = __builtin_ctz(st);
      st &= st - 1;
      for (int t = 0; t < 10; t++) acc[t] += s.cinert[c][t];
    }
    for (int t = 0; t < 10; t++) s.crb[l][t] = acc[t];
  }
  wsync();
  // buf_i = crb[body(i)] * cdof_i
  if (l < m.nv) {
    T r[6];
    t_mulinertvec(r, s.crb[m.dof_bodyid[l]], s.cdof[l]);
    for (int t = 0; t < 6; t++) s.scr6a[l][t] = r[t];
  }
  for (int i = l; i < m.nmblock; i += NT) s.M[i] = 0;
  wsync();
  for (int e = l; e < m.nmentry; e += NT) {
    const int i = m.mentry_i[e], j = m.mentry_j[e];
    T v = 0;
    for (int t = 0; t < 6; t++) v += s.cdof[j][t] * s.scr6a[i][t];
    if (i == j) v += m.dof_armature[i];
    s.M[mblk(m, i, j)] = v;
    s.M[mblk(m, j, i)] = v;
  }
  wsync();
}

// dense Cholesky of an n x n block (row stride ld) into Lb (lower); one lane
template <typename T>
__device__ void chol_block(const T* A, T* Lb, int n, int ld) {
  for (int j = 0; j < n; j++) {
    T sjj = A[j * ld + j];
    for (int k = 0; k < j; k++) sjj -= Lb[j * ld + k] * Lb[j * ld + k];
    sjj = PM<T>::sqrt_(sjj > T(0) ? sjj : T(1e-30));
    Lb[j * ld + j] = sjj;
    const T inv = T(1) / sjj;
    for (int i = j + 1; i < n; i++) {
      T t = A[i * ld + j];
      for (int k = 0; k < j; k++) t -= Lb[i * ld + k] * Lb[j * ld + k];
      Lb[i * ld + j] = t * inv;
    }
  }
}

// x = (L L^T)^-1 b on one block; x, b are indexed through dof lists (idx) of a global vector
template <typename T>
__device__ void chol_solve_block(const T* Lb, int n, int ld, const int* idx, int adr, T* x, const T* b) {
  // the forward substitution's y lives in x itself (step i reads b[i] before writing y[i] there,
  // so x may alias b): no private array, whose frame (PH_MAXV floats) every caller of the solves
  // would carry although the scene's trees never take this path (<= 9 dofs: registers)
  for (int i = 0; i < n; i++) {
    T v = b[idx ? idx[i] : adr + i];
    for (int k = 0; k < i; k++) v -= Lb[i * ld + k] * x[idx ? idx[k] : adr + k];
    x[idx ? idx[i] : adr + i] = v / Lb[i * ld + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    T v = x[idx ? idx[i] : adr + i];
    for (int k = i + 1; k < n; k++) v -= Lb[k * ld + i] * x[idx ? idx[k] : adr + k];
    x[idx ? idx[i] : adr + i] = v / Lb[i * ld + i];
  }
}

// chol_block in registers for n <= N (same operation order, so the same factor): one lane,
// packed lower triangle, no LDS round trip per multiply-add.  Rows >= n are identity padding.
// A = M block (row stride n) + diag(h * damping) when damp != nullptr.
template <typename T, int N>
__device__ __forceinline__ void chol_reg(const T* A, int n, const T* damp, T h, T* L) {
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j <= i; j++)
      L[i * (i + 1) / 2 + j] = i < n ? A[i * n + j] + (i == j && damp ? h * damp[i] : T(0)) : T(i == j);
#pragma unroll
  for (int j = 0; j < N; j++) {
    T d = L[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; k++) d -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
    d = PM<T>::sqrt_(d > T(0) ? d : T(1e-30));
    L[j * (j + 1) / 2 + j] = d;
    const T inv = T(1) / d;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      T v = L[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; k++) v -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
      L[i * (i + 1) / 2 + j] = v * inv;
    }
  }
}
// x = (L L^T)^-1 b for a register factor (chol_solve_block's order); x, b at adr (may alias)
template <typename T, int N>
__device__ __forceinline__ void chol_solve_reg(const T* L, int n, T* x, const T* b) {
  T y[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    T v = i < n ? b[i] : T(0);
#pragma unroll
    for (int k = 0; k < i; k++) v -= L[i * (i + 1) / 2 + k] * y[k];
    y[i] = v / L[i * (i + 1) / 2 + i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    T v = y[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) v -= L[k * (k + 1) / 2 + i] * y[k];
    y[i] = v / L[i * (i + 1) / 2 + i];
  }
#pragma unroll
  for (int i = 0; i < N; i++)
    if (i < n) x[i] = y[i];
}

// ---- wave-parallel Cholesky of up to 7 blocks of n <= 9 at once.  Block g lives on the 9-lane
// group 9g .. 9g+8 (lane 63 idle); lane row r = l - 9g computes row r of the factor, and every
// finished column is broadcast (ds_bpermute) so that each lane of the group ends up holding the
// whole factor in registers (packed lower triangle P).  Column step j: every lane forms the pivot
// L[j][j] itself from the broadcast row j (the pivot lane's own arithmetic, so the same bits),
// its own L[r][j], then the column's broadcast, whose latency overlaps the next step's pivot row
// terms.  Same operation order as chol_reg (hence the same factor); the solves then run
// redundantly in every lane (chol_solve_reg on P) with no further cross-lane traffic.  Rows >= n
// are identity padding.
#define GCH_N 9
#define GCH_GROUPS 7
__device__ __forceinline__ int gch_group(int l) { return l / GCH_N; }
// in: Lrow = the lane's row of A (entries j <= r used), Ad[j] = A[j][j]; out: P (every lane)
template <typename T>
__device__ __forceinline__ void gch_factor(T Lrow[GCH_N], const T Ad[GCH_N], int r, int base, T P[45]) {
#pragma unroll
  for (int j = 0; j < GCH_N; j++) {
    T td = Ad[j];
#pragma unroll
    for (int k = 0; k < j; k++) td -= P[j * (j + 1) / 2 + k] * P[j * (j + 1) / 2 + k];
    const T d = PM<T>::sqrt_(td > T(0) ? td : T(1e-30));
    const T inv = T(1) / d;
    T t = Lrow[j];
#pragma unroll
    for (int k = 0; k < j; k++) t -= Lrow[k] * P[j * (j + 1) / 2 + k];
    Lrow[j] = r == j ? d : (r > j ? t * inv : Lrow[j]);
    P[j * (j + 1) / 2 + j] = d;
#pragma unroll
    for (int i = j + 1; i < GCH_N; i++) P[i * (i + 1) / 2 + j] = __shfl(Lrow[j], base + i);
  }
}

template <typename T>
__device__ __forceinline__ void st_factor_M(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int t = lane_id();
  if (m.ntree <= GCH_GROUPS && !__ballot(t < m.ntree && s.c_tree_dofnum[t] > GCH_N)) {
    // every tree block on its own 9-lane group
    const int g = gch_group(t), r = t - GCH_N * g;
    const bool on = g < m.ntree;
    const int n = on ? s.c_tree_dofnum[g] : 0, o = on ? s.c_tree_moff[g] : 0;
    T Lrow[GCH_N], Ad[GCH_N], P[45];
#pragma unroll
    for (int j = 0; j < GCH_N; j++) {
      Lrow[j] = r < n && j <= r ? s.M[o + r * n + j] : T(r == j);
      Ad[j] = j < n ? s.M[o + j * n + j] : T(1);
    }
    gch_factor(Lrow, Ad, r, GCH_N * g, P);
    if (r < n)
#pragma unroll
      for (int j = 0; j < GCH_N; j++)
        if (j <= r) s.L[o + r * n + j] = Lrow[j];
    wsync();
    return;
  }
  if (t < m.ntree) {
    const int n = s.c_tree_dofnum[t], o = s.c_tree_moff[t];
    if (n <= 9) {
      T L[45];
      chol_reg<T, 9>(s.M + o, n, (const T*)nullptr, T(0), L);
#pragma unroll
      for (int i = 0; i < 9; i++)
#pragma unroll
        for (int j = 0; j <= i; j++)
          if (i < n) s.L[o + i * n + j] = L[i * (i + 1) / 2 + j];
    } else {
      chol_block(s.M + o, s.L + o, n, n);
    }
  }
  wsync();
}

// x = M_t^-1 b on one tree block with the factor in s.L (registers for n <= 9)
template <typename T, bool REG = true>
__device__ __forceinline__ void tree_solve(const Env<T>& s, int o, int a, int n, T* x, const T* b) {
  if (REG && n <= 9) {
    T L[45];
#pragma unroll
    for (int i = 0; i < 9; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) L[i * (i + 1) / 2 + j] = i < n ? s.L[o + i * n + j] : T(i == j);
    chol_solve_reg<T, 9>(L, n, x + a, b + a);
  } else {
    chol_solve_block(s.L + o, n, n, (const int*)nullptr, a, x, b);
  }
}

// x = M^-1 b (tree blocks, lane per tree); x and b may alias
template <typename T, bool REG = true>
__device__ void solve_M(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, T* x, const T* b) {
  const DevPhys<T>& m = phys<T>();
  const int t = lane_id();
  if (t < m.ntree) tree_solve<T, REG>(s, s.c_tree_moff[t], s.c_tree_dofadr[t], s.c_tree_dofnum[t], x, b);
  wsync();
}

// r = M v (tree blocks, lane per dof)
template <typename T>
__device__ T mulM_row(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int i, const T* v) {
  const int t = s.c_dof_tree[i];
  const int a = s.c_tree_dofadr[t], n = s.c_tree_dofnum[t], o = s.c_tree_moff[t] + (i - a) * n;
  T r = 0;
  // the scene's block sizes fully unrolled (all loads issue before the sum), same order
  if (n == 9) {
#pragma unroll
    for (int k = 0; k < 9; k++) r += s.M[o + k] * v[a + k];
  } else if (n == 6) {
#pragma unroll
    for (int k = 0; k < 6; k++) r += s.M[o + k] * v[a + k];
  } else {
    for (int k = 0; k < n; k++) r += s.M[o + k] * v[a + k];
  }
  return r;
}

// inclusive wave scan of a per-lane count, on DPP: row_shr 1, 2, 4, 8 inside each row of 16
// (bound_ctrl zero fill = the lanes below the shift add nothing), then the row totals by
// v_readlane.  Integer sums, so the same values as the six ds_bpermute (__shfl_up) steps it
// replaces, which each waited for an LDS round trip.  Call with the whole wave active.
__device__ __forceinline__ int wscan_incl(int x) {
  x += __builtin_amdgcn_mov_dpp(x, 0x111, 0xF, 0xF, true);
  x += __builtin_amdgcn_mov_dpp(x, 0x112, 0xF, 0xF, true);
  x += __builtin_amdgcn_mov_dpp(x, 0x114, 0xF, 0xF, true);
  x += __builtin_amdgcn_mov_dpp(x, 0x118, 0xF, 0xF, true);
  const int r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31),
            r2 = __builtin_amdgcn_readlane(x, 47);
  const int row = lane_id() >> 4;
  return x + (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
}
// ============================================================================ collision
#include "collide_dev.h"

template <typename T, class CLK>
__device__ void st_collision(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  clk.sub_start();
  clk.aux_start();
  // broadphase, three passes, survivors compacted in pair order throughout.
  // (1) body pairs: bounding spheres over each body's collidable geoms (bit per body pair, kept
  //     wave-uniform in four 64-bit words); (2) geom pairs of live body pairs: bounding spheres;
  //     (3) the exact box tests (convex: oriented boxes overlap; plane: the box reaches the plane)
  //     over the pass-(2) survivors only -- a compact list, so the divergent box tests occupy
  //     one or two lane chunks instead of one in every chunk of the pair table.
  uint64_t bpm[PH_MAXBP / 64];
#pragma unroll
  for (int w = 0; w < PH_MAXBP / 64; w++) {
    const int bp = w * NT + l;
    bool alive = false;
    if (w * NT < m.nbpair && bp < m.nbpair) {
      const T reach = m.bp_reach[bp];
      alive = true;
      if (reach >= 0) {
        const int b1 = m.bp_b1[bp], b2 = m.bp_b2[bp];
        T v[3];
#pragma unroll
        for (int k = 0; k < 3; k++)
          v[k] = s.xpos[b1][k] + s.xmat[b1][3 * k] * m.body_bcen[b1][0] + s.xmat[b1][3 * k + 1] * m.body_bcen[b1][1] +
                 s.xmat[b1][3 * k + 2] * m.body_bcen[b1][2] - s.xpos[b2][k] - s.xmat[b2][3 * k] * m.body_bcen[b2][0] -
                 s.xmat[b2][3 * k + 1] * m.body_bcen[b2][1] - s.xmat[b2][3 * k + 2] * m.body_bcen[b2][2];
        alive = t_dot3(v, v) <= reach * reach;
      }
    }
    bpm[w] = __ballot(alive);
  }
  clk.aux_lap(SC_AUX0);       // aux0: broadphase pass 1 (body pairs)
  int nlive = 0;
  // Branch-free per chunk, and the next chunk's two table words are loaded (unconditionally, at
  // a clamped index) while this one is tested.  With the loads behind the body-pair branch a
  // chunk waited for pair_pack, then for pair_reach, then for the LDS positions: two serial trips
  // to the model image (L1/L2) per chunk, ~900 cycles per chunk over the ~16 chunks of the table;
  // a prefetch under an exec branch does not help either, the wait counter then drains it too.
  const int plast = max(m.npair - 1, 0);
  uint32_t pk_n = m.pair_pack[min(l, plast)];
  T reach_n = m.pair_reach[min(l, plast)];
  for (int base = 0; base < m.npair; base += NT) {
    const int pi = base + l;
    const uint32_t pk = pk_n;
    const T reach = reach_n;
    const int pn = min(pi + NT, plast);
    pk_n = m.pair_pack[pn];
    reach_n = m.pair_reach[pn];
    const int bp = pk >> 24;
    const uint64_t w01 = (bp & 64) ? bpm[1] : bpm[0], w23 = (bp & 64) ? bpm[3] : bpm[2];
    const uint64_t word = (bp & 128) ? w23 : w01;
    const int g1 = pk & 255, g2 = (pk >> 8) & 255;
    T v[3] = {s.gpos[g1][0] - s.gpos[g2][0], s.gpos[g1][1] - s.gpos[g2][1], s.gpos[g1][2] - s.gpos[g2][2]};
    const bool keep = (pi < m.npair) & (bool)((word >> (bp & 63)) & 1) &
                      ((reach < T(0)) | (t_dot3(v, v) <= reach * reach));
    const uint64_t bal = __ballot(keep);
    const int at = nlive + __popcll(bal & ((1ull << l) - 1));
    if (keep && at < PH_MAXLIVE) s.live[at] = (short)pi;
    nlive += __popcll(bal);
  }
  wsync();
  if (PNP_COMPACT && nlive > PH_MAXLIVE) {   // (the full build's list holds every candidate pair)
    if (l == 0) { s.ovf |= PNP_OVF_CONTACTS; s.nlive = 0; s.ncon_raw = 0; s.nconvex = 0; s.ncon = 0; }
    wsync();
    return;
  }
  clk.aux_lap(SC_AUX0 + 1);   // aux1: broadphase pass 2 (geom-pair spheres)
  clk.count(SC_AUX0 + 2, nlive);   // aux2: sphere survivors (count)
  // cheap exact pre-test over the sphere survivors (~180 per sub-step here: the shelf boards'
  // bounding spheres are large): each geom's bounding sphere against the other's bounding box,
  // both ways, and the plane test; compacted in place (a chunk reads its entries into registers
  // before any lane writes, and writes land at or below the read positions), so that the
  // separating-axis tests below run over one chunk of survivors instead of every chunk
  // Branch-free like pass 2: every lane runs both tests and selects by kind, and the next
  // chunk's list entries and table words are fetched while this chunk is tested (they lie at or
  // above (chunk + 1) * 64, beyond every write of this chunk).
  int nsph = nlive;
  nlive = 0;
  int pi_n = nsph > 0 ? s.live[min(l, nsph - 1)] : 0;
  uint32_t pk_p = m.pair_pack[pi_n];
  T mg_p = m.pair_margin[pi_n];
  for (int base = 0; base < nsph; base += NT) {
    const int k = base + l;
    const int pi = pi_n;
    const uint32_t pk = pk_p;
    const T pmg = mg_p;
    pi_n = s.live[min(k + NT, nsph - 1)];
    pk_p = m.pair_pack[pi_n];
    mg_p = m.pair_margin[pi_n];
    const int g1 = pk & 255, g2 = (pk >> 8) & 255, kind = (pk >> 16) & 255;
    const T mg = pmg + T(1e-6);
    const bool sph = !c_sphere_obb_disjoint(m, s, g1, g2, mg) & !c_sphere_obb_disjoint(m, s, g2, g1, mg);
    const bool pln = !c_plane_obb_clear(m, s, g1, g2, pmg);
    const bool keep = (k < nsph) & ((kind == PH_PAIR_CONVEX || kind == PH_PAIR_BOX) ? sph
                                     : kind == PH_PAIR_PLANE                       ? pln
                                                                                   : true);
    const uint64_t bal = __ballot(keep);
    wsync();
    if (keep) s.live[nlive + __popcll(bal & ((1ull << l) - 1))] = (short)pi;
    nlive += __popcll(bal);
  }
  wsync();
  // exact oriented-box tests over the pre-test survivors, compacted in place likewise
  nsph = nlive;
  nlive = 0;
  for (int base = 0; base < nsph; base += NT) {
    const int k = base + l;
    bool keep = false;
    int pi = 0;
    if (k < nsph) {
      pi = s.live[k];
      const uint32_t pk = m.pair_pack[pi];
      const int g1 = pk & 255, g2 = (pk >> 8) & 255, kind = (pk >> 16) & 255;
      keep = true;
      // convex and box-box pairs share one oriented-box separating-axis test (box-box: the
      // boxes themselves, inflated by margin + 1 um, so that a pair the box-box collider's own
      // SAT would keep is never culled)
      if (kind == PH_PAIR_CONVEX || kind == PH_PAIR_BOX)
        keep = !c_convex_obb_disjoint(m, s, g1, g2, m.pair_margin[pi] + (kind == PH_PAIR_BOX ? T(1e-6) : T(0)));
    }
    const uint64_t bal = __ballot(keep);
    wsync();
    if (keep) s.live[nlive + __popcll(bal & ((1ull << l) - 1))] = (short)pi;
    nlive += __popcll(bal);
  }
  wsync();
  clk.sub_lap(SC_BROAD);
  // narrowphase, one pass: every lane collides its pair once, its contacts go to a staging area
  // through an LDS slot counter, then each lands at (contacts so far) + (exclusive scan of the
  // per-lane counts) + (its number within the pair) -- the order a sequential loop over the live
  // pairs produces.  If a chunk stages more than 64 contacts it falls back to a second collide
  // pass writing at the scanned offsets.  Contact order: primitive pairs in pair order, then the
  // convex (MPR) pairs in pair order (st_collision_convex).
  // (a lane's geoms and kind come from the one packed table word, PH_PAIR_CONVEX being
  // c_is_convex_pair's test; the staged contacts get their geoms by shuffles: one model-image
  // trip per chunk for the pair instead of three)
  int ncon = 0, nconvex = 0;
  for (int base = 0; base < nlive; base += NT) {
    const int k = base + l;
    const int pair = k < nlive ? s.live[k] : 0;
    const uint32_t pk = m.pair_pack[pair];
    const int pg1 = pk & 255, pg2 = (pk >> 8) & 255;
    const bool cvx = k < nlive && ((pk >> 16) & 255) == PH_PAIR_CONVEX;
    nconvex += __popcll(__ballot(cvx));
    if (l == 0) s.cst_n = 0;
    wsync();
    StageSink<T> ss{&s.cst_n, s.cst_val, s.cst_key, l};
    if (k < nlive && !cvx) collide_geoms(m, s, pg1, pg2, ss);
    wsync();
    const int staged = s.cst_n;
    const int incl = wscan_incl(ss.n);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    const int off = ncon + incl - ss.n;
    if (staged <= NT && !__ballot(ss.n >= 16)) {
      const int key = l < staged ? s.cst_key[l] : 0;
      const int src = key >> 4;
      const int at = __shfl(off, src) + (key & 15);
      const int sg1 = __shfl(pg1, src), sg2 = __shfl(pg2, src);
      if (l < staged && at < PH_MAXCON) {
        Con<T>& c = s.con[at];
        c.dist = s.cst_val[l][0];
        for (int t = 0; t < 3; t++) c.pos[t] = s.cst_val[l][1 + t];
        for (int t = 0; t < 9; t++) c.frame[t] = t < 3 ? s.cst_val[l][4 + t] : T(0);
        c_params(m, c, sg1, sg2);
      }
    } else if (ss.n) {
      LdsSink<T> ls{s.con + off, PH_MAXCON - off};
      if (ls.cap > 0) {
        collide_geoms(m, s, pg1, pg2, ls);
        for (int c = 0; c < ss.n && c < ls.cap; c++) c_params(m, s.con[off + c], pg1, pg2);
      }
    }
    wsync();
    ncon += total;
  }
  if (l == 0) {
    s.nlive = nlive;
    s.ncon_raw = ncon;
    s.nconvex = nconvex;
    s.ncon = min(ncon, PH_MAXCON);
    if (ncon > PH_MAXCON) CAP_FULL(8u);
  }
  wsync();
  clk.sub_lap(SC_NARROW);
}

#if PNP_MW
// ---- helper wave of the wide gym kernel (env_step_wide_kernel runs MW_WAVES waves per env; wave
// 0 runs the step, the others wait in mw_helper).  Wave 0 posts a command in s.mw_cmd and meets the
// helpers at a workgroup barrier (A), every wave does its part, and a second barrier (B) ends the
// part; MW_EXIT (posted once, at the end of the kernel) releases them.  Wave 0 issues no other
// workgroup barrier while helpers wait (its stage clock is the NoClock).
enum { MW_EXIT = 0, MW_MPR = 1, MW_FAN = 2 };
// Four waves, one per SIMD: the wide tier's Env (192 contacts) holds one env per CU, so the helpers
// cost no residency, and multiccd makes up to five MPR runs per convex pair to spread.  (Round 2 /
// early round 3, at two envs per CU: two waves, four were slower -- profiles/r03/ab_mpr_helper_waves.log.)
// Each wave runs 64 / PNP_MPR_G items at a time, one per lane group (round 6).
constexpr int MW_WAVES = PNP_WIDE ? 4 : 2;   // full build: 2 x 3 envs per CU
constexpr int MW_GROUPS = 64 / PNP_MPR_G;
// A round's convex pairs (up to RN, listed by wave 0 in cst_key in live-list order), each with
// `per` staging slots (cst_val, mw_hit): slot per o holds pair o's first MPR contact, slots
// per o + 1 + t its multiccd trial t (positions relative to geom 1's centre).  Items are taken one
// at a time by whichever wave is free (an LDS counter): MW_MPR items are the pairs, MW_FAN items
// (pair, trial) of the pairs with a first contact.  The same functions as st_collision_convex's
// serial c_convex (c_convex_shapes / c_mpr_contact / c_fan_rotate): the same bits.
__device__ void convex_part(Env<float>& s, int cmd) {
  const DevPhys<float>& m = phys<float>();
  const int l = lane_id();
  const int kind = cmd & 255;
  // n and the taken slot are wave-uniform (SGPRs), so the loop's exit is a scalar branch: with
  // a per-lane exit the compiler's structured loop could run on with lane 0 masked off, where
  // readfirstlane no longer reads the lane that took the slot.  At most n trips in any case.
  const int n = __builtin_amdgcn_readfirstlane(cmd >> 8);
  const int per = m.multiccd ? C_MULTI : 1;
  // a wave takes MW_GROUPS consecutive items (o wave-uniform), lane group q item o + q: a pair's four
  // multiccd trials (items 4 i .. 4 i + 3) run side by side in one wave
  const int q = l / PNP_MPR_G;
  for (int it = 0; it < n; it++) {
    int o = 0;
    if (l == 0) o = atomicAdd(&s.mw_next, MW_GROUPS);
    o = __builtin_amdgcn_readfirstlane(__shfl(o, 0));
    if (o >= n) return;
    const int oi = o + q;   // this group's item
    if (oi < n) {           // (group-uniform)
      const int po = kind == MW_FAN ? s.mw_fan[oi >> 2] : oi;   // round-local pair
      const int slot = per * po + (kind == MW_FAN ? 1 + (oi & 3) : 0);
      const int p = s.cst_key[po];
      const int g1 = m.pair_g1[p], g2 = m.pair_g2[p];
      const float margin = fmaxf(m.geom_margin[g1], m.geom_margin[g2]);
      const bool hit = c_convex_run<float, PNP_MPR_G>(s, g1, g2, margin, kind == MW_FAN ? (oi & 3) : -1,
                                                      s.cst_val + per * po, slot - per * po);
      if ((l & (PNP_MPR_G - 1)) == 0) s.mw_hit[slot] = hit;
    }
  }
}
__device__ void mw_helper(Env<float>& s) {
  for (;;) {
    __syncthreads();   // A: a command is posted
    const int cmd = s.mw_cmd;
    if ((cmd & 255) == MW_EXIT) return;
    convex_part(s, cmd);
    __syncthreads();   // B: the part is done
  }
}
// wave 0: run one part on every wave of the workgroup
__device__ __forceinline__ void mw_run(Env<float>& s, int cmd) {
  if (lane_id() == 0) {
    s.mw_next = 0;
    s.mw_cmd = cmd;
  }
  __syncthreads();   // A
  convex_part(s, cmd);
  __syncthreads();   // B
}
// wave 0: per round of up to RN convex pairs, list them, run their first MPR and then their
// multiccd trials on every wave, decide each pair's fan in trial order (lane per pair: the same
// distinct-position tests as c_convex) and append the contacts in live-list order (the order
// st_collision_convex's one-pair-at-a-time loop produces; same bits)
__device__ __attribute__((noinline)) void st_collision_convex_mw(Env<float>& s) {
  const DevPhys<float>& m = phys<float>();
  const int l = lane_id();
  int ncon = s.ncon_raw;
  const int nconv = s.nconvex, nlive = s.nlive;
  const int per = m.multiccd ? C_MULTI : 1, RN = NT / per;
  int base = 0, ord = 0;   // live-list chunk and convex ordinal the listing has reached
  for (int r = 0; RN * r < nconv; r++) {
    const int n = min(RN, nconv - RN * r);
    int got = 0;
    while (got < n && base < nlive) {   // list this round's pairs (chunks may straddle rounds)
      const int k = base + l;
      const int pair = k < nlive ? s.live[k] : 0;
      const bool cvx = k < nlive && c_is_convex_pair(m, m.pair_g1[pair], m.pair_g2[pair]);
      const uint64_t bal = __ballot(cvx);
      const int o = ord + __popcll(bal & ((1ull << l) - 1ull));
      if (cvx && o >= RN * r && o < RN * r + n) s.cst_key[o - RN * r] = (unsigned short)pair;
      const int c = __popcll(bal);
      if (ord + c > RN * r + n) break;   // this chunk continues into the next round: keep it
      ord += c;
      got = ord - RN * r;
      base += NT;
    }
    if (l < NT) s.mw_hit[l] = 0;
    wsync();
    mw_run(s, MW_MPR | (n << 8));
    const bool first = l < n && s.mw_hit[per * l];
    if (per > 1) {   // the trials of the pairs with a first contact (no fan for a sphere: c_convex)
      bool fan = first;
      if (first) {
        const int p = s.cst_key[l];
        fan = m.geom_type[m.pair_g1[p]] != 2 && m.geom_type[m.pair_g2[p]] != 2;
      }
      const uint64_t hb = __ballot(fan);
      if (fan) s.mw_fan[__popcll(hb & ((1ull << l) - 1ull))] = (unsigned char)l;
      wsync();
      const int nh = __popcll(hb);
      if (nh) mw_run(s, MW_FAN | ((4 * nh) << 8));
    }
    // lane o: pair o's fan in trial order (accepted slots as a bit mask)
    unsigned acc = 0;
    int cnt = 0, pg1 = 0;
    if (first) {
      const int p = s.cst_key[l];
      pg1 = m.pair_g1[p];
      const float tol = c_fan_tol(m, pg1, m.pair_g2[p]);
      acc = 1;
      for (int t = 1; t < per; t++) {
        if (!s.mw_hit[per * l + t]) continue;
        bool distinct = true;
        for (int i = 0; i < t; i++)
          if (((acc >> i) & 1) && c_fan_close(s.cst_val[per * l + t] + 1, s.cst_val[per * l + i] + 1, tol)) distinct = false;
        if (distinct) acc |= 1u << t;
      }
      cnt = __popc(acc);
    }
    const int excl = wscan_incl(cnt) - cnt;
    const int tot = __builtin_amdgcn_readlane(excl + cnt, 63);
    // staging slot l holds trial j of pair o: its place if accepted
    const int o = l / per, j = l - o * per;
    const unsigned ao = (unsigned)__shfl((int)acc, o);
    const int eo = __shfl(excl, o);
    const int at = ncon + eo + __popc(ao & ((1u << j) - 1u));
    if (o < n && ((ao >> j) & 1) && at < PH_MAXCON) {
      const int p = s.cst_key[o], g1 = m.pair_g1[p], g2 = m.pair_g2[p];
      CT org[3];
      c_geom_frame64(m, s, g1, org, (CT*)nullptr);
      const float pos[3] = {(float)(CT(s.cst_val[l][1]) + org[0]), (float)(CT(s.cst_val[l][2]) + org[1]),
                            (float)(CT(s.cst_val[l][3]) + org[2])};
      const float nrm[3] = {s.cst_val[l][4], s.cst_val[l][5], s.cst_val[l][6]};
      LdsSink<float> ls{s.con + at, 1};
      ls.emit(s.cst_val[l][0], pos, nrm);
      c_params(m, s.con[at], g1, g2);
    }
    (void)pg1;
    ncon += tot;
    wsync();
  }
  if (l == 0) {
    if (ncon > PH_MAXCON) CAP_FULL(8u);
    s.ncon = min(ncon, PH_MAXCON);
  }
  wsync();
}
#endif

// Convex (MPR) pairs of the live list, appended after the primitive contacts.  A stage of its
// own, out of line, and only called when the broadphase kept a convex pair: MPR's portal state
// then never shares a register allocation with the rest of the step, and steps without convex
// candidates pay neither its frame nor its callee-saved registers (inlined, or called
// unconditionally, it slowed the whole step by 17-20 %).
template <typename T>
__device__ __attribute__((noinline)) void st_collision_convex(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  const int nlive = s.nlive;
  int ncon = s.ncon_raw;
  for (int base = 0; base < nlive; base += NT) {
    const int k = base + l;
    const int pair = k < nlive ? s.live[k] : 0;
    uint64_t todo = __ballot(k < nlive && c_is_convex_pair(m, m.pair_g1[pair], m.pair_g2[pair]));
    while (todo) {                                  // the wave takes the pairs one at a time, in order
      const int src = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      const int p = __builtin_amdgcn_readlane(pair, src);
      const int g1 = m.pair_g1[p], g2 = m.pair_g2[p];
#if PNP_COMPACT
      // The compact build runs no MPR: a convex pair it cannot prove separated (c_convex_screen)
      // hands the sub-step to the full tier, like a capacity overflow, and the full tier's fp64
      // MPR decides (the same contacts: a proven pair has none).  Round 3 ran the first MPR here
      // (handing over only pairs in contact: every overlap of bounding boxes handed over had cost
      // C3 30 %, the arm swinging near a board); in fp64 (round 4) its frame grew the kernel's
      // scratch 292 -> 704 B per lane and cost C3 2 % although C3's envs rarely run it.
      if (!c_convex_screen(m, s, g1, g2, fmax(m.geom_margin[g1], m.geom_margin[g2]))) {
        if (l == 0) CAP_FULL(8u);
        wsync();
        return;
      }
      const int n = 0;
#else
      // the pair's contacts (up to C_MULTI with multiccd) staged in cst_val, then lanes 0.. append
      const int n = c_convex(m, s, g1, g2, fmax(m.geom_margin[g1], m.geom_margin[g2]), s.cst_val);
#endif
      if (l < n && ncon + l < PH_MAXCON) {
        const T pos[3] = {s.cst_val[l][1], s.cst_val[l][2], s.cst_val[l][3]};
        const T nrm[3] = {s.cst_val[l][4], s.cst_val[l][5], s.cst_val[l][6]};
        LdsSink<T> ls{s.con + ncon + l, 1};
        ls.emit(s.cst_val[l][0], pos, nrm);
        c_params(m, s.con[ncon + l], g1, g2);
      }
      ncon += n;
      wsync();
    }
  }
  if (l == 0) {
    if (ncon > PH_MAXCON) CAP_FULL(8u);
    s.ncon = min(ncon, PH_MAXCON);
  }
  wsync();
}

// ============================================================================ constraints
template <typename T>
__device__ T impedance_(const T* si, T x) {
  const T dmin = fmin(fmax(si[0], T(0.0001)), T(0.9999)), dmax = fmin(fmax(si[1], T(0.0001)), T(0.9999));
  const T width = si[2], mid = si[3], power = si[4];
  x = fabs(x);
  if (width <= T(1e-15) || x >= width) return dmax;
  T y = x / width;
  if (power == T(2)) {
    if (y <= mid) y = y * y / mid;
    else y = T(1) - (T(1) - y) * (T(1) - y) / (T(1) - mid);
  } else if (power != T(1)) {
    if (y <= mid) y = pow(y, power) / pow(mid, power - 1);
    else y = T(1) - pow(T(1) - y, power) / pow(T(1) - mid, power - 1);
  }
  return dmin + y * (dmax - dmin);
}

// impedance of row r from its pos / margin / diagApprox (mj_makeImpedance): stores D and the
// position part of the reference acceleration; the velocity part (-b J qvel) is added by
// finish_rows once the row's Jacobian is complete (b parked in efc_Jp meanwhile)
template <typename T>
__device__ __forceinline__ void row_imp(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, int r, T pos, T margin, T diag, const T* solref,
                        const T* solimp) {
  const DevPhys<T>& m = phys<T>();
  const T dmax = fmin(fmax(solimp[1], T(0.0001)), T(0.9999));
  T k, b;
  if (solref[0] > 0) {
    const T tc = fmax(solref[0], 2 * m.timestep), dr = solref[1];
    k = T(1) / (dmax * dmax * tc * tc * dr * dr);
    b = T(2) / (dmax * tc);
  } else {
    k = -solref[0] / (dmax * dmax);
    b = -solref[1] / dmax;
  }
  const T imp = impedance_(solimp, pos - margin);
#if !PNP_LEAN
  s.efc_pos[r] = pos;
#endif
  s.efc_D[r] = T(1) / fmax(T(1e-15), (1 - imp) * diag / imp);
  s.efc_aref[r] = -k * imp * (pos - margin);
  s.efc_Jp[r] = b;
}

// translational Jacobian column of world point pt on body b at dof d (0 if d does not move b)
template <typename T>
__device__ __forceinline__ void jac_col_rm(const Env<T>& s, int root, uint64_t dofmask, int d, const T pt[3], T jp[3], T jr[3]) {
  if (d < 0 || !(dofmask >> d & 1)) {
    jp[0] = jp[1] = jp[2] = 0;
    jr[0] = jr[1] = jr[2] = 0;
    return;
  }
  const T* c = s.subcom[root];
  const T off[3] = {pt[0] - c[0], pt[1] - c[1], pt[2] - c[2]};
  const T* cd = s.cdof[d];
  T t[3];
  t_cross(t, cd, off);
  for (int k = 0; k < 3; k++) { jp[k] = cd[3 + k] + t[k]; jr[k] = cd[k]; }
}
template <typename T>
__device__ __forceinline__ void jac_col(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int b, int d, const T pt[3], T jp[3], T jr[3]) {
  const DevPhys<T>& m = phys<T>();
  jac_col_rm(s, m.body_rootid[b], m.body_dofmask[b], d, pt, jp, jr);
}

template <typename T>
__device__ __forceinline__ void body_trees(const DevPhys<T>& /*image: phys<T>()*/, int b1, int b2, int& t0, int& t1) {
  const DevPhys<T>& m = phys<T>();
  t0 = m.body_dofmask[b1] ? m.body_tree[b1] : -1;
  t1 = m.body_dofmask[b2] ? m.body_tree[b2] : -1;
  if (t0 < 0) { t0 = t1; t1 = -1; }
  if (t0 == t1) t1 = -1;
}

// exclusive wave scan of a per-lane count; returns the offset, total in *tot
__device__ __forceinline__ int wscan(int n, int* tot) {
  const int incl = wscan_incl(n);
  *tot = __builtin_amdgcn_readlane(incl, 63);
  return incl - n;
}

// Constraint rows in MuJoCo order: weld (6 per equality), joint limits, contacts (2(dim-1) per
// contact, pyramidal edges J_n +- mu_k J_tk).  Every row is stored packed over the dofs of the
// <= 2 trees it touches (weld: arm 9; limits: 1 slot; cube-shelf: 6).
template <typename T>
__device__ void st_constraints(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  int nrow = 0, nslot = 0;
  // ---- weld
  for (int e = 0; e < m.neq; e++) {
    if (m.eq_type[e] != 1) continue;
    const T* data = m.eq_data[e];
    const int id0 = m.eq_obj1id[e], id1 = m.eq_obj2id[e];
    int t0, t1;
    body_trees(m, id0, id1, t0, t1);
    const int w = row_width(m, t0, t1);
    if (nrow + 6 > PH_MAXEFC || nslot + 6 * w > PH_MAXJSLOT) { if (l == 0) CAP_FULL(16u); break; }
    T pos0[3], pos1[3], q[4], q1[4], q2[4];
    d_mulmatvec3(pos0, s.xmat[id0], data + 3);
    d_mulmatvec3(pos1, s.xmat[id1], data);
    for (int k = 0; k < 3; k++) { pos0[k] += s.xpos[id0][k]; pos1[k] += s.xpos[id1][k]; }
    const T ts = data[10];
    d_mulquat(q, s.xquat[id0], data + 6);
    q1[0] = s.xquat[id1][0]; q1[1] = -s.xquat[id1][1]; q1[2] = -s.xquat[id1][2]; q1[3] = -s.xquat[id1][3];
    d_mulquat(q2, q1, q);
    T err[6];
    for (int k = 0; k < 3; k++) { err[k] = pos0[k] - pos1[k]; err[3 + k] = q2[1 + k] * ts; }
    if (sizeof(T) == 4 && e == m.weld_eq) {
      // the same residual from the fp64 poses (weld_pose_f64) and fp64 weld data, rounded once
      const double* kd = m.kd_eq_data;
      double p0[3], p1[3], qq[4], qc[4], qe[4];
      t_rotvecquat_mj(p0, kd + 3, &s.wpose[0][3]);
      t_rotvecquat_mj(p1, kd, &s.wpose[1][3]);
      d_mulquat(qq, &s.wpose[0][3], kd + 6);
      qc[0] = s.wpose[1][3]; qc[1] = -s.wpose[1][4]; qc[2] = -s.wpose[1][5]; qc[3] = -s.wpose[1][6];
      d_mulquat(qe, qc, qq);
      for (int k = 0; k < 3; k++) {
        err[k] = (T)((p0[k] + s.wpose[0][k]) - (p1[k] + s.wpose[1][k]));
        err[3 + k] = (T)(qe[1 + k] * kd[10]);
      }
    }
    T my_err = err[0];
#pragma unroll
    for (int k = 1; k < 6; k++) my_err = l == k ? err[k] : my_err;   // (no private-array indexing)
    if (l < 6) {
      const int r = nrow + l;
      s.efc_off[r] = nslot + l * w;
      s.efc_t0[r] = t0; s.efc_t1[r] = t1;
      s.efc_type[r] = 0; s.efc_id[r] = e;
      row_imp(m, s, r, my_err, T(0),
              l < 3 ? m.body_invweight0[id0][0] + m.body_invweight0[id1][0]
                    : m.body_invweight0[id0][1] + m.body_invweight0[id1][1],
              m.eq_solref[e], m.eq_solimp[e]);
    }
    if (l < w) {
      const int d = slot_dof(m, t0, t1, l);
      T jp0[3], jr0[3], jp1[3], jr1[3];
      jac_col(m, s, id0, d, pos0, jp0, jr0);
      jac_col(m, s, id1, d, pos1, jp1, jr1);
      T ax[3] = {jr0[0] - jr1[0], jr0[1] - jr1[1], jr0[2] - jr1[2]};
      T tq[4], t3[4];
      tq[0] = -q1[1] * ax[0] - q1[2] * ax[1] - q1[3] * ax[2];
      tq[1] = q1[0] * ax[0] + q1[2] * ax[2] - q1[3] * ax[1];
      tq[2] = q1[0] * ax[1] + q1[3] * ax[0] - q1[1] * ax[2];
      tq[3] = q1[0] * ax[2] + q1[1] * ax[1] - q1[2] * ax[0];
      d_mulquat(t3, tq, q);
      for (int k = 0; k < 3; k++) {
        s.efc_Jv[nslot + k * w + l] = jp0[k] - jp1[k];
        s.efc_Jv[nslot + (3 + k) * w + l] = T(0.5) * t3[1 + k] * ts;
      }
    }
    nrow += 6;
    nslot += 6 * w;
  }
  const int ne = nrow;
  // ---- joint limits: count per joint, scan rows and slots, emit (rows span the joint's tree)
  int nl = 0, wl = 0;
  if (l < m.njnt && m.jnt_limited[l] && (m.jnt_type[l] == 2 || m.jnt_type[l] == 3)) {
    const T v = s.qpos[m.jnt_qposadr[l]], mg = m.jnt_margin[l];
    nl = (v - m.jnt_range[l][0] < mg) + (m.jnt_range[l][1] - v < mg);
    wl = m.tree_dofnum[m.dof_tree[m.jnt_dofadr[l]]];
  }
  int nlim, nlslot;
  const int lo = wscan(nl, &nlim);
  const int so = wscan(nl * wl, &nlslot);
  if (nl) {
    int r = nrow + lo, sl = nslot + so;
    const T v = s.qpos[m.jnt_qposadr[l]], mg = m.jnt_margin[l];
    const int d = m.jnt_dofadr[l], t = m.dof_tree[d];
    for (int side = -1; side <= 1; side += 2) {
      const T dist = side * (m.jnt_range[l][(side + 1) / 2] - v);
      if (dist < mg && r < PH_MAXEFC && sl + wl <= PH_MAXJSLOT) {
        s.efc_off[r] = sl;
        s.efc_t0[r] = t; s.efc_t1[r] = -1;
        s.efc_type[r] = 3; s.efc_id[r] = l;
        for (int k = 0; k < wl; k++) s.efc_Jv[sl + k] = 0;
        s.efc_Jv[sl + d - m.tree_dofadr[t]] = T(-side);
        row_imp(m, s, r, dist, mg, m.dof_invweight0[d], m.jnt_solref[l], m.jnt_solimp[l]);
        r++;
        sl += wl;
      }
    }
  }
  if (nrow + nlim > PH_MAXEFC || nslot + nlslot > PH_MAXJSLOT) {
    if (l == 0) CAP_FULL(16u);
    nlim = 0;   // (rows past capacity were not written; drop the limits block entirely)
    nlslot = 0;
  }
  nrow += nlim;
  nslot += nlslot;
  wsync();
  // ---- contacts: per-contact row/slot bases by scan (64 contacts per pass), then lanes over
  // (contact, slot)
  const int nc = s.ncon;
  int kept_rows = nrow;
  bool spill = false;
  // The first 64 contacts' body data stays in the contact's lane (root bodies, dof masks,
  // invweight sums): the Jacobian-slot and row loops below fetch it by lane shuffles instead of
  // two more serial trips to the model image (geom -> body -> mask / root) per chunk.
  const bool fastc = nc <= NT;
  int kr1 = 0, kr2 = 0;
  uint64_t km1 = 0, km2 = 0;
  T ktran = 0, krot = 0;
  for (int cb = 0, rb = nrow, sb = nslot; cb < nc; cb += NT) {
    const int c = cb + l;
    int my_rows = 0, my_slots = 0, t0c = -1, t1c = -1;
    if (c < nc) {
      const Con<T>& con = s.con[c];
      const int b1 = m.geom_bodyid[con.g1], b2 = m.geom_bodyid[con.g2];
      body_trees(m, b1, b2, t0c, t1c);
      if (cb == 0) {
        kr1 = m.body_rootid[b1];
        kr2 = m.body_rootid[b2];
        km1 = m.body_dofmask[b1];
        km2 = m.body_dofmask[b2];
        ktran = m.body_invweight0[b1][0] + m.body_invweight0[b2][0];
        krot = m.body_invweight0[b1][1] + m.body_invweight0[b2][1];
      }
      my_rows = 2 * (con.dim - 1);
      my_slots = my_rows * row_width(m, t0c, t1c);
    }
    int trows, tslots;
    const int rbase = rb + wscan(my_rows, &trows);
    const int sbase = sb + wscan(my_slots, &tslots);
    const bool fits = c < nc && rbase + my_rows <= PH_MAXEFC && sbase + my_slots <= PH_MAXJSLOT;
    if (c < nc) {
      s.con_rbase[c] = fits ? rbase : -1;
      s.con_sbase[c] = sbase;
      s.con_t[c][0] = t0c;
      s.con_t[c][1] = t1c;
      s.con_dim[c] = (unsigned char)s.con[c].dim;
    }
    spill |= __ballot(c < nc && !fits) != 0;
    // last contact that fits bounds the row count (contacts are added in order; the row bases are
    // a prefix sum, so the highest fitting lane holds the largest end -- read it directly instead
    // of a six-step shuffle max)
    const uint64_t fm = __ballot(fits);
    const int lastrow = fm ? __builtin_amdgcn_readlane(rbase + my_rows, 63 - __builtin_clzll(fm)) : 0;
    kept_rows = max(kept_rows, lastrow);
    rb += trows;
    sb += tslots;
  }
  if (spill && l == 0) CAP_FULL(16u);
  wsync();
  // jacobian slots
  for (int base = 0; base < nc * PH_ROWW; base += NT) {
    const int idx = base + l;
    const int c = idx / PH_ROWW, k = idx % PH_ROWW;
    int r1 = 0, r2 = 0;
    uint64_t m1 = 0, m2 = 0;
    if (fastc) {   // (wave-uniform; every lane takes part in the shuffles)
      const int src = min(c, NT - 1);
      r1 = __shfl(kr1, src);
      r2 = __shfl(kr2, src);
      m1 = __shfl(km1, src);
      m2 = __shfl(km2, src);
    }
    // (a contact's slots are one 16-lane DPP row: PH_ROWW = 16; inactive slots take part in the
    // fp32 row reductions below with zeros)
    bool act = c < nc && s.con_rbase[c] >= 0;
    int t0 = 0, t1 = 0, w = 0;
    if (act) {
      t0 = s.con_t[c][0]; t1 = s.con_t[c][1]; w = row_width(m, t0, t1);
      act = k < w;
    }
    T cj[3] = {0, 0, 0};
    if (act) {
      const Con<T>& con = s.con[c];
      const int d = slot_dof(m, t0, t1, k);
      if (!fastc) {
        const int b1 = m.geom_bodyid[con.g1], b2 = m.geom_bodyid[con.g2];
        r1 = m.body_rootid[b1];
        r2 = m.body_rootid[b2];
        m1 = m.body_dofmask[b1];
        m2 = m.body_dofmask[b2];
      }
      T jp1[3], jr1[3], jp2[3], jr2[3];
      jac_col_rm(s, r1, m1, d, con.pos, jp1, jr1);
      jac_col_rm(s, r2, m2, d, con.pos, jp2, jr2);
      const T jd[3] = {jp2[0] - jp1[0], jp2[1] - jp1[1], jp2[2] - jp1[2]};
      for (int a = 0; a < 3; a++) cj[a] = con.frame[3 * a] * jd[0] + con.frame[3 * a + 1] * jd[1] + con.frame[3 * a + 2] * jd[2];
    }
    if constexpr (sizeof(T) == 4 && PNP_F32_SNAP) {
      // A tangent row at the rounding level of its normal row is rounding: two bodies of one tree
      // whose relative motion has no tangential component (the closed gripper's finger pads, face
      // to face: only the finger slides move them apart, along the normal) have J_t = 0 exactly in
      // fp64 (MuJoCo's pyramid edges J_n +- mu J_t are then equal, K1 = 0 and mj_solNoSlip leaves
      // the pair at its mean), but fp32 frames and joint axes rounded apart at ~6e-8 rad give J_t
      // ~1e-7: no-slip then projects the pair on noise and saturates it (the pads' finger
      // accelerations 1.4e-4 off in the tree's M-norm, tools/pads_stage_diag.py).  Such a row (its
      // largest entry within 16 fp32 ulps of the normal row's largest) is snapped to zero, so the
      // edges are equal as in fp64; a resolved tangent (J_t / J_n >~ 2e-6) is unchanged.
      // Only a contact between two bodies of one tree can cancel so (a world-body contact's
      // tangent rows are O(1)): the row reductions run only when the wave holds such a contact
      // (none on the settled C3 scene: cubes on boards).
      const bool same = act && r1 == r2 && r1 != 0;
      if (__ballot(same)) {
        const T nmax = rowmax16(fabs(cj[0])) * T(16 * 1.1920929e-7);
        const T t1m = rowmax16(fabs(cj[1])), t2m = rowmax16(fabs(cj[2]));
        if (same && t1m <= nmax) cj[1] = T(0);
        if (same && t2m <= nmax) cj[2] = T(0);
      }
    }
    if (act) {
      const Con<T>& con = s.con[c];
      const int sb = s.con_sbase[c];
      for (int a = 1; a < con.dim && a < 3; a++) {
        const T fri = con.friction[a - 1];
        s.efc_Jv[sb + (2 * (a - 1)) * w + k] = cj[0] + fri * cj[a];
        s.efc_Jv[sb + (2 * (a - 1) + 1) * w + k] = cj[0] - fri * cj[a];
      }
    }
  }
  // row scalars and impedance (lanes over rows)
  for (int base = 0; base < nc * 4; base += NT) {
    const int idx = base + l;
    const int c = idx / 4, q = idx % 4;
    T tran = 0, rot = 0;
    if (fastc) {
      const int src = min(c, NT - 1);
      tran = __shfl(ktran, src);
      rot = __shfl(krot, src);
    }
    if (c >= nc || s.con_rbase[c] < 0) continue;
    const Con<T>& con = s.con[c];
    if (q >= 2 * (con.dim - 1)) continue;
    const int r = s.con_rbase[c] + q, k = q / 2 + 1;
    const int t0 = s.con_t[c][0], t1 = s.con_t[c][1], w = row_width(m, t0, t1);
    if (!fastc) {
      const int b1 = m.geom_bodyid[con.g1], b2 = m.geom_bodyid[con.g2];
      tran = m.body_invweight0[b1][0] + m.body_invweight0[b2][0];
      rot = m.body_invweight0[b1][1] + m.body_invweight0[b2][1];
    }
    const T fri = con.friction[k - 1];
    s.efc_off[r] = s.con_sbase[c] + q * w;
    s.efc_t0[r] = t0; s.efc_t1[r] = t1;
    s.efc_type[r] = 6; s.efc_id[r] = c;
    row_imp(m, s, r, con.dist, con.includemargin, tran + fri * fri * (k < 3 ? tran : rot), con.solref, con.solimp);
    if (q == 0) s.con_b[c] = s.efc_Jp[r];   // (row_imp parks b there; the same for every row of c)
  }
  if (l == 0) {
    s.nefc = kept_rows;
    s.ne = ne;
  }
  wsync();
}

// ============================================================================ velocity stage
template <typename T>
__device__ void st_velocity(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  // cvel of bodies
  if (l < m.nbody) {
    T cv[6] = {0, 0, 0, 0, 0, 0};
    uint64_t dm = l ? m.body_dofmask[l] : 0;
    while (dm) {
      const int d = __builtin_ctzll(dm);
      dm &= dm - 1;
      for (int t = 0; t < 6; t++) cv[t] += s.cdof[d][t] * s.qvel[d];
    }
    for (int t = 0; t < 6; t++) s.cvel[l][t] = cv[t];
  }
  // cdof_dot
  if (l < m.nv) {
    const int j = m.dof_jntid[l];
    if (m.jnt_type[j] == 0 && l < m.jnt_dofadr[j] + 3) {
      for (int t = 0; t < 6; t++) s.cdofdot[l][t] = 0;
    } else {
      T cv[6] = {0, 0, 0, 0, 0, 0};
      uint64_t vm = m.dof_velmask[l];
      while (vm) {
        const int d = __builtin_ctzll(vm);
        vm &= vm - 1;
        for (int t = 0; t < 6; t++) cv[t] += s.cdof[d][t] * s.qvel[d];
      }
      T r[6];
      t_crossmotion(r, cv, s.cdof[l]);
      for (int t = 0; t < 6; t++) s.cdofdot[l][t] = r[t];
    }
    s.qfrc_passive[l] = -m.dof_damping[l] * s.qvel[l];
  }
  wsync();
  // RNE: cacc, cfrc_body
  if (l > 0 && l < m.nbody) {
    T ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    uint64_t dm = m.body_dofmask[l];
    while (dm) {
      const int d = __builtin_ctzll(dm);
      dm &= dm - 1;
      for (int t = 0; t < 6; t++) ca[t] += s.cdofdot[d][t] * s.qvel[d];
    }
    T f[6], tmp[6], tmp1[6];
    t_mulinertvec(f, s.cinert[l], ca);
    t_mulinertvec(tmp, s.cinert[l], s.cvel[l]);
    t_crossforce(tmp1, s.cvel[l], tmp);
    for (int t = 0; t < 6; t++) s.scr6b[l][t] = f[t] + tmp1[t];
  }
  wsync();
  if (l > 0 && l < m.nbody) {
    T acc[6] = {0, 0, 0, 0, 0, 0};
    uint32_t st = m.body_subtree[l];
    while (st) {
      const int c = __builtin_ctz(st);
      st &= st - 1;
      for (int t = 0; t < 6; t++) acc[t] += s.scr6b[c][t];
    }
    for (int t = 0; t < 6; t++) s.scr6[l][t] = acc[t];
  }
  wsync();
  if (l < m.nv) {
    T v = 0;
    for (int t = 0; t < 6; t++) v += s.cdof[l][t] * s.scr6[m.dof_bodyid[l]][t];
    s.qfrc_bias[l] = v;
  }
  // reference acceleration of the rows: aref = -b (J qvel) - k imp (pos - margin)
  for (int r = l; r < s.nefc; r += NT) {
    s.efc_aref[r] -= s.efc_Jp[r] * row_dot(s, r, s.qvel, T(0));
  }
  wsync();
}

// ============================================================================ acceleration
template <typename T>
__device__ void st_actuation_smooth(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nv) {
    // a dof driven by one actuator (every dof here) reads that actuator's constants by its own
    // index -- one round of independent loads -- instead of walking all nu actuators with a
    // compare per step; same arithmetic (f = 0 + gear * force)
    auto act_force = [&](int i) {
      T ctrl = s.ctrl[i];
      if (m.act_ctrllimited[i]) ctrl = fmin(fmax(ctrl, m.act_ctrlrange[i][0]), m.act_ctrlrange[i][1]);
      const T gear = m.act_gear[i];
      const T len = gear * s.qpos[m.act_qadr[i]], vel = gear * s.qvel[l];
      T force = m.act_gainprm[i][0] * ctrl;
      if (m.act_biastype[i]) force += m.act_biasprm[i][0] + m.act_biasprm[i][1] * len + m.act_biasprm[i][2] * vel;
      if (m.act_forcelimited[i]) force = fmin(fmax(force, m.act_forcerange[i][0]), m.act_forcerange[i][1]);
      return gear * force;
    };
    T f = 0;
    const int ia = m.dof_act[l];
    if (ia >= 0) {
      f += act_force(ia);
    } else if (ia == -2) {
      for (int i = 0; i < m.nu; i++)
        if (m.act_dof[i] == l) f += act_force(i);
    }
    s.qfrc_act[l] = f;
    s.qfrc_smooth[l] = s.qfrc_passive[l] - s.qfrc_bias[l] + f;
  }
  wsync();
  solve_M(m, s, s.qacc_smooth, s.qfrc_smooth);
  for (int r = l; r < s.nefc; r += NT) {
    s.efc_bb[r] = row_dot(s, r, s.qacc_smooth, -s.efc_aref[r]);
  }
  wsync();
}

// ============================================================================ Newton solver
// Island reductions.  The cost separates over islands (block-diagonal M, every row inside one
// island), so the solver runs per island: a single global cost would hide the 1e-10
// improvements of the 4 mg dummy island under the arm's cost in fp32, and a single global step
// length would tie every island to the arm's line search.  Island I is reduced on the 8-lane
// group I (lanes 8I .. 8I+7; <= PH_MAXT = 8 islands, so every island in one pass): the group sums
// its dofs / rows, rowsum8 (three DPP steps) finishes; the groups run concurrently.
template <typename T>
__device__ __forceinline__ T rowsum8(T v) {
  v += dpp_s<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_s<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_s<0x141>(v);   // row_half_mirror: the other quad of the 8
  return v;
}
template <typename T>
__device__ __forceinline__ T group_sum(const Env<T>& s, int I, const T* vd, const T* vr) {
  const int q = lane_id() & 7;
  T acc = 0;
  const int n = s.isl_n[I];
  if (vd)
    for (int c = q; c < n; c += 8) acc += vd[s.isl_dof[I][c]];
  if (vr)
    for (int rr = s.isl_roff[I] + q; rr < s.isl_roff[I + 1]; rr += 8) acc += vr[s.isl_row[rr]];
  return rowsum8(acc);
}
// two island sums in one pass: out[I] over island I's dofs of vd and rows of vr, out2[I] over its
// rows of vr2 -- one row walk, the two group reductions interleaved, one sync (same additions in
// the same order as island_sums(vd, vr) and island_sums(nullptr, vr2))
template <typename T>
__device__ __forceinline__ void island_sums2(Env<T>& s, const T* vd, const T* vr, T* out, const T* vr2, T* out2) {
  const int l = lane_id();
  const int I = l >> 3, q = l & 7;
  if (I < s.nisland) {
    T a = 0, b = 0;
    const int n = s.isl_n[I];
    for (int c = q; c < n; c += 8) a += vd[s.isl_dof[I][c]];
    for (int rr = s.isl_roff[I] + q; rr < s.isl_roff[I + 1]; rr += 8) {
      const int r = s.isl_row[rr];
      a += vr[r];
      b += vr2[r];
    }
    T ta = dpp_s<0xB1>(a), tb = dpp_s<0xB1>(b);
    a += ta; b += tb;
    ta = dpp_s<0x4E>(a); tb = dpp_s<0x4E>(b);
    a += ta; b += tb;
    ta = dpp_s<0x141>(a); tb = dpp_s<0x141>(b);
    a += ta; b += tb;
    if (q == 0) { out[I] = a; out2[I] = b; }
  }
  wsync();
}
// out[I] = group_sum for every island (vd / vr in LDS)
template <typename T>
__device__ __forceinline__ void island_sums(Env<T>& s, const T* vd, const T* vr, T* out) {
  const int l = lane_id();
  const int I = l >> 3;
  if (I < s.nisland) {
    const T c = group_sum(s, I, vd, vr);
    if ((l & 7) == 0) out[I] = c;
  }
  wsync();
}

// jar = J x - aref, active set (store), per-island cost -> out[I]
template <typename T>
__device__ void eval_cost(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, const T* x, bool store, T* out) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nv) s.v1[l] = x[l] - s.qacc_smooth[l];
  wsync();
  if (l < m.nv) s.v2[l] = T(0.5) * s.v1[l] * mulM_row(m, s, l, s.v1);
  for (int r = l; r < s.nefc; r += NT) {
    const T v = row_dot(s, r, x, -s.efc_aref[r]);
    const int a = r < s.ne || v < 0;
    if (store) { s.efc_jar[r] = v; s.efc_act[r] = a; }
    s.ntmp[r] = a ? T(0.5) * s.efc_D[r] * v * v : T(0);
  }
  wsync();
  island_sums(s, s.v2, s.ntmp, out);
}

template <typename T>
__device__ __forceinline__ int row_slot_(const Env<T>& s, int t0, int t1, int tree, int dof) {
  if (t0 == tree) return dof - s.c_tree_dofadr[t0];
  if (t1 == tree) return s.c_tree_dofnum[t0] + dof - s.c_tree_dofadr[t1];
  return -1;
}
#define row_slot(m, t0, t1, tree, dof) row_slot_(s, t0, t1, tree, dof)

// The slot of a lane's own dof (tree t, index li inside it) in row r, or -1.  Every load is
// unconditional (LDS reads cannot fault; invalid slots are clamped to 0 and masked by the caller),
// so consecutive rows' loads can be in flight together instead of one exec-masked branch and
// drain per row.
template <typename T>
__device__ __forceinline__ int own_slot(const Env<T>& s, int r, int t, int li, int& off) {
  const int a = s.efc_t0[r], b = s.efc_t1[r];
  off = s.efc_off[r];
  const int na = s.c_tree_dofnum[a];
  return a == t ? li : (b == t ? na + li : -1);
}
// g + sum over island I's rows of (J(r, slot of the lane's dof) * f1[r]) * f2[r] (f2 may be null),
// rows with an inactive flag skipped when act is set; same operation order as the plain loop
template <typename T>
__device__ __forceinline__ T dof_row_sum(T g, const Env<T>& s, int I, int t, int li, const T* f1, const T* f2,
                                         bool only_active) {
  const int e = s.isl_roff[I + 1];
#pragma unroll 2
  for (int rr = s.isl_roff[I]; rr < e; rr++) {
    const int r = s.isl_row[rr];
    int off;
    const int k = own_slot(s, r, t, li, off);
    const T jv = s.efc_Jv[off + (k >= 0 ? k : 0)];
    T c = jv * f1[r];
    if (f2) c = c * f2[r];
    const bool use = k >= 0 && (!only_active || s.efc_act[r]);
    g = use ? g + c : g;
  }
  return g;
}

// OR over the wave (DPP butterfly in each row of 16, then the four rows)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Islands = trees joined by constraint rows.  Only contact and equality rows can span two trees;
// their tree pairs form an 8 x 8 bit matrix (row t = bits 8t..8t+7) whose transitive closure
// (three boolean squarings) gives the components; island ids follow the lowest tree of each
// component, dofs keep increasing order inside an island (trees are contiguous dof ranges).
// Then the rows of each island (CSR, wave ballots) and the island Hessian entry offsets.
template <typename T, class CLK>
__device__ void build_islands(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  uint64_t e = 0;
  for (int c = l; c < s.ncon; c += NT) {
    if (s.con_rbase[c] >= 0 && s.con_t[c][1] >= 0) {
      const int a = s.con_t[c][0], b = s.con_t[c][1];
      e |= (1ull << (8 * a + b)) | (1ull << (8 * b + a));
    }
  }
  for (int r = l; r < s.ne; r += NT) {
    const int a = s.efc_t0[r], b = s.efc_t1[r];
    if (a >= 0 && b >= 0) e |= (1ull << (8 * a + b)) | (1ull << (8 * b + a));
  }
  const uint64_t E = ((uint64_t)wave_or((uint32_t)(e >> 32)) << 32) | wave_or((uint32_t)e);
  // transitive closure (Warshall on bit rows): lane t < 8 holds row t; step k ORs row k into
  // every row that reaches k.  The rows are then gathered back into the 8 x 8 matrix R.
  uint32_t row = l < 8 ? (uint32_t)(E >> (8 * l)) & 0xFFu : 0u;
  row |= l < 8 ? 1u << l : 0u;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t rk = (uint32_t)__builtin_amdgcn_readlane((int)row, k);
    row = (row >> k & 1u) ? row | rk : row;
  }
  uint64_t R = 0;
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const uint64_t bits = __ballot(row >> b & 1u) & 0xFFull;   // bit t = row t has bit b
#pragma unroll
    for (int t = 0; t < 8; t++) R |= ((bits >> t) & 1ull) << (8 * t + b);
  }
  const int nt = m.ntree;
  uint32_t roots = 0;
#pragma unroll
  for (int t = 0; t < 8; t++)
    if (t < nt && __builtin_ctz((uint32_t)(R >> (8 * t)) & 0xFFu) == t) roots |= 1u << t;
  const int nis = __builtin_popcount(roots);
  auto island_of = [&](int t) {
    const int low = __builtin_ctz((uint32_t)(R >> (8 * t)) & 0xFFu);
    return __builtin_popcount(roots & ((1u << low) - 1u));
  };
  // Island bookkeeping in registers: the tree sizes are read once, island sizes and every
  // per-island offset (Hessian / row / dense-block) are prefix sums over <= 8 islands that each
  // lane forms from readlane broadcasts, and the island row order comes from per-island ballots
  // (a counting sort) instead of one LDS pass over the rows per island.
  int tdn[8];
#pragma unroll
  for (int u = 0; u < 8; u++) tdn[u] = u < nt ? s.c_tree_dofnum[u] : 0;
  if (l < nt) s.tree_island[l] = island_of(l);
  if (l < m.nv) {
    const int t = s.c_dof_tree[l];
    const uint32_t comp = (uint32_t)(R >> (8 * t)) & 0xFFu;
    int pos = l - s.c_tree_dofadr[t];
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (u < t && (comp >> u & 1u)) pos += tdn[u];
    s.isl_dof[island_of(t)][pos] = (unsigned char)l;
    s.dof_ipos[l] = (unsigned char)pos;
  }
  if (l < nt) {
    const uint32_t comp = (uint32_t)(R >> (8 * l)) & 0xFFu;
    int pos = 0;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (u < l && (comp >> u & 1u)) pos += tdn[u];
    s.tree_ipos[l] = pos;
  }
  // island sizes: lane I sums its trees
  int nI = 0;
#pragma unroll
  for (int t = 0; t < 8; t++)
    if (t < nt && island_of(t) == l) nI += tdn[t];
  // rows by island (counting sort): lane J counts island J's rows over the row chunks ...
  int rc = 0;
  const int nefc = s.nefc;
  for (int base = 0; base < nefc; base += NT) {
    const int r = base + l;
    const int I = r < nefc ? island_of(s.efc_t0[r]) : -1;
#pragma unroll
    for (int J = 0; J < 8; J++) {
      if (J >= nis) break;
      const int c = __popcll(__ballot(I == J));
      if (l == J) rc += c;
    }
  }
  // ... exclusive prefix sums over the island lanes (row, Hessian and dense-block offsets) ...
  const bool isl = l < nis;
  int ro = isl ? rc : 0, eo = isl ? nI * (nI + 1) / 2 : 0, jo = isl ? rc * nI : 0;
  // (row_shr inside the first DPP row, zero-filled below the shift: lanes 0..7 get the scan)
  ro += __builtin_amdgcn_mov_dpp(ro, 0x111, 0xF, 0xF, true);
  eo += __builtin_amdgcn_mov_dpp(eo, 0x111, 0xF, 0xF, true);
  jo += __builtin_amdgcn_mov_dpp(jo, 0x111, 0xF, 0xF, true);
  ro += __builtin_amdgcn_mov_dpp(ro, 0x112, 0xF, 0xF, true);
  eo += __builtin_amdgcn_mov_dpp(eo, 0x112, 0xF, 0xF, true);
  jo += __builtin_amdgcn_mov_dpp(jo, 0x112, 0xF, 0xF, true);
  ro += __builtin_amdgcn_mov_dpp(ro, 0x114, 0xF, 0xF, true);
  eo += __builtin_amdgcn_mov_dpp(eo, 0x114, 0xF, 0xF, true);
  jo += __builtin_amdgcn_mov_dpp(jo, 0x114, 0xF, 0xF, true);
  const int rtot = __builtin_amdgcn_readlane(ro, 7), etot = __builtin_amdgcn_readlane(eo, 7),
            jtot = __builtin_amdgcn_readlane(jo, 7);
  // an island with more rows than the line search's per-group register cache (the solver's
  // whole-wave paths start there: PNP_BIG_ISLANDS)
  const bool bigrows = __ballot(isl && rc > PNP_BIG_ROWS) != 0;
  ro -= isl ? rc : 0;
  eo -= isl ? nI * (nI + 1) / 2 : 0;
  jo -= isl ? rc * nI : 0;
  // ... then every row lands at its island's offset + its rank among the island's earlier rows
  int run = ro;
  for (int base = 0; base < nefc; base += NT) {
    const int r = base + l;
    const int I = r < nefc ? island_of(s.efc_t0[r]) : -1;
    const uint64_t below = (1ull << l) - 1;
#pragma unroll
    for (int J = 0; J < 8; J++) {
      if (J >= nis) break;
      const uint64_t bal = __ballot(I == J);
      const int at = __builtin_amdgcn_readlane(run, J);
      if (I == J) s.isl_row[at + __popcll(bal & below)] = (short)r;
      if (l == J) run += __popcll(bal);
    }
  }
  // per-island tables: lane I writes its entries, lane 0 the end markers
  if (isl) {
    s.isl_n[l] = nI;
    s.isl_roff[l] = ro;
    s.isl_eoff[l] = eo;
    s.isl_joff[l] = jo;
  }
  if (l == 0) {
    s.nisland = nis;
    s.isl_roff[nis] = rtot;
    s.isl_eoff[nis] = etot;
    s.isl_joff[nis] = jtot;
    s.jt_ok = jtot <= PH_JTCAP;
    // the widest tier's jt decides dense vs slot path (a tier that can hand over does so when its
    // jt is too small); the full / wide Hessian stores fit every island partition of PH_MAXV
    // dofs, the compact build's the common ones
    if ((PNP_COMPACT || (PNP_HANDS && s.hand)) && (!s.jt_ok || etot > PH_HCAP)) s.ovf |= PNP_OVF_JT;
    // the compact build has no whole-wave solver paths: it hands such islands over
    if (!PNP_BIG_ISLANDS && bigrows) s.ovf |= PNP_OVF_JT;
  }
  wsync();
  clk.aux_lap(SC_AUX0 + 3);   // aux3: islands (closure, dof lists, row lists)
  // dense island Jacobian blocks: zero, then lane per row scatters its packed slots (tree t's
  // slots are contiguous columns from tree_ipos[t] in the island's dof order)
  if (s.jt_ok) {
    const int tot = s.isl_joff[nis];
    for (int e = l; e < tot; e += NT) s.jt[e] = T(0);
    wsync();
    for (int rr = l; rr < s.nefc; rr += NT) {
      const int r = s.isl_row[rr];
      const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], off = s.efc_off[r];
      const int I = s.tree_island[t0], n = s.isl_n[I];
      T* row = s.jt + s.isl_joff[I] + (rr - s.isl_roff[I]) * n;
      const int n0 = s.c_tree_dofnum[t0], w = row_width(m, t0, t1);
      const int p0 = s.tree_ipos[t0], p1 = t1 >= 0 ? s.tree_ipos[t1] - n0 : 0;
      for (int k = 0; k < w; k++) row[k < n0 ? p0 + k : p1 + k] = s.efc_Jv[off + k];
    }
    wsync();
  }
  clk.aux_lap(SC_AUX0 + 4);   // aux4: dense island Jacobian blocks
}

// g + sum over island I's rows (island row order) of jt(row, a) * f[row] with the dense blocks:
// a = the dof's island position, f in island row order (zero for rows that do not count)
template <typename T>
__device__ __forceinline__ T jt_dof_sum(const Env<T>& s, int I, int a, T g, const T* f) {
  const int n = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0;
  const T* col = s.jt + s.isl_joff[I] + a;
  const T* fr = f + r0;
#pragma unroll 4
  for (int k = 0; k < nr; k++) g += col[k * n] * fr[k];
  return g;
}
// out[rr] = v[isl_row[rr]] (island row order)
template <typename T>
__device__ __forceinline__ void gather_rows(const Env<T>& s, const T* v, T* out) {
  for (int rr = lane_id(); rr < s.nefc; rr += NT) out[rr] = v[s.isl_row[rr]];
}

// Cholesky + solve of one island's Hessian block held in registers (n <= N), lane-private.
// out = -(H^-1) g on the island's dofs.  The block is Jacobi-scaled first (H' = S H S with
// S = diag(H)^-1/2): islands mix a 1e-12 kg m^2 rotational inertia (the r = 1 mm dummy sphere)
// with 1e-5 constraint terms, and unscaled fp32 Cholesky would lose most digits there.
template <typename T, int N>
__device__ __forceinline__ void island_newton_dir_reg(Env<T>& s, int I, int n) {
  const unsigned char* idx = s.isl_dof[I];
  int id[N];
#pragma unroll
  for (int a = 0; a < N; a++) id[a] = a < n ? idx[a] : 0;
  T sc[N];
#pragma unroll
  for (int a = 0; a < N; a++) {
    const T h = a < n ? HI(I, a, a) : T(1);
    sc[a] = h > T(0) ? T(1) / PM<T>::sqrt_(h) : T(1);
  }
  T L[N * (N + 1) / 2];
#pragma unroll
  for (int a = 0; a < N; a++)
#pragma unroll
    for (int b = 0; b <= a; b++) L[a * (a + 1) / 2 + b] = a < n ? HI(I, a, b) * sc[a] * sc[b] : T(a == b);
#pragma unroll
  for (int j = 0; j < N; j++) {
    T d = L[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; k++) d -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
    d = PM<T>::sqrt_(d > T(0) ? d : T(1e-30));
    L[j * (j + 1) / 2 + j] = d;
    const T inv = T(1) / d;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      T t = L[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
      L[i * (i + 1) / 2 + j] = t * inv;
    }
  }
  T y[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    T v = i < n ? s.grad[id[i]] * sc[i] : T(0);
#pragma unroll
    for (int k = 0; k < i; k++) v -= L[i * (i + 1) / 2 + k] * y[k];
    y[i] = v / L[i * (i + 1) / 2 + i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    T v = y[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) v -= L[k * (k + 1) / 2 + i] * y[k];
    y[i] = v / L[i * (i + 1) / 2 + i];
  }
#pragma unroll
  for (int i = 0; i < N; i++)
    if (i < n) s.p[id[i]] = -y[i] * sc[i];
}

// Newton direction of one island of more than 9 dofs (a merged island: the arm holding a box, or
// resting on one) on the whole wave, in place of the packed block (the factor consumes H).  Jacobi
// scaling as island_newton_dir_reg.  Factor: left-looking Cholesky in chol_reg's operation order;
// lane r keeps row r of the scaled block in registers and publishes each finished entry L[r][j]
// into the packed block, and column j's pivot and every lane's row term read the finished row j
// from there (one address per wave: broadcast reads).  Solves by columns: forward, y_k from lane
// k's right-hand side (readlane) and every lane r > k subtracting L[r][k] y_k from its own (the
// row-oriented order); back, x_k likewise and lane r < k subtracting L[k][r] x_k, read from the
// packed factor.  (Lane-serial, this island's factor and solves were a chain of ~n^3 / 3
// dependent LDS round trips: 100-200k cycles per Newton iteration for 15-21 dofs.)
// NB: the register row length, a compile-time bound on n (the loops must unroll completely, or
// the row array goes to scratch).  One instantiation (PH_MAXV): a dispatch over 16 / 24 / 36 cost
// C3 1.1 % through st_newton's register allocation around the three call sites.
template <typename T, int NB>
__device__ __attribute__((noinline)) void island_newton_dir_wave(Env<T>& s, int I, int n) {
  const int l = lane_id();
  const bool lr = l < n;
  const int rc = lr ? l : 0;
  T* Hb = s.Hp + s.isl_eoff[I];   // entry (a, b), a >= b, at a (a + 1) / 2 + b
  const int id = s.isl_dof[I][rc];
  const T hd = Hb[rc * (rc + 1) / 2 + rc];
  const T sc = lr && hd > T(0) ? T(1) / PM<T>::sqrt_(hd) : T(1);
  T A[NB];
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const T sj = rdlane(sc, j < NT ? j : 0);
    const T h = Hb[rc * (rc + 1) / 2 + (j <= rc ? j : 0)];
    A[j] = lr && j <= l ? h * sc * sj : T(l == j);
  }
  wsync();   // every row is in registers before the factor overwrites the block
  // (every loop has a constant trip count and guards on n, so that all of them unroll and the
  // row stays in registers)
#pragma unroll
  for (int j = 0; j < NB; j++) {
    if (j < n) {
      const T* Lj = Hb + j * (j + 1) / 2;   // finished row j of the factor (entries k < j)
      T td = rdlane(A[j], j);
      T t = A[j];
#pragma unroll
      for (int k = 0; k < j; k++) {
        const T ljk = Lj[k];
        td -= ljk * ljk;
        t -= A[k] * ljk;
      }
      const T d = PM<T>::sqrt_(td > T(0) ? td : T(1e-30));
      const T inv = T(1) / d;
      A[j] = l == j ? d : (l > j ? t * inv : A[j]);
      if (lr && l >= j) Hb[l * (l + 1) / 2 + j] = A[j];
      wsync();
    }
  }
  // forward: y = L^-1 (S g)
  T b = lr ? s.grad[id] * sc : T(0);
#pragma unroll
  for (int k = 0; k < NB; k++) {
    if (k < n) {
      const T yk = rdlane(b, k) / rdlane(A[k], k);
      b = l == k ? yk : (l > k ? b - A[k] * yk : b);
    }
  }
  // back: x = L^-T y
#pragma unroll
  for (int k = NB - 1; k >= 0; k--) {
    if (k < n) {
      const T lkr = Hb[k * (k + 1) / 2 + (l < k ? l : 0)];
      const T xk = rdlane(b, k) / rdlane(A[k], k);
      b = l == k ? xk : (l < k ? b - lkr * xk : b);
    }
  }
  if (lr) s.p[id] = -b * sc;
  wsync();
}

// Exact minimiser of each island's convex piecewise quadratic phi_I(a) = cost_I(x + a p)
// (semi-smooth Newton on phi', bracketed).  Island I runs on the 8-lane group I = lane >> 3: its
// rows are summed by the group's lanes with rowsum8 (three DPP steps), so all 8 islands bracket
// at once, each independently of the others.  An island stops once its Newton step is at the
// rounding level of the step length (|a_new - a| <= 4 eps |a|) or its bracket has collapsed.
// Islands with isl_flag set (done) keep a = 0.  Leaves the step lengths in s.isl_alpha.
// ---------------------------------------------------------------- fp32: per-island Newton
// The fp32 builds solve every island to its exact minimiser on its own (per-island warm start,
// exact line search and convergence), as before round 4.  MuJoCo's iteration (one step length and
// one improvement / gradient test for the whole problem, st_newton below) cannot be carried in
// fp32: the arm island's cost and derivative carry rounding of ~1e-7 x (weld forces x rows), which
// swamps a cube island's whole contribution to the shared line-search derivative and improvement
// -- measured (round 4, the global variant in fp32): a cube's velocity change 0.137 off the oracle,
// qacc 3.8e-4 -- whereas the islands' exact minimisers are what MuJoCo's fp64 iteration reaches
// once the active set settles (its exits fire at gradient ~1e-16 after the step that lands there).
// The fp64 instantiation runs MuJoCo's iteration and exits exactly (tools/noslip_exit_diag.py:
// iteration counts equal to the oracle's env by env).
template <typename T, class CLK>
__device__ void line_search_islands(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nv) s.v1[l] = s.x[l] - s.qacc_smooth[l];
  for (int r = l; r < s.nefc; r += NT) {
    s.efc_Jp[r] = row_dot(s, r, s.p, T(0));
  }
  wsync();
  if (l < m.nv) {
    const T mp = mulM_row(m, s, l, s.p);
    s.v2[l] = mp * s.p[l];
    s.grad[l] = mp * s.v1[l];   // the gradient is no longer needed this iteration
  }
  wsync();
  clk.aux_lap(SC_AUX0 + 5);   // aux5: line search J p, M p
  const int q = l & 7;
  int itc = 0;   // bracketing iterations of the lane's island (stage profile count)
  // Islands with more rows than a group's register cache (closed fingers pressed together put
  // 200-400 rows on the arm island): bracketed on the whole wave, one after the other, each
  // row read once per bracketing iteration by 64 lanes (the group path below would walk it 8
  // rows at a time, ~35 dependent LDS rounds per iteration).  Same bracketing; the row sums
  // reduce over 64 lanes instead of 8 (rounding only).
  constexpr int RK = PNP_BIG_ROWS / 8;
  const uint32_t big = PNP_BIG_ISLANDS ? (uint32_t)__ballot(l < s.nisland && !s.isl_flag[l] &&
                                                            s.isl_roff[l + 1] - s.isl_roff[l] > 8 * RK)
                                       : 0u;
  for (uint32_t bm = big; bm; bm &= bm - 1) {
    const int I = __builtin_ctz(bm);
    const int n = s.isl_n[I];
    const T A0 = wsum(l < n ? s.v2[s.isl_dof[I][l]] : T(0)), B0 = wsum(l < n ? s.grad[s.isl_dof[I][l]] : T(0));
    const int r0 = s.isl_roff[I], r1 = s.isl_roff[I + 1];
    T lo = 0, hi = T(-1), a = 1;
    int it = 0;
    for (; it < 60; it++) {
      T d1 = 0, d2 = 0;
      for (int rr = r0 + l; rr < r1; rr += NT) {
        const int r = s.isl_row[rr];
        const T jp = s.efc_Jp[r], v = s.efc_jar[r] + a * jp;
        if (r < s.ne || v < 0) { d1 += s.efc_D[r] * v * jp; d2 += s.efc_D[r] * jp * jp; }
      }
      d1 = wsum(d1) + A0 * a + B0;
      d2 = wsum(d2) + A0;
      if (!(d2 > T(0))) { a = 0; break; }
      if (d1 == T(0)) break;
      if (d1 > 0) hi = a; else lo = a;
      T an = a - d1 / d2;
      if (!(an > lo) || (hi >= T(0) && !(an < hi))) an = hi >= T(0) ? T(0.5) * (lo + hi) : T(2) * a;
      const bool fin = fabs(an - a) <= T(4) * PM<T>::eps() * fabs(a) || (hi >= T(0) && hi - lo <= PM<T>::eps() * hi);
      a = an;
      if (fin) break;
    }
    if (l == 0) s.isl_alpha[I] = a;
    if ((l >> 3) == I) itc = it + 1;
  }
  {
    const int I = l >> 3;
    if (I >= s.nisland || (big >> I & 1u)) goto ls_done;
    if (s.isl_flag[I]) {
      if (q == 0) s.isl_alpha[I] = 0;
      goto ls_done;
    }
    const T A0 = group_sum(s, I, s.v2, (const T*)nullptr), B0 = group_sum(s, I, s.grad, (const T*)nullptr);
    const int r0 = s.isl_roff[I], r1 = s.isl_roff[I + 1];
    // the lane's rows (rr = r0 + q + 8 k) are fixed over the iterations: islands of up to 32
    // rows keep (Jp, jar, D, equality) in registers (larger ones took the wave path above)
    T rjp[RK], rjar[RK], rD[RK];
    bool req[RK], rin[RK];
#pragma unroll
    for (int k = 0; k < RK; k++) {
      const int rr = r0 + q + 8 * k;
      rin[k] = rr < r1;
      const int r = s.isl_row[rin[k] ? rr : r0];
      rjp[k] = s.efc_Jp[r];
      rjar[k] = s.efc_jar[r];
      rD[k] = s.efc_D[r];
      req[k] = r < s.ne;
    }
    const bool small = r1 - r0 <= 8 * RK;
    T lo = 0, hi = T(-1), a = 1;
    for (int it = 0; it < 60; it++) {
      itc++;
      T d1 = 0, d2 = 0;
      if (small) {
#pragma unroll
        for (int k = 0; k < RK; k++) {
          const T jp = rjp[k], v = rjar[k] + a * jp;
          const bool on = rin[k] && (req[k] || v < 0);
          d1 = on ? d1 + rD[k] * v * jp : d1;
          d2 = on ? d2 + rD[k] * jp * jp : d2;
        }
      } else {
        for (int rr = r0 + q; rr < r1; rr += 8) {
          const int r = s.isl_row[rr];
          const T jp = s.efc_Jp[r], v = s.efc_jar[r] + a * jp;
          if (r < s.ne || v < 0) { d1 += s.efc_D[r] * v * jp; d2 += s.efc_D[r] * jp * jp; }
        }
      }
      d1 = rowsum8(d1) + A0 * a + B0;
      d2 = rowsum8(d2) + A0;
      if (!(d2 > T(0))) { a = 0; break; }
      if (d1 == T(0)) break;
      if (d1 > 0) hi = a; else lo = a;
      T an = a - d1 / d2;
      if (!(an > lo) || (hi >= T(0) && !(an < hi))) an = hi >= T(0) ? T(0.5) * (lo + hi) : T(2) * a;
      // converged once the Newton step is at the rounding level of a (waiting for an == a bit
      // for bit cost extra rounds of last-bit oscillation), or the bracket has collapsed
      const bool fin = fabs(an - a) <= T(4) * PM<T>::eps() * fabs(a) || (hi >= T(0) && hi - lo <= PM<T>::eps() * hi);
      a = an;
      if (fin) break;
    }
    if (q == 0) s.isl_alpha[I] = a;
  }
ls_done:
  wsync();
  clk.aux_lap(SC_AUX0 + 6);   // aux6: line search bracketing per island
  {
    int mx = 0;
#pragma unroll
    for (int g = 0; g < 8; g++) mx = max(mx, __builtin_amdgcn_readlane(itc, 8 * g));
    clk.count(SC_AUX0 + 7, mx);   // aux7: line-search bracketing iterations (max over islands)
  }
}

template <typename T, class CLK>
__device__ T line_search(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  // MuJoCo 2.3.3 PrimalLineSearch: one step length for the whole problem (2.3.3 has no islands),
  // along the Newton direction p of every island: 0 when |p| < mjMINVAL (or phi'(0) >= 0), else
  // the exact minimiser of the convex piecewise quadratic phi(a) = cost(x + a p) by Newton steps on
  // phi' with bracketing (MuJoCo's iterate stops at |phi'| < gtol; the exact minimiser is the
  // oracle's).  Lane l holds rows l + 64 k (k < 2) in registers; larger row counts
  // stream the rest from LDS (the wide tier's 200-700 rows).  Returns the step (wave-uniform);
  // the fp64 instantiation's (st_newton; the fp32 builds: line_search_islands).
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nv) s.v1[l] = s.x[l] - s.qacc_smooth[l];
  for (int r = l; r < s.nefc; r += NT) {
    s.efc_Jp[r] = row_dot(s, r, s.p, T(0));
  }
  wsync();
  T pp = 0, A0 = 0, B0 = 0;
  if (l < m.nv) {
    const T mp = mulM_row(m, s, l, s.p);
    A0 = mp * s.p[l];
    B0 = mp * s.v1[l];
    pp = s.p[l] * s.p[l];
  }
  A0 = wsum(A0);
  B0 = wsum(B0);
  const T snorm = PM<T>::sqrt_(wsum(pp));
  clk.aux_lap(SC_AUX0 + 5);   // aux5: line search J p, M p
  const int n = s.nefc, ne = s.ne;
  T rjp[2], rjar[2], rD[2];
  bool req[2], rin[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int r = l + NT * k;
    rin[k] = r < n;
    const int rc = rin[k] ? r : 0;
    rjp[k] = s.efc_Jp[rc];
    rjar[k] = s.efc_jar[rc];
    rD[k] = s.efc_D[rc];
    req[k] = r < ne;
  }
  // phi'(a) - (A0 a + B0) and phi''(a) - A0 over the rows active at a (equality rows always)
  auto deriv = [&](T a, T& d1, T& d2) {
    d1 = 0;
    d2 = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const T jp = rjp[k], v = rjar[k] + a * jp;
      const bool on = rin[k] && (req[k] || v < 0);
      d1 = on ? d1 + rD[k] * v * jp : d1;
      d2 = on ? d2 + rD[k] * jp * jp : d2;
    }
    for (int r = l + 2 * NT; r < n; r += NT) {
      const T jp = s.efc_Jp[r], v = s.efc_jar[r] + a * jp;
      if (r < ne || v < 0) { d1 += s.efc_D[r] * v * jp; d2 += s.efc_D[r] * jp * jp; }
    }
    d1 = wsum(d1) + A0 * a + B0;
    d2 = wsum(d2) + A0;
  };
  T a = 0;
  int it = 0;
  if (snorm >= T(1e-15)) {
    T d1, d2;
    deriv(T(0), d1, d2);
    if (d1 < T(0)) {
      T lo = 0, hi = T(-1);
      a = 1;
      for (; it < 60; it++) {
        deriv(a, d1, d2);
        if (!(d2 > T(0))) { a = 0; break; }
        if (d1 == T(0)) break;
        if (d1 > 0) hi = a; else lo = a;
        T an = a - d1 / d2;
        if (!(an > lo) || (hi >= T(0) && !(an < hi))) an = hi >= T(0) ? T(0.5) * (lo + hi) : T(2) * a;
        // converged once the Newton step is at the rounding level of a (waiting for an == a bit
        // for bit costs extra rounds of last-bit oscillation), or the bracket has collapsed
        const bool fin = fabs(an - a) <= T(4) * PM<T>::eps() * fabs(a) || (hi >= T(0) && hi - lo <= PM<T>::eps() * hi);
        a = an;
        if (fin) break;
      }
    }
  }
  clk.aux_lap(SC_AUX0 + 6);   // aux6: line search bracketing
  clk.count(SC_AUX0 + 7, it + 1);   // aux7: line-search bracketing iterations
  return a;
}

// Newton direction of every island on its own 9-lane group (see st_newton); out of line so that
// its ~80 live factor / solve registers do not raise the register pressure of the whole solver
// (callee-saved spills of every st_newton call)
template <typename T>
__device__ __attribute__((noinline)) void newton_dir_groups(Env<T>& s, bool done) {
  const int l = lane_id();
  // every island on its own 9-lane group; the Jacobi-scaled factor is kept in NL while the
  // island's H block stays valid (isl_hvalid), so a refining step only solves
  const int g = gch_group(l), r = l - GCH_N * g, base = GCH_N * g;
  const bool on = g < s.nisland && !s.isl_flag[g];
  const int n = on ? s.isl_n[g] : 0;
  const int rc = r < n ? r : 0;
  const int id = s.isl_dof[g][rc];
  const int e0 = on ? s.isl_eoff[g] : 0;
  const T* Hg = s.Hp + e0;   // the island's packed block (entry (a, b) at a (a + 1) / 2 + b)
  const T hd = Hg[rc * (rc + 1) / 2 + rc];
  const T sc = r < n && hd > T(0) ? T(1) / PM<T>::sqrt_(hd) : T(1);
  T Lrow[GCH_N], Ad[GCH_N], scv[GCH_N], P[45], y[GCH_N];
#pragma unroll
  for (int i = 0; i < GCH_N; i++)
#pragma unroll
    for (int k = 0; k <= i; k++) P[i * (i + 1) / 2 + k] = T(i == k);
  T* Ls = &s.NL[0][0][0];
  const bool fac = on && !s.isl_hvalid[g];
#pragma unroll
  for (int j = 0; j < GCH_N; j++) {
    scv[j] = __shfl(sc, base + j);
    const int jc = j < n ? j : 0;
    const int idj = s.isl_dof[g][jc];
    Lrow[j] = fac && r < n && j <= r ? Hg[rc * (rc + 1) / 2 + (j <= rc ? j : 0)] * sc * scv[j] : T(r == j);
    Ad[j] = j < n ? Hg[jc * (jc + 1) / 2 + jc] * scv[j] * scv[j] : T(1);
    y[j] = j < n ? s.grad[idj] * scv[j] : T(0);
  }
  if (__ballot(fac)) gch_factor(Lrow, Ad, r, base, P);
  if (fac)
#pragma unroll
    for (int j = 0; j < GCH_N; j++) Ls[(base + r) * GCH_N + j] = Lrow[j];
  if (on && !fac)   // H block unchanged since its factorisation: the kept factor
#pragma unroll
    for (int i = 0; i < GCH_N; i++)
#pragma unroll
      for (int k = 0; k <= i; k++) P[i * (i + 1) / 2 + k] = i < n ? Ls[(base + i) * GCH_N + k] : T(i == k);
  chol_solve_reg<T, GCH_N>(P, GCH_N, y, y);
  T x = 0;
#pragma unroll
  for (int i = 0; i < GCH_N; i++) x = r == i ? y[i] : x;
  if (on && r < n) s.p[id] = -x * sc;
  wsync();
  if (l < s.nisland && !done) s.isl_hvalid[l] = 1;
}

// Hessian block of an island with many rows (closed fingers: 200-400 rows on the arm island) on
// the matrix cores: J^T diag(D) J is a (n x nr) (nr x n) product, n <= 16 island dofs, so one
// v_mfma_f32_16x16x4_f32 tile per 4 rows (A = J^T: lane l holds J[k0 + l/16][l%16], B = D J:
// the same element times D), two independent accumulators (the MFMA's dependent latency is 40
// cycles), then M's block entries added and the lower triangle stored.  The scalar path (lane
// per entry) walks every row once per entry.  fp32 MFMA is exact f32 (an fmaf chain per
// element); the sums associate differently from the scalar loop (rounding only).
__device__ __attribute__((noinline)) void hess_mfma(Env<float>& s, int I) {
  const int l = lane_id();
  const int n = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0;
  const float* J = s.jt + s.isl_joff[I];
  const float* D = s.rr_d + r0;
  const int c = l & 15, kk = l >> 4;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  auto elem = [&](int k, float& x, float& dx) {
    const bool on = k < nr && c < n;
    const float v = J[on ? k * n + c : 0], d = D[k < nr ? k : 0];
    x = on ? v : 0.f;
    dx = on ? d * v : 0.f;
  };
  int k0 = 0;
  for (; k0 + 8 <= nr; k0 += 8) {
    float x0, b0, x1, b1;
    elem(k0 + kk, x0, b0);
    elem(k0 + 4 + kk, x1, b1);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1, b1, acc1, 0, 0, 0);
  }
  for (; k0 < nr; k0 += 4) {
    float x0, b0;
    elem(k0 + kk, x0, b0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, b0, acc0, 0, 0, 0);
  }
  // lane l holds H[4 (l / 16) + r][l % 16], r = 0..3
  const int e0 = s.isl_eoff[I];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int a = 4 * kk + r, b = c;
    if (a < n && b <= a) {
      const int i = s.isl_dof[I][a], j = s.isl_dof[I][b];
      const int ti = s.c_dof_tree[i], tj = s.c_dof_tree[j];
      const float h = ti == tj ? s.M[mblk(m, i, j)] : 0.f;
      s.Hp[e0 + a * (a + 1) / 2 + b] = h + (acc0[r] + acc1[r]);
    }
  }
}

// ---- fp32 Newton: mixed-precision iterative refinement
// Once an island's Newton step kept its active set, x is the minimiser of that quadratic up to the
// fp32 solve's own error, cond(H) eps: with the closed fingers' pad contacts (200+ rows on the
// arm, cond(H) ~6e3) ~5e-6 of |x|, and a second fp32 Newton step does not improve it (its gradient
// carries the same fp32 rounding; round 4: the closed-finger fixture's arm tree 1.4-1.6e-4 against
// a one-ulp floor of 5e-5).  Instead: the gradient g = M (x - x_smooth) + J^T D (J x - aref) of
// that quadratic accumulated in fp64 from the fp32 data (products of fp32 values are exact in
// fp64; D (J x - aref) is kept as an fp32 pair), then p = -H^-1 g with the island's kept factor
// and x += p, no line search (the quadratic's own minimiser); the rows' jar / active set are
// re-evaluated at the new x (fp64 accumulation).  An island whose active set still holds is done;
// one whose set changed goes on with Newton iterations.  (CPU model of the arm island, tools/
// mpir_model.py: fp32 Newton + fp32 refinement 1.4-1.2e-5 .. 5e-6 of |x|, one fp64-residual
// refinement 6e-8 .. 1.3e-7 -- the fp32 data's own rounding.)  This replaces the second,
// line-searched Newton iteration fp32 ran on 63 % of the C3 sub-steps.
template <typename T>
__device__ __forceinline__ double row_dot64(const Env<T>& s, int r, const T* x) {
  const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], off = s.efc_off[r];
  const int n0 = s.c_tree_dofnum[t0], a0 = s.c_tree_dofadr[t0];
  const int t1c = t1 >= 0 ? t1 : 0;
  const int n1 = t1 >= 0 ? s.c_tree_dofnum[t1c] : 0, a1 = s.c_tree_dofadr[t1c];
  const T* J = s.efc_Jv + off;
  double v = 0;
#pragma unroll 3
  for (int q = 0; q < n0; q++) v += (double)J[q] * (double)x[a0 + q];
#pragma unroll 3
  for (int q = 0; q < n1; q++) v += (double)J[n0 + q] * (double)x[a1 + q];
  return v;
}
// fp64 gradient of the island quadratics at x (active set efc_act, dense island blocks): s.grad =
// g rounded to fp32, s.v2 = g^2 (for the island norms)
__device__ __attribute__((noinline)) void newton_refine_grad(Env<float>& s) {
  const DevPhys<float>& m = phys<float>();
  const int l = lane_id();
  const int nisl = s.nisland;
  // rows, island row order: f = D (J x - aref) on the active rows, an fp32 pair (rr_f + rr_d; the
  // Hessian blocks are kept, so rr_d is free)
  for (int rr = l; rr < s.nefc; rr += NT) {
    const int r = s.isl_row[rr];
    const double jar = row_dot64(s, r, s.x) - (double)s.efc_aref[r];
    const double f = s.efc_act[r] ? (double)s.efc_D[r] * jar : 0.0;
    const float hi = (float)f;
    s.rr_f[rr] = hi;
    s.rr_d[rr] = (float)(f - (double)hi);
  }
  wsync();
  // islands with more rows than a wave: lane (dof a, slice k) sums rows k, k + S .. in fp64 (as the
  // fp32 gradient's whole-wave path), partials as fp32 pairs in ntmp, then lane a's sum as a pair
  // in v2 / p (p is rewritten by the direction below)
  const uint32_t bigg = PNP_BIG_ISLANDS ? (uint32_t)__ballot(l < nisl && s.isl_roff[l + 1] - s.isl_roff[l] > NT &&
                                                             s.isl_n[l] <= 32)
                                        : 0u;
  for (uint32_t bm = bigg; bm; bm &= bm - 1) {
    const int I = __builtin_ctz(bm);
    const int n = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0, S = NT / n;
    const int a = l % n, k0 = l / n;
    if (k0 < S) {
      const float* col = s.jt + s.isl_joff[I] + a;
      double part = 0;
      for (int k = k0; k < nr; k += S) part += (double)col[k * n] * ((double)s.rr_f[r0 + k] + (double)s.rr_d[r0 + k]);
      const float hi = (float)part;
      s.ntmp[l] = hi;
      s.ntmp[NT + l] = (float)(part - (double)hi);
    }
    wsync();
    if (l < n) {
      double g = 0;
      for (int k = 0; k < S; k++) g += (double)s.ntmp[l + k * n] + (double)s.ntmp[NT + l + k * n];
      const int d = s.isl_dof[I][l];
      const float hi = (float)g;
      s.v2[d] = hi;
      s.p[d] = (float)(g - (double)hi);
    }
    wsync();
  }
  if (l < m.nv) {
    const int t = s.c_dof_tree[l], I = s.tree_island[t];
    const int a = s.c_tree_dofadr[t], n = s.c_tree_dofnum[t], o = s.c_tree_moff[t] + (l - a) * n;
    double g = 0;
    for (int k = 0; k < n; k++) g += (double)s.M[o + k] * ((double)s.x[a + k] - (double)s.qacc_smooth[a + k]);
    if (bigg >> I & 1u) {
      g += (double)s.v2[l] + (double)s.p[l];
    } else {
      const int ni = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0;
      const float* col = s.jt + s.isl_joff[I] + s.dof_ipos[l];
#pragma unroll 4
      for (int k = 0; k < nr; k++) g += (double)col[k * ni] * ((double)s.rr_f[r0 + k] + (double)s.rr_d[r0 + k]);
    }
    s.grad[l] = (float)g;
    s.v2[l] = (float)(g * g);
  }
  wsync();
}
// x += p on the live islands (isl_flag clear), their rows' jar and active set re-evaluated at the
// new x (fp64 accumulation, rounded once); per island whether its active set changed -> isl_val
__device__ __attribute__((noinline)) void newton_refine_update(Env<float>& s) {
  const DevPhys<float>& m = phys<float>();
  const int l = lane_id();
  if (l < m.nv && !s.isl_flag[s.tree_island[s.c_dof_tree[l]]]) s.x[l] += s.p[l];
  wsync();
  for (int r = l; r < s.nefc; r += NT) {
    const unsigned char old = s.efc_act[r];
    s.efc_Jp[r] = (float)old;
    if (s.isl_flag[s.tree_island[s.efc_t0[r]]]) continue;
    const double jar = row_dot64(s, r, s.x) - (double)s.efc_aref[r];
    s.efc_jar[r] = (float)jar;
    s.efc_act[r] = r < s.ne || jar < 0;
  }
  wsync();
  {
    const int q = l & 7, I = l >> 3;
    bool ch = false;
    if (I < s.nisland)
      for (int rr = s.isl_roff[I] + q; rr < s.isl_roff[I + 1]; rr += 8) {
        const int r = s.isl_row[rr];
        ch |= (float)s.efc_act[r] != s.efc_Jp[r];
      }
    const bool any = ((__ballot(ch) >> (l & 56)) & 0xFFull) != 0;
    if (I < s.nisland && q == 0) s.isl_val[I] = any ? 1.0f : 0.0f;
  }
  wsync();
}

template <typename T, class CLK>
__device__ void st_newton_islands(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (s.nefc == 0) {
    if (l < m.nv) s.qacc[l] = s.qacc_smooth[l];
    if (l == 0) s.solver_iter = 0;
    wsync();
    return;
  }
  clk.aux_start();
  build_islands(m, s, clk);
  if (PNP_HANDS && s.ovf) return;
  // warm start per island: the better of qacc_warmstart and qacc_smooth (MuJoCo chooses for the
  // whole problem; per island the minimiser is the same and the start is better).  One pass:
  // cost(qacc_smooth) has no dof term and its jar is efc_bb (= J qacc_smooth - aref, same
  // arithmetic), and the chosen start's jar / active set are kept instead of re-evaluated.
  if (l < m.nv) s.v1[l] = s.qacc_ws[l] - s.qacc_smooth[l];
  wsync();
  if (l < m.nv) s.v2[l] = T(0.5) * s.v1[l] * mulM_row(m, s, l, s.v1);
  for (int r = l; r < s.nefc; r += NT) {
    const T v = row_dot(s, r, s.qacc_ws, -s.efc_aref[r]);
    const T bs = s.efc_bb[r];
    s.efc_jar[r] = v;
    s.ntmp[r] = r < s.ne || v < 0 ? T(0.5) * s.efc_D[r] * v * v : T(0);
    s.efc_Jp[r] = r < s.ne || bs < 0 ? T(0.5) * s.efc_D[r] * bs * bs : T(0);
  }
  wsync();
  island_sums2(s, s.v2, s.ntmp, s.isl_val, s.efc_Jp, s.isl_cost);
  if (l < PH_MAXT) {
    const bool ws = l < s.nisland && s.isl_val[l] < s.isl_cost[l];
    s.isl_alpha[l] = ws ? T(1) : T(0);
    if (ws) s.isl_cost[l] = s.isl_val[l];
    s.isl_flag[l] = 0;
    s.isl_hvalid[l] = 0;
  }
  wsync();
  if (l < m.nv) s.x[l] = s.isl_alpha[s.tree_island[s.c_dof_tree[l]]] != T(0) ? s.qacc_ws[l] : s.qacc_smooth[l];
  for (int r = l; r < s.nefc; r += NT) {
    const T v = s.isl_alpha[s.tree_island[s.efc_t0[r]]] != T(0) ? s.efc_jar[r] : s.efc_bb[r];
    s.efc_jar[r] = v;
    s.efc_act[r] = r < s.ne || v < 0;
  }
  wsync();
  clk.lap(8);
  // lane I (< nisland) keeps island I's convergence state
  T cost = l < s.nisland ? s.isl_cost[l] : T(0);
  bool done = l >= s.nisland;
  int unchanged = 0;                      // consecutive steps that kept the island's active set
  // gradient floor of a converged island (this solver's own test, not MuJoCo's exit: 100 eps of
  // the gradient scaled by 1 / (meaninertia nv) with meaninertia the mean of this step's diag(M),
  // as tuned in round 3; the model constant stat.meaninertia (0.16, about half of it on C3 states)
  // made the floor twice as strict and cost 0.18 Newton iterations per env-sub-step for nothing
  // the per-tree bar sees)
  const T meaninertia = wsum(l < m.nv ? s.M[mblk(m, l, l)] : T(0)) / T(m.nv);
  const T gscale = T(1) / (meaninertia * T(m.nv > 1 ? m.nv : 1));
  const T gtol = T(100) * PM<T>::eps();
  int it = 0;
  const int nent = s.isl_eoff[s.nisland];
  const bool jt = s.jt_ok;
  // group-parallel island factorisation when every island fits a 9-lane group
  const bool gch = s.nisland <= GCH_GROUPS && !__ballot(l < s.nisland && s.isl_n[l] > GCH_N);
  const int nisl = s.nisland;
  int nref = 0;   // refinement steps (not Newton iterations: solver_iter does not count them)
  for (; it < m.iterations; it++) {
    clk.sub_start();
    // every live island kept its active set over its last step and holds its Hessian factor: one
    // step of mixed-precision iterative refinement (newton_refine_grad) instead of another Newton
    // iteration
    if constexpr (sizeof(T) == 4) {
      if (jt && nref < 4 && !__ballot(l < nisl && !done && (unchanged < 1 || !s.isl_hvalid[l]))) {
        nref++;
        newton_refine_grad(s);
        clk.sub_lap(SC_N_GRAD);
        island_sums(s, s.v2, (const T*)nullptr, s.isl_val);
        if (!done && PM<T>::sqrt_(s.isl_val[l]) * gscale < gtol) done = true;
        if (l < PH_MAXT) s.isl_flag[l] = done;
        wsync();
        clk.sub_lap(SC_N_CONV);
        clk.lap(9);
        if (!__ballot(!done)) break;
        if (gch) {
          newton_dir_groups(s, done);
        } else {   // (every live island holds its factor: <= 9 dofs, the register path)
          const int n = !done ? s.isl_n[l] : 0;
          if (!done) island_newton_dir_reg<T, 9>(s, l, n);
          wsync();
        }
        clk.lap(10);
        newton_refine_update(s);
        bool anych = false;
        if (!done) {
          if (s.isl_val[l] != T(0)) {
            unchanged = 0;
            s.isl_hvalid[l] = 0;
            anych = true;
          } else {
            done = true;
          }
        }
        wsync();
        if (__ballot(anych)) {   // a changed island goes on with Newton iterations: its cost
          eval_cost(m, s, s.x, true, s.isl_cost);
          if (anych) cost = s.isl_cost[l];
        }
        clk.lap(11);
        if (!__ballot(!done)) break;
        it--;   // (a refinement is not a Newton iteration)
        continue;
      }
    }
    // gradient g = M (x - x_smooth) + J^T (D jar) over the dof's island rows
    if (l < m.nv) s.v1[l] = s.x[l] - s.qacc_smooth[l];
    if (jt)
      for (int rr = l; rr < s.nefc; rr += NT) {
        const int r = s.isl_row[rr];
        const bool a = s.efc_act[r];
        const T d = s.efc_D[r];
        s.rr_f[rr] = a ? d * s.efc_jar[r] : T(0);
        s.rr_d[rr] = a ? d : T(0);
      }
    wsync();
    // islands with many rows (closed fingers: 200-400 rows on the arm island): J^T (D jar) on the
    // whole wave -- lane (dof a, slice k) sums rows a + ... k, k + S, k + 2S .. (S = 64 / n
    // slices), then lane a adds its S partials -- instead of one lane per dof walking every row;
    // the sums land in v2 (dead here) for the dof lanes below
    const uint32_t bigg = PNP_BIG_ISLANDS && jt ? (uint32_t)__ballot(l < nisl && s.isl_roff[l + 1] - s.isl_roff[l] > NT &&
                                                                     s.isl_n[l] <= 32)
                                                : 0u;
    for (uint32_t bm = bigg; bm; bm &= bm - 1) {
      const int I = __builtin_ctz(bm);
      const int n = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0, S = NT / n;
      const int a = l % n, k0 = l / n;
      if (k0 < S) {
        const T* col = s.jt + s.isl_joff[I] + a;
        const T* fr = s.rr_f + r0;
        T part = 0;
        for (int k = k0; k < nr; k += S) part += col[k * n] * fr[k];
        s.ntmp[l] = part;
      }
      wsync();
      if (l < n) {
        T g = 0;
        for (int k = 0; k < S; k++) g += s.ntmp[l + k * n];
        s.v2[s.isl_dof[I][l]] = g;
      }
      wsync();
    }
    if (l < m.nv) {
      const int t = s.c_dof_tree[l], I = s.tree_island[t];
      const T mv = mulM_row(m, s, l, s.v1);
      const T g = (bigg >> I & 1u) ? mv + s.v2[l]
                : jt ? jt_dof_sum(s, I, s.dof_ipos[l], mv, s.rr_f)
                     : dof_row_sum(mv, s, I, t, l - s.c_tree_dofadr[t], s.efc_D, s.efc_jar, true);
      s.grad[l] = g;
      s.v2[l] = g * g;
    }
    wsync();
    clk.sub_lap(SC_N_GRAD);
    // an island whose last step kept its active set is at that quadratic's minimiser up to the
    // rounding of one Cholesky solve (cond(H) eps): done once its gradient is at the floor,
    // otherwise it takes one more (refining) Newton step
    island_sums(s, s.v2, (const T*)nullptr, s.isl_val);
    if (!done && unchanged >= 1 && PM<T>::sqrt_(s.isl_val[l]) * gscale < gtol) done = true;
    if (l < PH_MAXT) s.isl_flag[l] = done;
    wsync();
    clk.sub_lap(SC_N_CONV);
    if (!__ballot(!done)) { clk.lap(9); break; }
    // Hessian island blocks (lower triangle, lane per entry): M + sum_active D J J^T; blocks of
    // islands whose active set is unchanged since their last assembly are reused as they are;
    // fp32 islands with many rows on the matrix cores (hess_mfma)
    uint32_t bigh = 0;
    if constexpr (sizeof(T) == 4 && PNP_BIG_ISLANDS) {
      if (jt)
        bigh = (uint32_t)__ballot(l < nisl && !s.isl_flag[l] && !s.isl_hvalid[l] &&
                                  s.isl_roff[l + 1] - s.isl_roff[l] > NT && s.isl_n[l] <= 16);
      for (uint32_t bm = bigh; bm; bm &= bm - 1) hess_mfma(s, __builtin_ctz(bm));
    }
    for (int e = l; e < nent; e += NT) {
      // the entry's island: comparisons against the offsets (independent LDS loads issued
      // together) instead of a loop that waits on one load per island
      int I = 0;
#pragma unroll
      for (int J = 1; J <= PH_MAXT; J++) I += J < nisl && e >= s.isl_eoff[J] ? 1 : 0;
      const int eI = s.isl_eoff[I], nI = s.isl_n[I], r0I = s.isl_roff[I], e1I = s.isl_roff[I + 1],
                joI = s.isl_joff[I];
      if (s.isl_flag[I] || s.isl_hvalid[I] || (bigh >> I & 1u)) continue;
      const int le = e - eI;
      int a = (int)((PM<float>::sqrt_(8.0f * le + 1.0f) - 1.0f) * 0.5f);
      while (a * (a + 1) / 2 > le) a--;
      while ((a + 1) * (a + 2) / 2 <= le) a++;
      const int b = le - a * (a + 1) / 2;
      const int i = s.isl_dof[I][a], j = s.isl_dof[I][b];
      const int ti = s.c_dof_tree[i], tj = s.c_dof_tree[j];
      T h = ti == tj ? s.M[mblk(m, i, j)] : T(0);
      const int li = i - s.c_tree_dofadr[ti], lj = j - s.c_tree_dofadr[tj];
      const int e1 = e1I;
      if (jt) {
        const int n = nI, r0 = r0I;
        const T* ja = s.jt + joI + a;
        const T* jb = s.jt + joI + b;
        const T* dr = s.rr_d + r0;
#pragma unroll 4
        for (int k = 0; k < e1 - r0; k++) h += ja[k * n] * dr[k] * jb[k * n];
      } else
#pragma unroll 2
      for (int rr = r0I; rr < e1; rr++) {   // unconditional loads (see own_slot)
        const int r = s.isl_row[rr];
        const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], off = s.efc_off[r];
        const int n0 = s.c_tree_dofnum[t0];
        const int ki = t0 == ti ? li : (t1 == ti ? n0 + li : -1);
        const int kj = t0 == tj ? lj : (t1 == tj ? n0 + lj : -1);
        const T c = s.efc_Jv[off + (ki >= 0 ? ki : 0)] * s.efc_D[r] * s.efc_Jv[off + (kj >= 0 ? kj : 0)];
        h = ki >= 0 && kj >= 0 && s.efc_act[r] ? h + c : h;
      }
      s.Hp[e] = h;   // = HI(I, a, b)
    }
    wsync();
    clk.sub_lap(SC_N_HESS);
    clk.lap(9);
    // Newton direction per island (lane per island); the register path leaves H intact, the
    // in-place LDS path (merged islands > 9 dofs) consumes it
    if (gch) {
      newton_dir_groups(s, done);
    } else {
      // one unrolled register variant (islands of <= 9 dofs padded with identity): lanes holding
      // 6- and 9-dof islands run the same code instead of two divergent copies; larger (merged)
      // islands one after the other on the whole wave
      const int n = !done ? s.isl_n[l] : 0;
      if (!done && n <= 9) island_newton_dir_reg<T, 9>(s, l, n);
      if (!done) s.isl_hvalid[l] = n <= 9;
      wsync();
      for (uint32_t bm = (uint32_t)__ballot(n > 9); bm; bm &= bm - 1) {
        const int I = __builtin_ctz(bm), nI = s.isl_n[I];
        island_newton_dir_wave<T, PH_MAXV>(s, I, nI);
      }
    }
    wsync();
    clk.lap(10);
    clk.aux_start();
    line_search_islands(m, s, clk);
    clk.lap(11);
    if (l < m.nv) s.x[l] += s.isl_alpha[s.tree_island[s.c_dof_tree[l]]] * s.p[l];
    // remember the active set the step was computed with
    for (int r = l; r < s.nefc; r += NT) s.efc_Jp[r] = (T)s.efc_act[r];
    wsync();
    eval_cost(m, s, s.x, true, s.isl_cost);
    // active-set change per island (rows of island I on DPP row I & 3)
    {
      const int q = l & 7, I = l >> 3;
      bool ch = false;
      if (I < s.nisland)
        for (int rr = s.isl_roff[I] + q; rr < s.isl_roff[I + 1]; rr += 8) {
          const int r = s.isl_row[rr];
          ch |= (T)s.efc_act[r] != s.efc_Jp[r];
        }
      const bool any = ((__ballot(ch) >> (l & 56)) & 0xFFull) != 0;
      if (I < s.nisland && q == 0) s.isl_val[I] = any ? T(1) : T(0);
    }
    wsync();
    // island converged: two consecutive steps kept its active set (then its piecewise quadratic
    // is a single quadratic there and x its minimiser, refined once), or its cost stopped
    // decreasing
    if (!done) {
      const bool changed = s.isl_val[l] != T(0);
      const T nc = s.isl_cost[l];
      const T impr = cost - nc;
      unchanged = changed ? 0 : unchanged + 1;
      if (changed) s.isl_hvalid[l] = 0;
      if (unchanged >= 2 || !(impr > 0) || !(s.isl_alpha[l] > T(0))) done = true;
      cost = nc;
    }
    wsync();
    clk.lap(12);
    if (!__ballot(!done)) { it++; break; }
  }
  clk.lap(12);
  if (l == 0) s.solver_iter = it;
  for (int r = l; r < s.nefc; r += NT) s.efc_force[r] = s.efc_act[r] ? -s.efc_D[r] * s.efc_jar[r] : T(0);
  if (l < m.nv) s.qacc[l] = s.x[l];
  wsync();
}

template <typename T, class CLK>
__device__ void st_newton(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if constexpr (sizeof(T) == 4) {
    st_newton_islands(m, s, clk);
    return;
  }
  if (s.nefc == 0) {
    if (l < m.nv) s.qacc[l] = s.qacc_smooth[l];
    if (l == 0) s.solver_iter = 0;
    wsync();
    return;
  }
  clk.aux_start();
  build_islands(m, s, clk);
  if (PNP_HANDS && s.ovf) return;
  // warm start (mj_fwdConstraint): qacc_warmstart unless its cost exceeds qacc_smooth's, for the
  // whole problem.  One pass: cost(qacc_smooth) has no dof term and its jar is efc_bb (= J
  // qacc_smooth - aref, same arithmetic), and the chosen start's jar / active set are kept instead
  // of re-evaluated.  The costs are kept per island (island I's dofs and rows; they sum to the
  // problem's cost): the improvement test below sums per-island differences, so a small island's
  // progress does not cancel against the arm's cost in fp32.
  if (l < m.nv) s.v1[l] = s.qacc_ws[l] - s.qacc_smooth[l];
  wsync();
  if (l < m.nv) s.v2[l] = T(0.5) * s.v1[l] * mulM_row(m, s, l, s.v1);
  for (int r = l; r < s.nefc; r += NT) {
    const T v = row_dot(s, r, s.qacc_ws, -s.efc_aref[r]);
    const T bs = s.efc_bb[r];
    s.efc_jar[r] = v;
    s.ntmp[r] = r < s.ne || v < 0 ? T(0.5) * s.efc_D[r] * v * v : T(0);
    s.efc_Jp[r] = r < s.ne || bs < 0 ? T(0.5) * s.efc_D[r] * bs * bs : T(0);
  }
  wsync();
  island_sums2(s, s.v2, s.ntmp, s.isl_val, s.efc_Jp, s.isl_cost);
  const int nisl = s.nisland;
  const bool ws = !(wsum(l < nisl ? s.isl_val[l] : T(0)) > wsum(l < nisl ? s.isl_cost[l] : T(0)));
  if (l < PH_MAXT) {
    if (ws && l < nisl) s.isl_cost[l] = s.isl_val[l];
    s.isl_flag[l] = 0;
    s.isl_hvalid[l] = 0;
  }
  wsync();
  if (l < m.nv) s.x[l] = ws ? s.qacc_ws[l] : s.qacc_smooth[l];
  for (int r = l; r < s.nefc; r += NT) {
    const T v = ws ? s.efc_jar[r] : s.efc_bb[r];
    s.efc_jar[r] = v;
    s.efc_act[r] = r < s.ne || v < 0;
  }
  wsync();
  clk.lap(8);
  // MuJoCo 2.3.3 mj_solNewton's iteration and exits (oracle/physics.c solve_newton): direction
  // -H^-1 g per island (H is block-diagonal over islands, so this is the problem's Newton
  // direction), one line search for the whole problem, stop at a zero step, then after each step
  // once scale (cost_old - cost) < tolerance or scale |g| < tolerance (scale = 1 / (meaninertia
  // nv), the model statistic), or after `iterations` steps.  (fp64 only: st_newton_islands above.)
  T cost = l < nisl ? s.isl_cost[l] : T(0);   // lane I: island I's cost
  const bool idle = l >= nisl;                 // lane I: no island I
  const T scale = T(1) / (m.meaninertia * T(m.nv > 1 ? m.nv : 1));
  T improvement = 0;
  int it = 0;
  const int nent = s.isl_eoff[s.nisland];
  const bool jt = s.jt_ok;
  // group-parallel island factorisation when every island fits a 9-lane group
  const bool gch = s.nisland <= GCH_GROUPS && !__ballot(l < s.nisland && s.isl_n[l] > GCH_N);
  for (;;) {
    clk.sub_start();
    // gradient g = M (x - x_smooth) + J^T (D jar) over the dof's island rows
    if (l < m.nv) s.v1[l] = s.x[l] - s.qacc_smooth[l];
    if (jt)
      for (int rr = l; rr < s.nefc; rr += NT) {
        const int r = s.isl_row[rr];
        const bool a = s.efc_act[r];
        const T d = s.efc_D[r];
        s.rr_f[rr] = a ? d * s.efc_jar[r] : T(0);
        s.rr_d[rr] = a ? d : T(0);
      }
    wsync();
    // islands with many rows (closed fingers: 200-400 rows on the arm island): J^T (D jar) on the
    // whole wave -- lane (dof a, slice k) sums rows a + ... k, k + S, k + 2S .. (S = 64 / n
    // slices), then lane a adds its S partials -- instead of one lane per dof walking every row;
    // the sums land in v2 (dead here) for the dof lanes below
    const uint32_t bigg = PNP_BIG_ISLANDS && jt ? (uint32_t)__ballot(l < nisl && s.isl_roff[l + 1] - s.isl_roff[l] > NT &&
                                                                     s.isl_n[l] <= 32)
                                                : 0u;
    for (uint32_t bm = bigg; bm; bm &= bm - 1) {
      const int I = __builtin_ctz(bm);
      const int n = s.isl_n[I], r0 = s.isl_roff[I], nr = s.isl_roff[I + 1] - r0, S = NT / n;
      const int a = l % n, k0 = l / n;
      if (k0 < S) {
        const T* col = s.jt + s.isl_joff[I] + a;
        const T* fr = s.rr_f + r0;
        T part = 0;
        for (int k = k0; k < nr; k += S) part += col[k * n] * fr[k];
        s.ntmp[l] = part;
      }
      wsync();
      if (l < n) {
        T g = 0;
        for (int k = 0; k < S; k++) g += s.ntmp[l + k * n];
        s.v2[s.isl_dof[I][l]] = g;
      }
      wsync();
    }
    T g2 = 0;
    if (l < m.nv) {
      const int t = s.c_dof_tree[l], I = s.tree_island[t];
      const T mv = mulM_row(m, s, l, s.v1);
      const T g = (bigg >> I & 1u) ? mv + s.v2[l]
                : jt ? jt_dof_sum(s, I, s.dof_ipos[l], mv, s.rr_f)
                     : dof_row_sum(mv, s, I, t, l - s.c_tree_dofadr[t], s.efc_D, s.efc_jar, true);
      s.grad[l] = g;
      g2 = g * g;
    }
    wsync();
    clk.sub_lap(SC_N_GRAD);
    if (it > 0) {
      const T gradient = scale * PM<T>::sqrt_(wsum(g2));
      if (improvement < m.tolerance || gradient < m.tolerance) { clk.sub_lap(SC_N_CONV); clk.lap(9); break; }
    }
    clk.sub_lap(SC_N_CONV);
    if (it >= m.iterations) { clk.lap(9); break; }
    // Hessian island blocks (lower triangle, lane per entry): M + sum_active D J J^T; blocks of
    // islands whose active set is unchanged since their last assembly are reused as they are;
    // fp32 islands with many rows on the matrix cores (hess_mfma)
    uint32_t bigh = 0;
    if constexpr (sizeof(T) == 4 && PNP_BIG_ISLANDS) {
      if (jt)
        bigh = (uint32_t)__ballot(l < nisl && !s.isl_hvalid[l] && s.isl_roff[l + 1] - s.isl_roff[l] > NT &&
                                  s.isl_n[l] <= 16);
      for (uint32_t bm = bigh; bm; bm &= bm - 1) hess_mfma(s, __builtin_ctz(bm));
    }
    for (int e = l; e < nent; e += NT) {
      // the entry's island: comparisons against the offsets (independent LDS loads issued
      // together) instead of a loop that waits on one load per island
      int I = 0;
#pragma unroll
      for (int J = 1; J <= PH_MAXT; J++) I += J < nisl && e >= s.isl_eoff[J] ? 1 : 0;
      const int eI = s.isl_eoff[I], nI = s.isl_n[I], r0I = s.isl_roff[I], e1I = s.isl_roff[I + 1],
                joI = s.isl_joff[I];
      if (s.isl_hvalid[I] || (bigh >> I & 1u)) continue;
      const int le = e - eI;
      int a = (int)((PM<float>::sqrt_(8.0f * le + 1.0f) - 1.0f) * 0.5f);
      while (a * (a + 1) / 2 > le) a--;
      while ((a + 1) * (a + 2) / 2 <= le) a++;
      const int b = le - a * (a + 1) / 2;
      const int i = s.isl_dof[I][a], j = s.isl_dof[I][b];
      const int ti = s.c_dof_tree[i], tj = s.c_dof_tree[j];
      T h = ti == tj ? s.M[mblk(m, i, j)] : T(0);
      const int li = i - s.c_tree_dofadr[ti], lj = j - s.c_tree_dofadr[tj];
      const int e1 = e1I;
      if (jt) {
        const int n = nI, r0 = r0I;
        const T* ja = s.jt + joI + a;
        const T* jb = s.jt + joI + b;
        const T* dr = s.rr_d + r0;
#pragma unroll 4
        for (int k = 0; k < e1 - r0; k++) h += ja[k * n] * dr[k] * jb[k * n];
      } else
#pragma unroll 2
      for (int rr = r0I; rr < e1; rr++) {   // unconditional loads (see own_slot)
        const int r = s.isl_row[rr];
        const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], off = s.efc_off[r];
        const int n0 = s.c_tree_dofnum[t0];
        const int ki = t0 == ti ? li : (t1 == ti ? n0 + li : -1);
        const int kj = t0 == tj ? lj : (t1 == tj ? n0 + lj : -1);
        const T c = s.efc_Jv[off + (ki >= 0 ? ki : 0)] * s.efc_D[r] * s.efc_Jv[off + (kj >= 0 ? kj : 0)];
        h = ki >= 0 && kj >= 0 && s.efc_act[r] ? h + c : h;
      }
      s.Hp[e] = h;   // = HI(I, a, b)
    }
    wsync();
    clk.sub_lap(SC_N_HESS);
    clk.lap(9);
    // Newton direction per island (lane per island); the register path leaves H intact, the
    // in-place LDS path (merged islands > 9 dofs) consumes it
    if (gch) {
      newton_dir_groups(s, false);
    } else {
      // one unrolled register variant (islands of <= 9 dofs padded with identity): lanes holding
      // 6- and 9-dof islands run the same code instead of two divergent copies; larger (merged)
      // islands one after the other on the whole wave
      const int n = !idle ? s.isl_n[l] : 0;
      if (!idle && n <= 9) island_newton_dir_reg<T, 9>(s, l, n);
      if (!idle) s.isl_hvalid[l] = n <= 9;
      wsync();
      for (uint32_t bm = (uint32_t)__ballot(n > 9); bm; bm &= bm - 1) {
        const int I = __builtin_ctz(bm), nI = s.isl_n[I];
        island_newton_dir_wave<T, PH_MAXV>(s, I, nI);
      }
    }
    wsync();
    clk.lap(10);
    clk.aux_start();
    const T alpha = line_search(m, s, clk);
    clk.lap(11);
    if (alpha == T(0)) { clk.lap(12); break; }
    if (l < m.nv) s.x[l] += alpha * s.p[l];
    it++;
    // remember the active set the step was computed with
    for (int r = l; r < s.nefc; r += NT) s.efc_Jp[r] = (T)s.efc_act[r];
    wsync();
    eval_cost(m, s, s.x, true, s.isl_cost);
    // active-set change per island (rows of island I on DPP row I & 3)
    {
      const int q = l & 7, I = l >> 3;
      bool ch = false;
      if (I < s.nisland)
        for (int rr = s.isl_roff[I] + q; rr < s.isl_roff[I + 1]; rr += 8) {
          const int r = s.isl_row[rr];
          ch |= (T)s.efc_act[r] != s.efc_Jp[r];
        }
      const bool any = ((__ballot(ch) >> (l & 56)) & 0xFFull) != 0;
      if (I < s.nisland && q == 0) s.isl_val[I] = any ? T(1) : T(0);
    }
    wsync();
    // improvement = scale (cost_old - cost), summed over the islands' own differences
    {
      const bool changed = !idle && s.isl_val[l] != T(0);
      const T nc = !idle ? s.isl_cost[l] : T(0);
      if (changed) s.isl_hvalid[l] = 0;
      improvement = scale * wsum(cost - nc);
      cost = nc;
    }
    wsync();
    clk.lap(12);
  }
  clk.lap(12);
  if (l == 0) s.solver_iter = it;
  for (int r = l; r < s.nefc; r += NT) s.efc_force[r] = s.efc_act[r] ? -s.efc_D[r] * s.efc_jar[r] : T(0);
  if (l < m.nv) s.qacc[l] = s.x[l];
  wsync();
}

// ============================================================================ no-slip
// x = (L L^T)^-1 j for one dense tree block of compile-time size N (L row-major, N x N): the
// substitutions fully unrolled, y / x in registers -- the block's loads are independent of the
// substitution chain and issue together (a runtime-n loop kept y in private memory and waited on
// each L load in turn).  Same operations in the same order as the generic loop below.
template <int N, typename T>
__device__ __forceinline__ void tree_solve_fixed(const T* L, const T* j, T* x_out) {
  T y[N], x[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    T v = j[i];
#pragma unroll
    for (int k = 0; k < i; k++) v -= L[i * N + k] * y[k];
    y[i] = v / L[i * N + i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    T v = y[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) v -= L[k * N + i] * x[k];
    x[i] = v / L[i * N + i];
  }
#pragma unroll
  for (int i = 0; i < N; i++) x_out[i] = x[i];
}

// bd of the pair starting at contact row r (st_noslip): Jd . (qacc_smooth + b qvel) over the
// row's <= 2 trees, tree by tree (9- and 6-dof trees unrolled: independent loads issued together)
template <int N, typename T>
__device__ __forceinline__ T pair_bd_tree(const T* J0, const T* J1, const T* qs, const T* qv, T b) {
  T a = 0;
#pragma unroll
  for (int i = 0; i < N; i++) a += (J0[i] - J1[i]) * (qs[i] + b * qv[i]);
  return a;
}
template <typename T>
__device__ __forceinline__ void pair_bd(Env<T>& s, int r) {
  const int t0 = s.efc_t0[r], t1 = s.efc_t1[r];
  const T* J0 = s.efc_Jv + s.efc_off[r];
  const T* J1 = s.efc_Jv + s.efc_off[r + 1];
  const T b = s.con_b[s.efc_id[r]];
  T bd = 0;
  int base = 0;
  for (int h = 0; h < 2; h++) {
    const int t = h ? t1 : t0;
    if (t < 0) continue;
    const int n = s.c_tree_dofnum[t], d0 = s.c_tree_dofadr[t];
    if (n == 9) bd += pair_bd_tree<9>(J0 + base, J1 + base, s.qacc_smooth + d0, s.qvel + d0, b);
    else if (n == 6) bd += pair_bd_tree<6>(J0 + base, J1 + base, s.qacc_smooth + d0, s.qvel + d0, b);
    else
      for (int i = 0; i < n; i++) bd += (J0[base + i] - J1[base + i]) * (s.qacc_smooth[d0 + i] + b * s.qvel[d0 + i]);
    base += n;
  }
  s.efc_bb[r] = bd;
}

// Dense long-list sweep (st_noslip): the group's island v in registers, lane q = island dof q;
// each pair's difference rows Jd, Wd are formed at the lane's island position straight from the
// dense blocks (jt, and W in jt's layout), its K1 and 1 / K1 from the per-call table (efc_jar at
// the pair's island row positions, dead after the Newton stage), so an update is one row sum of
// Jd v, the projection and a lane-local v += Wd dl.  List entries are island row positions.
// Software pipeline: list entry 3 pairs ahead, the row's efc index 2 ahead, its
// J / W / bd / f / K1 entries 1 ahead.  Islands are independent under Gauss-Seidel: a group
// sweeps its (<= 2) islands one after the other, each in its own row order.
template <typename T>
__device__ __attribute__((noinline)) void st_noslip_dense_sweep(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s,
                                                                int iend0, int iend1) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id(), grp = l >> 4, q = l & 15;
  {   // Delassus blocks, lane per pair: A_ab = J_a . W_b over the island's dofs
    const int L0 = s.ns_len[0], L1 = s.ns_len[1], L2 = s.ns_len[2], L3 = s.ns_len[3];
    const int tot = L0 + L1 + L2 + L3;
    for (int e = l; e < tot; e += NT) {
      const int g = e < L0 ? 0 : (e < L0 + L1 ? 1 : (e < L0 + L1 + L2 ? 2 : 3));
      const int k = e - (g > 0 ? L0 : 0) - (g > 1 ? L1 : 0) - (g > 2 ? L2 : 0);
      const int p = s.ns_list[g][k];
      const int I = s.tree_island[s.efc_t0[s.isl_row[p]]], n = s.isl_n[I];
      const int o = s.isl_joff[I] + (p - s.isl_roff[I]) * n;
      const T* J = s.jt + o;
      const T* W = s.efc_Wv + o;
      T K1 = 0;   // Jd . Wd (st_noslip)
      for (int c = 0; c < n; c++) K1 += (J[c] - J[n + c]) * (W[c] - W[n + c]);
      // 1 / K1 = 0 for a flat pair (K1 < 1e-15), whose forces then stay at their mean
      s.efc_jar[p] = K1;
      s.efc_jar[p + 1] = K1 < T(1e-15) ? T(0) : T(1) / K1;
    }
  }
  wsync();
  // the group's (<= 2) islands: I = grp and grp + 4
  struct DSet {
    int k0, cnt, maxc, n, r0, jo, qq, d;
    bool lane_on;
  };
  auto mkset = [&](int si) {
    DSet z;
    const int I = grp + 4 * si;
    const bool has = I < s.nisland;
    z.k0 = si ? iend0 : 0;
    z.cnt = has ? (si ? iend1 : iend0) - z.k0 : 0;
    z.maxc = max(max(__builtin_amdgcn_readlane(z.cnt, 0), __builtin_amdgcn_readlane(z.cnt, 16)),
                 max(__builtin_amdgcn_readlane(z.cnt, 32), __builtin_amdgcn_readlane(z.cnt, 48)));
    z.n = has ? s.isl_n[I] : 0;
    z.r0 = has ? s.isl_roff[I] : 0;
    z.lane_on = q < z.n;
    z.qq = z.lane_on ? q : 0;
    z.d = z.lane_on ? s.isl_dof[I][q] : 0;
    z.jo = has ? s.isl_joff[I] - z.r0 * z.n : 0;   // (row position p, island dof c) at jo + p n + c
    return z;
  };
  const DSet S0 = mkset(0), S1 = mkset(1);
  T v0 = S0.lane_on ? s.v2[S0.d] : T(0), v1 = S1.lane_on ? s.v2[S1.d] : T(0);
  struct DRow {   // stage 2
    int p, j;
    bool act;
  };
  struct DRaw {   // stage 1
    int j;
    bool act;
    T Jd, Wd, bd, f0, f1, K1, iK1;
  };
  // one Gauss-Seidel sweep over the set's island; returns the group's improvement (MuJoCo
  // costChange summed over the pair updates; uniform in the group's 16 lanes)
  auto sweep = [&](const DSet& z, T& v) -> T {
    auto dlist = [&](int k) { return k < z.cnt ? (int)s.ns_list[grp][z.k0 + k] : -1; };
    auto drow = [&](int p) {
      DRow x;
      x.act = p >= 0;
      x.p = x.act ? p : z.r0;   // (an inactive slot reads the island's first row, masked below)
      x.j = s.isl_row[x.p];
      return x;
    };
    auto draw = [&](const DRow& x) {
      DRaw w;
      w.j = x.j;
      w.act = x.act;
      const int o = z.jo + x.p * z.n + z.qq;
      const T J0 = s.jt[o], J1 = s.jt[o + z.n], W0 = s.efc_Wv[o], W1 = s.efc_Wv[o + z.n];
      const bool on = x.act && z.lane_on;
      w.Jd = on ? J0 - J1 : T(0);
      w.Wd = on ? W0 - W1 : T(0);
      w.bd = s.efc_bb[x.j];
      w.f0 = s.efc_force[x.j];
      w.f1 = s.efc_force[x.j + 1];
      w.K1 = s.efc_jar[x.p];
      w.iK1 = s.efc_jar[x.p + 1];
      return w;
    };
    T impr = 0;
    // The pair's 2 x 2 projection on its difference row (st_noslip): r0 - r1 = Jd v + bd (one
    // row sum), y = clamp((f0 - mid) - (r0 - r1) / K1, +-mid) (= -K0 / K1), K1 and 1 / K1 from
    // the table.  An inactive slot has zero Jd and Wd, so v does not move.  The update moves the
    // forces along (1, -1) by dl, so MuJoCo's costChange 0.5 d^T A d + d^T r is
    // dl (0.5 dl K1 + (r0 - r1)), and v moves by Wd dl.
    auto update = [&](const DRaw& cur) {
      const T rd = rowsum16(cur.Jd * v) + cur.bd;
      const T f0 = cur.f0, f1 = cur.f1;
      const T mid = T(0.5) * (f0 + f1);
      T y = cur.iK1 != T(0) ? (f0 - mid) - rd * cur.iK1 : T(0);
      y = y < -mid ? -mid : (y > mid ? mid : y);
      const T n0 = mid + y, n1 = mid - y;
      const T dl = T(0.5) * ((n0 - f0) - (n1 - f1));
      impr = cur.act ? impr - dl * (T(0.5) * dl * cur.K1 + rd) : impr;
      v += cur.Wd * dl;
      if (cur.act && q == 0) { s.efc_force[cur.j] = n0; s.efc_force[cur.j + 1] = n1; }
    };
    // unrolled by two with the stage registers alternating (ra / rb), so that the loop carries
    // no register moves and no wait on the loads it has just issued
    DRaw ra = draw(drow(dlist(0)));
    DRow x1 = drow(dlist(1));
    int p2 = dlist(2);
    for (int k = 0; k < z.maxc; k += 2) {
      const int p3 = dlist(k + 3);
      const DRow x2 = drow(p2);
      const DRaw rb = draw(x1);
      update(ra);
      if (k + 1 >= z.maxc) break;
      const int p4 = dlist(k + 4);
      const DRow x3 = drow(p3);
      ra = draw(x2);
      update(rb);
      x1 = x3;
      p2 = p4;
    }
    wsync();   // the next sweep reads the forces this one wrote
    return impr;
  };
  // mj_solNoSlip's loop: a sweep over every island, then stop once the problem's scaled
  // improvement is below noslip_tolerance (islands are independent under Gauss-Seidel, so one
  // sweep of each in turn is one sweep of the problem)
  const T scale = T(1) / (m.meaninertia * T(m.nv > 1 ? m.nv : 1));
  int iter = 0;
  while (iter < m.noslip_iterations) {
    T impr = 0;
    if (S0.maxc) impr += sweep(S0, v0);
    if (S1.maxc) impr += sweep(S1, v1);
    impr = (rdlane(impr, 0) + rdlane(impr, 16)) + (rdlane(impr, 32) + rdlane(impr, 48));
    iter++;
    if (impr * scale < m.noslip_tolerance) break;
  }
  if (S0.lane_on) s.v2[S0.d] = v0;
  if (S1.lane_on) s.v2[S1.d] = v1;
  if (l == 0) s.noslip_iter = iter;
  wsync();
}

template <typename T, class CLK>
__device__ void st_noslip(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l == 0) s.noslip_iter = 0;
  if (m.noslip_iterations <= 0 || s.nefc == 0) return;
  clk.sub_start();
  // mj_solNoSlip's exit: after each sweep, stop once the sweep's improvement (MuJoCo costChange
  // summed over the pair updates) scaled by 1 / (meaninertia nv) is below noslip_tolerance.  Every
  // path below reduces its per-group improvement (uniform in the group's 16 lanes) over the four
  // groups after a sweep.  costChange's restore of a pair whose cost rose by more than 1e-10 is not
  // applied: the projection is the exact minimiser of the pair's 2 x 2 problem over an interval
  // that holds the old forces, so the change is <= 0 but for rounding (oracle: applied).
  const T ns_scale = T(1) / (m.meaninertia * T(m.nv > 1 ? m.nv : 1));
  auto ns_total = [](T g) { return (rdlane(g, 0) + rdlane(g, 16)) + (rdlane(g, 32) + rdlane(g, 48)); };
  constexpr int NSR = 8;   // short lists (see the force-space path below)
  // Pair lists: islands are independent under Gauss-Seidel (block-diagonal M, rows inside one
  // island), so island I runs on DPP row (I mod 4) — 16 lanes, one slot per lane — in its own
  // row order, and up to 4 pairs are updated at once; each island sees exactly the sequential
  // order, so the result equals the one-pair-at-a-time sweep.
  const int grp = l >> 4, q = l & 15;
  // end of the group's first / second island in its list (group-uniform; two scalars, not an
  // array: a runtime index would put it in scratch)
  int iend0 = 0, iend1 = 0;
  {
    int len = 0, si = 0;
    for (int I = grp; I < s.nisland; I += 4, si++) {
      for (int base = s.isl_roff[I]; base < s.isl_roff[I + 1]; base += 16) {
        const int rr = base + q;
        bool start = false;
        int r = 0;
        if (rr < s.isl_roff[I + 1]) {
          r = s.isl_row[rr];
          start = s.efc_type[r] == 6 && ((r - s.con_rbase[s.efc_id[r]]) & 1) == 0;
        }
        const uint32_t bits = (uint32_t)(__ballot(start) >> (16 * grp)) & 0xFFFFu;
        if (start) s.ns_list[grp][len + __popc(bits & ((1u << q) - 1u))] = (short)r;
        len += __popc(bits);
      }
      if (si == 0) iend0 = len;
      else iend1 = len;
    }
    if (q == 0) s.ns_len[grp] = len;
  }
  // Every path below updates a pair (rows j, j + 1 = J_n +- mu J_t of one contact) through its
  // difference row Jd = J_j - J_j+1 (= 2 mu J_t) and Wd = W_j - W_j+1 = M^-1 Jd^T: with r = J v + b
  // and A = J W (symmetric), MuJoCo's K1 = a00 + a11 - a01 - a10 is Jd . Wd and its
  // K0 = mid (a00 - a11) + bc0 - bc1 is (r0 - r1) + K1 (mid - f0) -- the same projection, without
  // forming K1 and K0 as differences of Delassus entries: between two bodies of one tree (closed
  // fingers pressed together) J_t is small against J_n, K1 ~ 1e-6 beside entries ~20, and the
  // differences of fp32 entries are rounding (the fp32 kernel then left pairs at their mean
  // that MuJoCo saturates: fingers 0.07 m/s^2 off).  r0 - r1 = Jd . v + (b0 - b1), and b0 - b1 =
  // Jd . qacc_smooth - (aref0 - aref1) with aref0 - aref1 = -b Jd . qvel (the two rows share the
  // contact's position term): bd = Jd . (qacc_smooth + b qvel), replacing efc_bb[j] (dead after
  // Newton) for the sweeps -- formed by the pair's first row in the W loops below (pair_bd).
  wsync();
  const int maxlen = max(max(s.ns_len[0], s.ns_len[1]), max(s.ns_len[2], s.ns_len[3]));
  bool small = true;
  for (int I = grp; I < s.nisland; I += 4) small = small && s.isl_n[I] <= 16;
  // Dense long lists: a group with more than NSR pairs (closed fingers pressed together put
  // 50-150 pairs on the arm island) on islands of <= 16 dofs, with the dense island Jacobian
  // blocks (jt): W is built in jt's layout and each pair's 2 x 2 Delassus block once per call
  // (st_noslip_dense_sweep).  Every tier takes this path under the same conditions (jt_ok
  // holds below the wide tier, which hands over otherwise).
  const bool dense = s.jt_ok && maxlen > NSR && !__ballot(!small);
  if (dense) {
    // the list entries become island row positions (jt / W row index); efc_Jp is free here
    for (int rr = l; rr < s.nefc; rr += NT) s.efc_Jp[s.isl_row[rr]] = T(rr);
    wsync();
#pragma unroll
    for (int g = 0; g < 4; g++)
      for (int k = l; k < s.ns_len[g]; k += NT) s.ns_list[g][k] = (short)(int)s.efc_Jp[s.ns_list[g][k]];
    // W_r = M^-1 J_r^T for contact rows, dense: the row's island block row, zero off its trees
    for (int rr = l; rr < s.nefc; rr += NT) {
      const int r = s.isl_row[rr];
      if (s.efc_type[r] != 6) continue;
      if (((r - s.con_rbase[s.efc_id[r]]) & 1) == 0) pair_bd(s, r);
      const int t0 = s.efc_t0[r], t1 = s.efc_t1[r];
      const int I = s.tree_island[t0], n = s.isl_n[I];
      T* row = s.efc_Wv + s.isl_joff[I] + (rr - s.isl_roff[I]) * n;
      for (int c = 0; c < n; c++) row[c] = T(0);
      int base = 0;
      for (int h = 0; h < 2; h++) {
        const int t = h ? t1 : t0;
        if (t < 0) continue;
        const int nt = s.c_tree_dofnum[t], o = s.c_tree_moff[t];
        const T* Jr = s.efc_Jv + s.efc_off[r] + base;
        T* Wr = row + s.tree_ipos[t];   // the tree's dofs are contiguous in island order
        if (nt == 9) tree_solve_fixed<9>(s.L + o, Jr, Wr);
        else if (nt == 6) tree_solve_fixed<6>(s.L + o, Jr, Wr);
        else {
          for (int i = 0; i < nt; i++) {   // forward substitution into Wr (no private array)
            T v = Jr[i];
            for (int k = 0; k < i; k++) v -= s.L[o + i * nt + k] * Wr[k];
            Wr[i] = v / s.L[o + i * nt + i];
          }
          for (int i = nt - 1; i >= 0; i--) {
            T v = Wr[i];
            for (int k = i + 1; k < nt; k++) v -= s.L[o + k * nt + i] * Wr[k];
            Wr[i] = v / s.L[o + i * nt + i];
          }
        }
        base += nt;
      }
    }
  } else {
    {   // zero the 8 slots past the last row: the tail of the force-space setup's unmasked reads
      const int rl = s.nefc - 1;
      const int end = s.efc_off[rl] + row_width(m, s.efc_t0[rl], s.efc_t1[rl]);
      if (l < 8) s.efc_Wv[end + l] = T(0);
    }
    // W_r = M^-1 J_r^T for contact rows (block-diagonal M: solve per tree of the row)
    for (int r = l; r < s.nefc; r += NT) {
      if (s.efc_type[r] != 6) continue;
      if (((r - s.con_rbase[s.efc_id[r]]) & 1) == 0) pair_bd(s, r);
      const int t0 = s.efc_t0[r], t1 = s.efc_t1[r];
      int base = 0;
      for (int h = 0; h < 2; h++) {
        const int t = h ? t1 : t0;
        if (t < 0) continue;
        const int n = s.c_tree_dofnum[t], o = s.c_tree_moff[t];
        if (n == 9 || n == 6) {
          const T* Jr = s.efc_Jv + s.efc_off[r] + base;
          T* Wr = s.efc_Wv + s.efc_off[r] + base;
          if (n == 9) tree_solve_fixed<9>(s.L + o, Jr, Wr);
          else tree_solve_fixed<6>(s.L + o, Jr, Wr);
          base += n;
          continue;
        }
        for (int i = 0; i < n; i++) {   // forward substitution into the W row (no private array)
          T v = EJ(r, base + i);
          for (int k = 0; k < i; k++) v -= s.L[o + i * n + k] * EW(r, base + k);
          EW(r, base + i) = v / s.L[o + i * n + i];
        }
        for (int i = n - 1; i >= 0; i--) {
          T v = EW(r, base + i);
          for (int k = i + 1; k < n; k++) v -= s.L[o + k * n + i] * EW(r, base + k);
          EW(r, base + i) = v / s.L[o + i * n + i];
        }
        base += n;
      }
    }
  }
  clk.sub_lap(SC_NS_W);
  if constexpr (sizeof(T) == 4 && PNP_F32_NS_NEWTON) {
    // fp32: the constraint acceleration v = qacc - qacc_smooth from Newton's own iterate, not
    // M^-1 J^T f recomputed from the forces: where large contact forces cancel on a dof (the pads
    // pressed together push both fingers with ~100x the net force) the fp32 sum J^T f carries
    // their rounding (the fingers' generalized forces 1.4e-3 N off on the `pads` fixture,
    // tools/pads_stage_diag.py), while Newton's iterate is accurate to ~2e-7.  The Newton forces
    // are kept in efc_aref (dead after Newton) for st_finish_accel, which adds only the no-slip
    // sweeps' force changes.  (fp64 keeps MuJoCo's recomputation, the oracle's to 1e-9.)
    for (int r = l; r < s.nefc; r += NT) s.efc_aref[r] = s.efc_force[r];
    if (l < m.nv) s.v2[l] = s.qacc[l] - s.qacc_smooth[l];
    wsync();
  } else {
    // v = M^-1 J^T f over the dof's island rows
    const bool jt = s.jt_ok;
    if (jt) {
      gather_rows(s, s.efc_force, s.rr_g);
      wsync();
    }
    if (l < m.nv) {
      const int t = s.c_dof_tree[l], I = s.tree_island[t];
      const T g = jt ? jt_dof_sum(s, I, s.dof_ipos[l], T(0), s.rr_g)
                     : dof_row_sum(T(0), s, I, t, l - s.c_tree_dofadr[t], s.efc_force, (const T*)nullptr, false);
      s.v2[l] = g;
    }
    wsync();
    solve_M(m, s, s.v2, s.v2);
  }
  const int glen = s.ns_len[grp];
  clk.sub_lap(SC_NS_LISTS);
  clk.count(SN_NS_SWEEP, maxlen);
  clk.count(SN_NS_DENSE, dense ? 1 : 0);
  if (dense) {
    st_noslip_dense_sweep(m, s, iend0, iend1);
    return;
  }
  // One pair of opposing pyramid edges per group and step; sparse rows have <= 16 slots = one
  // DPP row.  A pair's J, W, b and slot dofs are read-only here, so the next pair's are loaded
  // while the current one is updated; only v2 and the forces (written by the previous update)
  // are read after the hand-off.
  struct NsPair {
    int j, d;
    bool act, on;
    T Jd, Wd, bd;   // the pair's difference row (see above)
  };
  auto fetch = [&](int k) {
    NsPair p;
    p.act = k < glen;
    p.j = p.act ? s.ns_list[grp][k] : 0;
    const int t0 = s.efc_t0[p.j], t1 = s.efc_t1[p.j], w = row_width(m, t0, t1);
    p.on = p.act && q < w;
    const int qq = p.on ? q : 0;                 // unconditional, in-range loads; masked below
    const int o0 = s.efc_off[p.j], o1 = s.efc_off[p.j + 1];
    p.d = p.on ? slot_dof(m, t0, t1, qq) : 0;
    const T J0 = s.efc_Jv[o0 + qq], J1 = s.efc_Jv[o1 + qq];
    const T W0 = s.efc_Wv[o0 + qq], W1 = s.efc_Wv[o1 + qq];
    p.Jd = p.on ? J0 - J1 : T(0);
    p.Wd = p.on ? W0 - W1 : T(0);
    p.bd = s.efc_bb[p.j];
    return p;
  };
  // Short sweeps (every group's list <= NSR pairs, the common case: an island of a box resting on
  // a board has 8) keep the whole sweep in registers.
  // Force space (the common case: every group's pairs act on the same trees, so their packed
  // slots address the same dofs): lane q of a group owns pair q of the group's list and keeps its
  // difference residual rd_q = Jd_q v + bd_q and its row of the difference Delassus block
  // Ad_qj = Jd_q . Wd_j (j over the group's pairs; Ad_qq = K1_q) in registers.  A pair update
  // reads its residual and K1 by DPP row broadcasts, projects as below, and adds Ad(:, pair) dl to
  // every lane's residual -- rd = Jd (v0 + Wd dl) + bd without the v round trip through LDS and
  // the row sum per update.  Same projection; residuals differ from the v-space sweep by rounding.
  {
    bool uni = true;
    int jr = 0, o0 = 0, o1 = 0, w = 0;
    const bool mine = q < glen && q < NSR;
    if (mine) {
      jr = s.ns_list[grp][q];
      const int j0 = s.ns_list[grp][0];
      uni = s.efc_t0[jr] == s.efc_t0[j0] && s.efc_t1[jr] == s.efc_t1[j0];
      o0 = s.efc_off[jr];
      o1 = s.efc_off[jr + 1];
      w = row_width(m, s.efc_t0[jr], s.efc_t1[jr]);
    }
    if (maxlen <= NSR && !__ballot(!uni)) {
      T rd = 0, Ad[NSR];
      if (!__ballot(mine && w > 8)) {
        // rows of <= 8 slots (a free body against the world): fully unrolled, every load of a
        // row issued back to back
        const int t0 = s.efc_t0[jr], t1 = s.efc_t1[jr];
        const int n0 = s.c_tree_dofnum[t0], d0 = s.c_tree_dofadr[t0];
        const int d1 = t1 >= 0 ? s.c_tree_dofadr[t1] - n0 : 0;
        // 8 slots read per row with no masking of the loads: Jd is zero past the row's width and
        // the W slots past a contact row are the next contact row's or the zeroed tail
        T Jd[8];
        rd = mine ? s.efc_bb[jr] : T(0);
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const T jd = s.efc_Jv[o0 + k] - s.efc_Jv[o1 + k];
          const T vd = s.v2[k < n0 ? d0 + k : (d1 + k < PH_MAXV ? d1 + k : 0)];
          Jd[k] = mine && k < w ? jd : T(0);
          rd += Jd[k] * vd;
        }
#pragma unroll
        for (int j = 0; j < NSR; j++) {
          const int jj = s.ns_list[grp][j < glen ? j : 0];
          const T* W0 = s.efc_Wv + s.efc_off[jj];
          const T* W1 = s.efc_Wv + s.efc_off[jj + 1];
          T a = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) a += Jd[k] * (W0[k] - W1[k]);
          Ad[j] = j < glen ? a : T(0);
        }
      } else {
        if (mine) {
          const int t0 = s.efc_t0[jr], t1 = s.efc_t1[jr];
          rd = s.efc_bb[jr];
          for (int k = 0; k < w; k++) rd += (s.efc_Jv[o0 + k] - s.efc_Jv[o1 + k]) * s.v2[slot_dof(m, t0, t1, k)];
        }
#pragma unroll
        for (int j = 0; j < NSR; j++) {
          T a = 0;
          if (mine && j < glen) {
            const int jj = s.ns_list[grp][j];
            const int p0 = s.efc_off[jj], p1 = s.efc_off[jj + 1];
            for (int k = 0; k < w; k++)
              a += (s.efc_Jv[o0 + k] - s.efc_Jv[o1 + k]) * (s.efc_Wv[p0 + k] - s.efc_Wv[p1 + k]);
          }
          Ad[j] = a;
        }
      }
      // per pair: K1 (its own Ad diagonal) and 1 / K1 (0 for a flat pair: forces stay at their mean)
      T F0[NSR], F1[NSR], KK[NSR], IK[NSR];
#pragma unroll
      for (int k = 0; k < NSR; k++) {
        const int jk = k < glen ? s.ns_list[grp][k] : 0;
        F0[k] = s.efc_force[jk];
        F1[k] = s.efc_force[jk + 1];
      }
#define NS_BC(K)                                  \
      {                                           \
        const T k1 = rowbcast<K>(Ad[K]);          \
        KK[K] = k1;                               \
        IK[K] = k1 < T(1e-15) ? T(0) : T(1) / k1; \
      }
      NS_BC(0) NS_BC(1) NS_BC(2) NS_BC(3) NS_BC(4) NS_BC(5) NS_BC(6) NS_BC(7)
#undef NS_BC
      int iter = 0;
      while (iter < m.noslip_iterations) {
        T impr = 0;
      // the 2 x 2 projection on the difference row (st_noslip_dense_sweep's update)
#define NS_UPD(K)                                                                          \
        if (K < maxlen) {                                                                 \
          const T rdk = rowbcast<K>(rd);                                                  \
          const T f0 = F0[K], f1 = F1[K];                                                 \
          const T mid = T(0.5) * (f0 + f1);                                               \
          T y = IK[K] != T(0) ? (f0 - mid) - rdk * IK[K] : T(0);                          \
          y = y < -mid ? -mid : (y > mid ? mid : y);                                      \
          const T n0 = mid + y, n1 = mid - y;                                             \
          const bool act = K < glen;                                                      \
          const T dl = act ? T(0.5) * ((n0 - f0) - (n1 - f1)) : T(0);                     \
          rd += Ad[K] * dl;                                                               \
          impr -= dl * (T(0.5) * dl * KK[K] + rdk);                                       \
          if (act) { F0[K] = n0; F1[K] = n1; }                                            \
        }
        NS_UPD(0) NS_UPD(1) NS_UPD(2) NS_UPD(3) NS_UPD(4) NS_UPD(5) NS_UPD(6) NS_UPD(7)
#undef NS_UPD
        iter++;
        if (ns_total(impr) * ns_scale < m.noslip_tolerance) break;
      }
      if (l == 0) s.noslip_iter = iter;
#pragma unroll
      for (int k = 0; k < NSR; k++)
        if (k < glen && q == 0) { s.efc_force[s.ns_list[grp][k]] = F0[k]; s.efc_force[s.ns_list[grp][k] + 1] = F1[k]; }
      wsync();
      return;
    }
  }
  // Long lists (a group with more than NSR pairs: closed fingers pressed together put 50+
  // contacts on the arm island) whose islands have <= 16 dofs: the island's v in registers, lane
  // q of the group = the island's dof q.  An update is then two row sums of J v, the 2 x 2
  // projection and a lane-local v += W df -- no v round trip through LDS and no wave sync
  // between updates (the streaming path below spends ~1.5k cycles per update on those).  A pair's
  // J / W entries are read from its packed slots at the lane's dof, one pair ahead, with its 2 x 2
  // Delassus block.  Islands are independent under Gauss-Seidel, so a group sweeps its (<= 2)
  // islands one after the other: each island sees the sequential order.  Rounding differs from
  // the streaming path (row sums in island-dof lane order).
  if (maxlen > NSR) {
    if (!__ballot(!small)) {
      // tree sizes packed 4 bits each (dofnum - 1, <= PH_MAXTDOF = 16): a row's first-tree width
      // is one bit-field extract, not a select chain over the trees
      static_assert(PH_MAXT <= 8 && PH_MAXTDOF <= 16, "tree sizes must pack into 4-bit fields");
      uint32_t tdn_pack = 0;
#pragma unroll
      for (int t = 0; t < PH_MAXT; t++)
        tdn_pack |= (uint32_t)((t < m.ntree ? s.c_tree_dofnum[t] : 1) - 1) << (4 * t);
      struct LSet {
        int k0, cnt, maxc, d, td, dloc;
        bool lane_on;
      };
      auto mkset = [&](int si) {
        LSet z;
        const int I = grp + 4 * si;
        const bool has = I < s.nisland;
        z.k0 = si ? iend0 : 0;
        z.cnt = has ? (si ? iend1 : iend0) - z.k0 : 0;
        z.maxc = max(max(__builtin_amdgcn_readlane(z.cnt, 0), __builtin_amdgcn_readlane(z.cnt, 16)),
                     max(__builtin_amdgcn_readlane(z.cnt, 32), __builtin_amdgcn_readlane(z.cnt, 48)));
        const int n = has ? s.isl_n[I] : 0;
        z.lane_on = q < n;
        z.d = z.lane_on ? s.isl_dof[I][q] : 0;
        z.td = s.c_dof_tree[z.d];
        z.dloc = z.d - s.c_tree_dofadr[z.td];
        return z;
      };
      const LSet S0 = mkset(0), S1 = mkset(1);
      T v0 = S0.lane_on ? s.v2[S0.d] : T(0), v1 = S1.lane_on ? s.v2[S1.d] : T(0);
      struct DRow {   // stage 2
        int j, t0, t1, off0, off1;
        bool act;
      };
      struct DRaw {   // stage 3
        int j;
        bool act;
        T Jd, Wd, bd, f0, f1;
      };
      // one sweep of the set's island, v in registers (lane q = island dof q); returns the group's
      // improvement.  Software pipeline over the pairs, one LDS level per stage, so that no wait
      // inside the loop covers a load issued in the same iteration: list entry 3 pairs ahead, the
      // row's trees and offsets 2 ahead, its J / W / b / f entries 1 ahead; the Delassus block of
      // a pair is formed at its own update (off the chain through v).  Tree sizes come from
      // registers.
      auto sweep = [&](const LSet& z, T& v) -> T {
        auto dlist = [&](int k) { return k < z.cnt ? (int)s.ns_list[grp][z.k0 + k] : -1; };
        auto drow = [&](int jj) {
          DRow x;
          x.act = jj >= 0;
          x.j = x.act ? jj : 0;   // (row 0 exists: nefc > 0)
          x.t0 = s.efc_t0[x.j];
          x.t1 = s.efc_t1[x.j];
          x.off0 = s.efc_off[x.j];
          x.off1 = s.efc_off[x.j + 1];
          return x;
        };
        auto draw = [&](const DRow& x) {
          const int n0 = x.t0 >= 0 ? (int)((tdn_pack >> (4 * x.t0)) & 15u) + 1 : 0;
          const int slot = z.td == x.t0 ? z.dloc : (z.td == x.t1 ? n0 + z.dloc : -1);
          const bool on = x.act && z.lane_on && slot >= 0;
          const int sl = on ? slot : 0;                 // unconditional, in-range loads; masked below
          DRaw p;
          p.j = x.j;
          p.act = x.act;
          const T J0 = s.efc_Jv[x.off0 + sl], J1 = s.efc_Jv[x.off1 + sl];
          const T W0 = s.efc_Wv[x.off0 + sl], W1 = s.efc_Wv[x.off1 + sl];
          p.Jd = on ? J0 - J1 : T(0);
          p.Wd = on ? W0 - W1 : T(0);
          p.bd = s.efc_bb[x.j];
          p.f0 = s.efc_force[x.j];
          p.f1 = s.efc_force[x.j + 1];
          return p;
        };
        T impr = 0;
        DRaw cur = draw(drow(dlist(0)));
        DRow x1 = drow(dlist(1));
        int j2 = dlist(2);
        for (int k = 0; k < z.maxc; k++) {
          const int j3 = dlist(k + 3);
          const DRow x2 = drow(j2);
          const DRaw nxt = draw(x1);
          // the projection on the pair's difference row (st_noslip_dense_sweep's update)
          const T K1 = rowsum16(cur.Jd * cur.Wd);
          const T rd = rowsum16(cur.Jd * v) + cur.bd;
          const T f0 = cur.f0, f1 = cur.f1;
          const T mid = T(0.5) * (f0 + f1);
          const bool flat = K1 < T(1e-15);
          T y = flat ? T(0) : (f0 - mid) - rd / K1;
          y = y < -mid ? -mid : (y > mid ? mid : y);
          const T n0 = mid + y, n1 = mid - y;
          const T dl = cur.act ? T(0.5) * ((n0 - f0) - (n1 - f1)) : T(0);
          impr -= dl * (T(0.5) * dl * K1 + rd);
          v += cur.Wd * dl;
          if (cur.act && q == 0) { s.efc_force[cur.j] = n0; s.efc_force[cur.j + 1] = n1; }
          cur = nxt;
          x1 = x2;
          j2 = j3;
        }
        wsync();   // the next sweep reads the forces this one wrote
        return impr;
      };
      int iter = 0;
      while (iter < m.noslip_iterations) {
        T impr = 0;
        if (S0.maxc) impr += sweep(S0, v0);
        if (S1.maxc) impr += sweep(S1, v1);
        iter++;
        if (ns_total(impr) * ns_scale < m.noslip_tolerance) break;
      }
      if (S0.lane_on) s.v2[S0.d] = v0;
      if (S1.lane_on) s.v2[S1.d] = v1;
      if (l == 0) s.noslip_iter = iter;
      wsync();
      return;
    }
  }
  if (maxlen <= NSR) {
    NsPair P[NSR];
    T K1s[NSR], F0[NSR], F1[NSR];
#pragma unroll
    for (int k = 0; k < NSR; k++) {
      P[k] = fetch(k < maxlen ? k : 0);
      P[k].act = P[k].act && k < maxlen;
      P[k].on = P[k].on && k < maxlen;
      K1s[k] = rowsum16(P[k].Jd * P[k].Wd);
      F0[k] = s.efc_force[P[k].j];
      F1[k] = s.efc_force[P[k].j + 1];
    }
    int iter = 0;
    while (iter < m.noslip_iterations) {
      T impr = 0;
#pragma unroll
      for (int k = 0; k < NSR; k++) {
        if (k >= maxlen) break;
        const NsPair& cur = P[k];
        const T vd = cur.on ? s.v2[cur.d] : T(0);
        const T rd = rowsum16(cur.Jd * vd) + cur.bd;
        const T f0 = F0[k], f1 = F1[k];
        const T mid = T(0.5) * (f0 + f1);
        const T K1 = K1s[k];
        T y = K1 < T(1e-15) ? T(0) : (f0 - mid) - rd / K1;
        if (y < -mid) y = -mid; else if (y > mid) y = mid;
        const T n0 = mid + y, n1 = mid - y;
        const T dl = T(0.5) * ((n0 - f0) - (n1 - f1));
        if (cur.on) s.v2[cur.d] = vd + cur.Wd * dl;
        impr = cur.act ? impr - dl * (T(0.5) * dl * K1 + rd) : impr;
        if (cur.act) { F0[k] = n0; F1[k] = n1; }
        wsync();
      }
      iter++;
      if (ns_total(impr) * ns_scale < m.noslip_tolerance) break;
    }
    if (l == 0) s.noslip_iter = iter;
#pragma unroll
    for (int k = 0; k < NSR; k++)
      if (P[k].act && q == 0) { s.efc_force[P[k].j] = F0[k]; s.efc_force[P[k].j + 1] = F1[k]; }
    wsync();
    return;
  }
  clk.count(SN_NS_STREAM, 1);
  int iter = 0;
  while (iter < m.noslip_iterations) {
    T impr = 0;
    NsPair cur = fetch(0);
    for (int k = 0; k < maxlen; k++) {
      const NsPair nxt = fetch(k + 1 < maxlen ? k + 1 : k);
      const T vd = cur.on ? s.v2[cur.d] : T(0);
      const T K1 = rowsum16(cur.Jd * cur.Wd);
      const T rd = rowsum16(cur.Jd * vd) + cur.bd;
      const T f0 = s.efc_force[cur.j], f1 = s.efc_force[cur.j + 1];
      const T mid = T(0.5) * (f0 + f1);
      T y = K1 < T(1e-15) ? T(0) : (f0 - mid) - rd / K1;
      if (y < -mid) y = -mid; else if (y > mid) y = mid;
      const T n0 = mid + y, n1 = mid - y;
      const T dl = T(0.5) * ((n0 - f0) - (n1 - f1));
      if (cur.on) s.v2[cur.d] += cur.Wd * dl;
      impr = cur.act ? impr - dl * (T(0.5) * dl * K1 + rd) : impr;
      if (cur.act && q == 0) { s.efc_force[cur.j] = n0; s.efc_force[cur.j + 1] = n1; }
      wsync();
      cur = nxt;
    }
    iter++;
    if (ns_total(impr) * ns_scale < m.noslip_tolerance) break;
  }
  if (l == 0) s.noslip_iter = iter;
  wsync();
}

template <typename T>
__device__ void st_finish_accel(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (s.nefc == 0) return;
  const bool jt = s.jt_ok;
  constexpr bool f32 = sizeof(T) == 4 && PNP_F32_NS_NEWTON;
  if (f32 && m.noslip_iterations > 0) {
    // fp32 (st_noslip): qacc = Newton's qacc + M^-1 J^T (f - f_newton), f_newton in efc_aref --
    // only the forces no-slip changed enter the sum
    for (int r = l; r < s.nefc; r += NT) s.efc_aref[r] = s.efc_force[r] - s.efc_aref[r];
    wsync();
  }
  const T* fsrc = f32 && m.noslip_iterations > 0 ? s.efc_aref : s.efc_force;
  if (jt) {
    gather_rows(s, fsrc, s.rr_g);
    wsync();
  }
  if (l < m.nv) {
    // J^T f over the dof's island rows (the other rows do not touch it)
    const int t = s.c_dof_tree[l], I = s.tree_island[t];
    const T g = jt ? jt_dof_sum(s, I, s.dof_ipos[l], T(0), s.rr_g)
                   : dof_row_sum(T(0), s, I, t, l - s.c_tree_dofadr[t], fsrc, (const T*)nullptr, false);
    s.v2[l] = f32 ? g : s.qfrc_smooth[l] + g;
  }
  wsync();
  if (m.noslip_iterations > 0) {
    if constexpr (f32) {
      solve_M(m, s, s.v2, s.v2);
      if (l < m.nv) s.qacc[l] += s.v2[l];
      wsync();
    } else {
      solve_M(m, s, s.qacc, s.v2);
    }
  }
}

// ============================================================================ reset / Euler
template <typename T>
__device__ void reset_state(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nq) s.qpos[l] = m.qpos0[l];
  if (l < m.nv) { s.qvel[l] = 0; s.qacc_ws[l] = 0; }
  if (l < m.nu) s.ctrl[l] = 0;
  if (l < m.nmocap) {
    const int b = m.mocap_body[l];
    for (int t = 0; t < 3; t++) s.mocap_pos[3 * l + t] = m.body_pos[b][t];
    for (int t = 0; t < 4; t++) s.mocap_quat[4 * l + t] = m.body_quat[b][t];
  }
  if (l == 0) s.time = 0;
  wsync();
}

template <typename T>
__device__ __forceinline__ bool is_bad(T x) { return !(fabs(x) <= T(1e10)); }

template <typename T>
__device__ void st_euler(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  const T h = m.timestep;
  // qfrc = M qacc ; (M + h D) qacc_e = qfrc  (implicit joint damping)
  if (l < m.nv) s.v1[l] = mulM_row(m, s, l, s.qacc);
  wsync();
  if (m.ntree <= GCH_GROUPS && !__ballot(l < m.ntree && s.c_tree_dofnum[l] > GCH_N)) {
    // every tree's M + h D on its own 9-lane group (undamped trees: M + h 0 = M, the same factor
    // st_factor_M made); rows through the dead solver scratch for the column reads
    const int g = gch_group(l), r = l - GCH_N * g, base = GCH_N * g;
    const bool on = g < m.ntree;
    const int n = on ? s.c_tree_dofnum[g] : 0, o = on ? s.c_tree_moff[g] : 0, a = on ? s.c_tree_dofadr[g] : 0;
    T Lrow[GCH_N], Ad[GCH_N], P[45], y[GCH_N];
#pragma unroll
    for (int j = 0; j < GCH_N; j++) {
      y[j] = T(0);
      Lrow[j] = r < n && j <= r ? s.M[o + r * n + j] + (j == r ? h * m.dof_damping[a + r] : T(0)) : T(r == j);
      Ad[j] = j < n ? s.M[o + j * n + j] + h * m.dof_damping[a + j] : T(1);
    }
    gch_factor(Lrow, Ad, r, base, P);
    chol_solve_reg<T, GCH_N>(P, n, y, s.v1 + a);
    T x = 0;
#pragma unroll
    for (int i = 0; i < GCH_N; i++) x = r == i ? y[i] : x;
    if (r < n) s.v2[a + r] = x;
  } else if (l < m.ntree) {
    const int n = s.c_tree_dofnum[l], o = s.c_tree_moff[l], a = s.c_tree_dofadr[l];
    bool damped = false;
    for (int i = 0; i < n; i++) damped |= m.dof_damping[a + i] != T(0);
    if (!damped) {
      // M + h*0 = M exactly: the factor from st_factor_M is this block's factor
      tree_solve(s, o, a, n, s.v2, s.v1);
    } else if (n <= 9) {
      T L[45];
      chol_reg<T, 9>(s.M + o, n, m.dof_damping + a, h, L);
      chol_solve_reg<T, 9>(L, n, s.v2 + a, s.v1 + a);
    } else {
      T* A = s.Hp;   // scratch (dead solver storage): the tree blocks' layout, nmblock <= PH_HCAP
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) A[o + i * n + j] = s.M[o + i * n + j] + (i == j ? h * m.dof_damping[a + i] : T(0));
      chol_block(A + o, A + o, n, n);
      chol_solve_block(A + o, n, n, (const int*)nullptr, a, s.v2, s.v1);
    }
  }
  wsync();
  if (l < m.nv) s.qvel[l] += h * s.v2[l];
  wsync();
  if (l < m.njnt) {
    const int qa = m.jnt_qposadr[l], da = m.jnt_dofadr[l];
    if (m.jnt_type[l] == 0) {
      for (int k = 0; k < 3; k++) s.qpos[qa + k] += h * s.qvel[da + k];
      T ax[3] = {s.qvel[da + 3], s.qvel[da + 4], s.qvel[da + 5]}, qr[4] = {1, 0, 0, 0};
      const T ang = h * t_normalize3(ax);
      if (ang != T(0)) {
        T sn, cs;
        d_sincos(ang * T(0.5), &sn, &cs);
        qr[0] = cs; qr[1] = ax[0] * sn; qr[2] = ax[1] * sn; qr[3] = ax[2] * sn;
      }
      T q[4] = {s.qpos[qa + 3], s.qpos[qa + 4], s.qpos[qa + 5], s.qpos[qa + 6]};
      t_normalize4(q);
      d_mulquat(q, q, qr);
      for (int k = 0; k < 4; k++) s.qpos[qa + 3 + k] = q[k];
    } else {
      s.qpos[qa] += h * s.qvel[da];
    }
  }
  if (l < m.nv) s.qacc_ws[l] = s.qacc[l];
  if (l == 0) s.time += h;
  wsync();
}

// ============================================================================ forward / kernel

// debug record of the contacts (PNP_DBG_CON): written right after collision, because the contact
// list shares storage with the solver's scratch
template <typename T>
__device__ void dump_contacts(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, double* o) {
  const DevPhys<T>& m = phys<T>();
  for (int c = lane_id(); c < s.ncon; c += NT) {
    double* q = o + PNP_DBG_CON + c * PNP_DBG_CON_STRIDE;
    for (int t = 0; t < 3; t++) q[t] = s.con[c].pos[t];
    for (int t = 0; t < 9; t++) q[3 + t] = s.con[c].frame[t];
    q[12] = s.con[c].dist;
    q[13] = m.geom_id[s.con[c].g1];
    q[14] = m.geom_id[s.con[c].g2];
    q[15] = s.con[c].dim;
  }
}

// debug record of the smooth forces: written before the solver, because the lean builds keep
// qfrc_bias / qfrc_actuator in storage the solver stages reuse
template <typename T>
__device__ void dump_smooth(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, double* o) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nv) {
    o[PNP_DBG_BIAS + l] = s.qfrc_bias[l];
    o[PNP_DBG_ACT + l] = s.qfrc_act[l];
    o[PNP_DBG_QACC_SMOOTH + l] = s.qacc_smooth[l];
  }
  for (int r = l; r < s.nefc; r += NT) o[PNP_DBG_EFC_AREF + r] = s.efc_aref[r];   // (fp32 no-slip reuses it)
}

template <typename T, class CLK>
__device__ void forward(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk, double* dbg = nullptr) {
  const DevPhys<T>& m = phys<T>();
  st_kinematics(m, s, clk); clk.lap(1);
  st_compos_crb(m, s);      clk.lap(2);
  st_factor_M(m, s);        clk.lap(3);
  st_collision(m, s, clk);
  if (s.nconvex) {
    clk.sub_start();
#if PNP_MW
    if constexpr (sizeof(T) == 4) {
      if (PNP_MPR_G < 64 || s.mw > 1) st_collision_convex_mw(s);
      else st_collision_convex(m, s);
    } else {
      st_collision_convex(m, s);
    }
#else
    st_collision_convex(m, s);
#endif
    clk.sub_lap(SC_CONVEX);
  }
  clk.lap(4);
  clk.count(SN_CON, s.ncon);
  clk.count(SN_CONVEX, s.nconvex);
  clk.count(SN_LIVE, s.nlive);
  if (PNP_HANDS && s.ovf) return;
  if (dbg) dump_contacts(m, s, dbg);
  st_constraints(m, s);     clk.lap(5);
  if (PNP_HANDS && s.ovf) return;
  st_velocity(m, s);        clk.lap(6);
  st_actuation_smooth(m, s); clk.lap(7);
  if (dbg) dump_smooth(m, s, dbg);
  st_newton(m, s, clk);     // laps 8..12 inside
  if (PNP_HANDS && s.ovf) return;
  clk.count(SN_EFC, s.nefc);
  clk.count(SN_ITER, s.solver_iter);
  clk.count(SN_ISLAND, s.nefc ? s.nisland : 0);
  st_noslip(m, s, clk);     clk.lap(13);
  clk.count(SN_NS_ITER, s.noslip_iter);
  st_finish_accel(m, s);    clk.lap(14);
}

template <typename T>
__device__ void forward(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  NoClock clk;
  forward(m, s, clk);
}

template <typename T>
__device__ void check_state(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  const bool bq = l < m.nq && is_bad(s.qpos[l]);
  const bool bv = l < m.nv && is_bad(s.qvel[l]);
  const uint64_t mq = __ballot(bq), mv = __ballot(bv);
  if (mq || mv) {
    if (l == 0) s.warn |= (mq ? 1u : 0u) | (mv ? 2u : 0u);
    wsync();
    reset_state(m, s);
  }
}

// save_qpos (gym env, last sub-step): the qpos the forward ran at, i.e. where MuJoCo's
// data.site_* / Jacobians stay after mj_step returns
template <typename T, class CLK>
__device__ void mj_step_dev(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, CLK& clk, T* save_qpos = nullptr) {
  const DevPhys<T>& m = phys<T>();
  clk.start();
  check_state(m, s);
  clk.lap(0);
  forward(m, s, clk);
  if (PNP_HANDS && s.ovf) return;   // state unchanged so far (check_state's reset is idempotent)
  const int l = lane_id();
  const uint64_t bad = __ballot(l < m.nv && is_bad(s.qacc[l]));
  if (bad) {
    if (l == 0) s.warn |= 4u;
    wsync();
    reset_state(m, s);
    forward(m, s, clk);
    if (PNP_HANDS && s.ovf) return;
  }
  if (save_qpos) {
    if (l < m.nq) save_qpos[l] = s.qpos[l];
    wsync();
  }
  st_euler(m, s);
  clk.lap(15);
}

template <typename T>
__device__ void load_env(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, const pnp_state_t<T>& st, int b,
                         int hand = 0) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < PH_MAXT) {
    s.c_tree_dofadr[l] = m.tree_dofadr[l];
    s.c_tree_dofnum[l] = m.tree_dofnum[l];
    s.c_tree_moff[l] = m.tree_moff[l];
  }
  if (l < PH_MAXV) s.c_dof_tree[l] = l < m.nv ? m.dof_tree[l] : 0;
  if (l < m.nq) s.qpos[l] = st.qpos[(size_t)b * m.nq + l];
  if (l < m.nv) { s.qvel[l] = st.qvel[(size_t)b * m.nv + l]; s.qacc_ws[l] = st.qacc_warmstart[(size_t)b * m.nv + l]; }
  if (l < m.nu) s.ctrl[l] = st.ctrl[(size_t)b * m.nu + l];
  if (l < 3 * m.nmocap) s.mocap_pos[l] = st.mocap_pos[(size_t)b * 3 * m.nmocap + l];
  if (l < 4 * m.nmocap) s.mocap_quat[l] = st.mocap_quat[(size_t)b * 4 * m.nmocap + l];
  if (l == 0) { s.time = st.time[b]; s.warn = st.warn[b] & 0xFFFFu; s.ovf = 0; s.hand = hand; }
#if PNP_MW
  if (l == 0) s.mw = 1;   // single-wave unless the kernel says otherwise (env_step_kernel)
#endif
  wsync();
}

template <typename T>
__device__ void store_env(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, const pnp_state_t<T>& st, int b) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nq) st.qpos[(size_t)b * m.nq + l] = s.qpos[l];
  if (l < m.nv) { st.qvel[(size_t)b * m.nv + l] = s.qvel[l]; st.qacc_warmstart[(size_t)b * m.nv + l] = s.qacc_ws[l]; }
  if (l == 0) { st.time[b] = s.time; st.warn[b] = s.warn; }   // ctrl / mocap are inputs only
}

// PNP_STEP_WAVES: minimum waves per SIMD the step kernel's registers are budgeted for (2 caps a
// wave at 256 VGPR+AGPR; only useful once the Env fits more than 4 envs per CU)
#ifndef PNP_STEP_WAVES
#define PNP_STEP_WAVES 1
#endif
// the full build's two-wave gym kernel (PNP_GYM_FULL_MW): waves per SIMD its registers are budgeted
// for -- 2 lets three envs' six waves share a CU, but only when every fp32 kernel of the build is
// budgeted alike (PNP_STEP_WAVES=2: the stages are shared functions)
#ifndef PNP_FULL_MW_EU
#define PNP_FULL_MW_EU 2
#endif
template <typename T, bool TIMED>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) step_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st, int B, int nsub,
                                                 unsigned long long* __restrict__ prof, int resume, int hand) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  const int b = blockIdx.x;
  if (b >= B) return;
  // resume pass: only the envs the previous tier handed over, from their sub-step; hand (full
  // build): hand overflowing sub-steps to the wide tier instead of truncating
  int k0 = 0;
  if (!PNP_COMPACT && resume) {
    const uint32_t w = st.warn[b];
    if (!(w & PNP_RESUME_FLAG)) return;
    k0 = (int)((w >> PNP_RESUME_SHIFT) & PNP_RESUME_MAXSUB);
  }
  load_env(m, s, st, b, hand);
  int k = k0;
  if constexpr (TIMED) {
    StageClock clk{prof + (size_t)b * PNP_NSTAGE, 0, 0};
    for (; k < nsub && !s.ovf; k++) mj_step_dev(m, s, clk);
  } else {
    NoClock clk;
    for (; k < nsub && !s.ovf; k++) mj_step_dev(m, s, clk);
  }
  // hand-over: sub-step k - 1 overflowed a capacity before changing the state
  if (PNP_HANDS && s.ovf && lane_id() == 0)
    s.warn |= PNP_RESUME_FLAG | ((uint32_t)s.ovf << PNP_RESUME_WHY_SHIFT) | ((uint32_t)(k - 1) << PNP_RESUME_SHIFT);
  wsync();
  store_env(m, s, st, b);
}

// debug: one forward, dump intermediates (layout PNP_DBG_* in include/pnp.h).  mode 0: this tier
// alone (truncating past its capacities like MuJoCo's full buffers); 1: a forward that outgrows
// this tier is handed to the next one (its record's COUNTS + 3, the warn slot, set to -1: a warn
// word is never negative); 2: resume -- only the envs whose record says handed over, rewritten
// whole by this tier.  So pnp_forward_debug sees the same capacities as pnp_step.
static_assert(PH_MAXCON <= PNP_DBG_MAXCON && PH_MAXEFC <= PNP_DBG_MAXEFC,
              "the debug record (include/pnp.h PNP_DBG_*) must hold every tier's contacts and rows");
template <typename T>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) forward_debug_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st, int B,
                                                          double* __restrict__ dbg, int mode) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  const int b = blockIdx.x;
  if (b >= B) return;
  double* o = dbg + (size_t)b * PNP_DBG_SIZE;
  if (mode == 2 && !(o[PNP_DBG_COUNTS + 3] < 0.0)) return;
  load_env(m, s, st, b, mode == 1);
  NoClock clk;
  forward(m, s, clk, o);
  const int l = lane_id();
  if (PNP_HANDS && s.ovf) {
    if (l == 0) o[PNP_DBG_COUNTS + 3] = -1.0;
    return;
  }
  const int nv = m.nv;
  for (int e = l; e < nv * nv; e += NT) {
    const int i = e / nv, j = e % nv;
    o[PNP_DBG_QM + e] = m.dof_tree[i] == m.dof_tree[j] ? (double)s.M[mblk(m, i, j)] : 0.0;
  }
  if (l < nv) {   // (bias, actuation, qacc_smooth: dump_smooth)
    o[PNP_DBG_QACC + l] = s.qacc[l];
    o[PNP_DBG_QACC_NEWTON + l] = s.x[l];
  }
  if (l == 0) {
    o[PNP_DBG_COUNTS + 0] = s.ncon;
    o[PNP_DBG_COUNTS + 1] = s.nefc;
    o[PNP_DBG_COUNTS + 2] = s.solver_iter;
    o[PNP_DBG_COUNTS + 3] = s.warn;
    o[PNP_DBG_NOSLIP_ITER] = s.noslip_iter;
  }
  for (int r = l; r < s.nefc; r += NT) {
    o[PNP_DBG_EFC_FORCE + r] = s.efc_force[r];
#if PNP_LEAN
    o[PNP_DBG_EFC_POS + r] = __builtin_nan("");   // (not kept by the lean builds: NaN, never compared)
#else
    o[PNP_DBG_EFC_POS + r] = s.efc_pos[r];
#endif
    o[PNP_DBG_EFC_D + r] = s.efc_D[r];
    o[PNP_DBG_EFC_TYPE + r] = s.efc_type[r];
    const int t0 = s.efc_t0[r], t1 = s.efc_t1[r], w = row_width(m, t0, t1);
    double* Jr = o + PNP_DBG_EFC_J + r * nv;
    for (int k = 0; k < nv; k++) Jr[k] = 0;
    for (int k = 0; k < w; k++) Jr[slot_dof(m, t0, t1, k)] = EJ(r, k);
  }
}

}  // namespace PNP_NS
using namespace PNP_NS;

// ============================================================================ host launchers
// The constant-segment images are made resident through ResidentLease (resident.cpp): stream-
// ordered copies, readers on other streams ordered after the copy, model switches after the
// readers of the old image.
#if PNP_COMPACT && PNP_GYM
// compact tier of the gym step (env_compact.hip): every env from sub-step 0; the full build's
// launch_env_step resumes the envs it hands over
#include "env_dev.h"

#elif PNP_COMPACT
int32_t launch_step_compact(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, int32_t nsub,
                            void* stream, unsigned long long* prof) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_COMPACT_F32, model, (const void*)&g_phys_f32, src, sizeof(DevPhys<float>),
                                       stream))
    return rc;
  auto k = prof ? step_kernel<float, true> : step_kernel<float, false>;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, B, nsub, prof, 0, 1);
  if (const int32_t rc = pnp_check_launch("step_kernel (compact)")) return rc;
  return lease.launched();
}

int32_t step_compact_lds_bytes() { return (int32_t)sizeof(Env<float>); }

#elif PNP_WIDE
// wide tier: the resume pass after the full kernel (resume = 1), or every env from sub-step 0
// (resume = 0: diagnostic PNP_STEP_COMPACT=3)
int32_t launch_step_wide(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, int32_t nsub,
                         void* stream, unsigned long long* prof, int resume) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE_F32, model, (const void*)&g_phys_f32, src, sizeof(DevPhys<float>),
                                       stream))
    return rc;
  auto k = prof ? step_kernel<float, true> : step_kernel<float, false>;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, B, nsub, prof, resume, 0);
  if (const int32_t rc = pnp_check_launch("step_kernel (wide)")) return rc;
  return lease.launched();
}

int32_t step_wide_lds_bytes() { return (int32_t)sizeof(Env<float>); }

int32_t launch_forward_debug_wide(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, double* dbg,
                                  void* stream) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE_F32, model, (const void*)&g_phys_f32, src, sizeof(DevPhys<float>),
                                       stream))
    return rc;
  hipLaunchKernelGGL(forward_debug_kernel<float>, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, B, dbg, 2);
  if (const int32_t rc = pnp_check_launch("forward_debug_kernel (wide)")) return rc;
  return lease.launched();
}

#include "env_dev.h"   // the gym step's wide resume pass

#elif PNP_WIDE64
// fp64 wide tier: the resume pass of pnp_step_f64 after the full fp64 kernel handed an env over
// (the single-env facade and the batched behaviour trees run in fp64; closed fingers on a cube make
// more than the full tier's 64 contacts); truncates past its own capacities with a warning
int32_t launch_step_wide64(const pnp_model* model, const pnp_state_t<double>* st, int32_t B, int32_t nsub,
                           void* stream) {
  const DevPhys<double>* src = phys_image<double>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE64_F64, model, (const void*)&g_phys_f64, src,
                                       sizeof(DevPhys<double>), stream))
    return rc;
  auto k = step_kernel<double, false>;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, B, nsub, (unsigned long long*)nullptr, 1, 0);
  if (const int32_t rc = pnp_check_launch("step_kernel (wide64)")) return rc;
  return lease.launched();
}

int32_t step_wide64_lds_bytes() { return (int32_t)sizeof(Env<double>); }

int32_t launch_forward_debug_wide64(const pnp_model* model, const pnp_state_t<double>* st, int32_t B, double* dbg,
                                    void* stream) {
  const DevPhys<double>* src = phys_image<double>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE64_F64, model, (const void*)&g_phys_f64, src,
                                       sizeof(DevPhys<double>), stream))
    return rc;
  hipLaunchKernelGGL(forward_debug_kernel<double>, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, B, dbg, 2);
  if (const int32_t rc = pnp_check_launch("forward_debug_kernel (wide64)")) return rc;
  return lease.launched();
}

#include "env_dev.h"   // the fp64 gym step's wide resume pass

#else

template <typename T>
int32_t phys_resident(const pnp_model* model, void* stream, ResidentLease& lease) {
  const DevPhys<T>* src = phys_image<T>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  const void* sym = sizeof(T) == 8 ? (const void*)&g_phys_f64 : (const void*)&g_phys_f32;
  return lease.acquire(sizeof(T) == 8 ? RES_FULL_F64 : RES_FULL_F32, model, sym, src, sizeof(DevPhys<T>), stream);
}
template int32_t phys_resident<float>(const pnp_model*, void*, ResidentLease&);
template int32_t phys_resident<double>(const pnp_model*, void*, ResidentLease&);

// PNP_STEP_COMPACT: unset / 1 = compact kernel + resume passes (default), 0 = the full kernel
// first (A/B runs, equivalence tests), 2 = the compact kernel alone — diagnostic only: handed-over
// envs are left at their hand-over sub-step with the resume bits set in warn, so that tests can
// see where hand-overs happen; 3 = the wide kernel alone (equivalence tests)
static int compact_mode() {
  const char* e = getenv("PNP_STEP_COMPACT");
  return e && (e[0] == '0' || e[0] == '2' || e[0] == '3') ? e[0] - '0' : 1;
}
static bool compact_enabled() { return compact_mode() == 1 || compact_mode() == 2; }
// PNP_STEP_WIDE: unset / 1 = fp32 sub-steps that outgrow the full kernel's capacities are finished
// by the wide tier (default), 0 = the full kernel truncates them with a warning (A/B runs)
static bool wide_enabled() {
  const char* e = getenv("PNP_STEP_WIDE");
  return !(e && e[0] == '0');
}
// PNP_GYM_COMPACT: unset / 1 = the fp32 gym step starts in the compact tier (default), 0 = in the
// full tier (A/B runs)
// (2: the compact gym kernel alone -- diagnostic: handed-over envs keep their resume bits)
static int gym_compact_mode() {
  const char* e = getenv("PNP_GYM_COMPACT");
  return e && (e[0] == '0' || e[0] == '2') ? e[0] - '0' : 1;
}
static bool gym_compact_enabled() { return gym_compact_mode() != 0; }

template <typename T>
static int32_t launch_step(pnp_model* model, const pnp_state_t<T>* st, int32_t B, int32_t nsub, void* stream,
                           double* dbg, unsigned long long* prof = nullptr) {
  if (!model || !st || B < 0 || nsub < 0) { pnp_set_error("pnp_step: bad argument"); return PNP_ERR_ARG; }
  if (B == 0 || (nsub == 0 && !dbg)) return PNP_OK;
  if (!st->qpos || !st->qvel || !st->ctrl || !st->mocap_pos || !st->mocap_quat || !st->qacc_warmstart ||
      !st->time || !st->warn) {
    pnp_set_error("pnp_step: null state buffer");
    return PNP_ERR_ARG;
  }
  const DevPhys<T>* dm = phys_image<T>(model);
  if (!dm) { pnp_set_error("pnp_step: model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = phys_resident<T>(model, stream, lease)) return rc;
  if (dbg) {
    // the full tier, handing what outgrows it to the wide tier (fp32: 192 contacts / 784 rows;
    // fp64: 96 / 400), which truncates like MuJoCo; PNP_STEP_WIDE=0: the full tier truncates
    const int hand = wide_enabled();
    auto k = forward_debug_kernel<T>;
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, B, dbg, hand);
    if (const int32_t rc = pnp_check_launch("forward_debug_kernel")) return rc;
    if (hand) {
      if constexpr (sizeof(T) == 8) {
        if (const int32_t rc = launch_forward_debug_wide64(model, reinterpret_cast<const pnp_state_t<double>*>(st), B,
                                                           dbg, stream))
          return rc;
      } else {
        if (const int32_t rc = launch_forward_debug_wide(model, reinterpret_cast<const pnp_state_t<float>*>(st), B,
                                                         dbg, stream))
          return rc;
      }
    }
    return lease.launched();
  }
  auto k = prof ? step_kernel<T, true> : step_kernel<T, false>;
  const bool tiers = sizeof(T) == 4 && nsub <= PNP_RESUME_MAXSUB;   // the resume bits hold the sub-step
  const int wide = tiers && wide_enabled();
  if constexpr (sizeof(T) == 8) {
    // fp64: the full kernel, handing the sub-steps that outgrow it to the fp64 wide tier
    const int w64 = nsub <= PNP_RESUME_MAXSUB && wide_enabled();
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, B, nsub, prof, 0, w64);
    if (const int32_t rc = pnp_check_launch("step_kernel (fp64)")) return rc;
    if (w64)
      if (const int32_t rc = launch_step_wide64(model, reinterpret_cast<const pnp_state_t<double>*>(st), B, nsub,
                                                stream))
        return rc;
    return lease.launched();
  }
  const auto* st32 = reinterpret_cast<const pnp_state_t<float>*>(st);
  if (tiers && compact_mode() == 3) {
    if (const int32_t rc = launch_step_wide(model, st32, B, nsub, stream, prof, 0)) return rc;
    return lease.launched();
  }
  if (tiers && compact_enabled()) {
    // compact kernel over every env, then the full kernel resumes the envs it handed over (an
    // env not handed over costs the resume pass one load of its warn word), then the wide kernel
    // the envs the full kernel handed over
    if (const int32_t rc = launch_step_compact(model, st32, B, nsub, stream, prof)) return rc;
    if (compact_mode() == 2) return lease.launched();
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, B, nsub, prof, 1, wide);
    if (const int32_t rc = pnp_check_launch("step_kernel (resume)")) return rc;
  } else {
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, B, nsub, prof, 0, wide);
    if (const int32_t rc = pnp_check_launch("step_kernel")) return rc;
  }
  if (wide)
    if (const int32_t rc = launch_step_wide(model, st32, B, nsub, stream, prof, 1)) return rc;
  return lease.launched();
}

extern "C" int32_t pnp_step(pnp_model* model, const pnp_state* st, int32_t B, int32_t nsub, void* stream) {
  return launch_step<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), B, nsub, stream, nullptr);
}
extern "C" int32_t pnp_step_f64(pnp_model* model, const pnp_state_f64* st, int32_t B, int32_t nsub, void* stream) {
  return launch_step<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), B, nsub, stream, nullptr);
}
extern "C" int32_t pnp_forward_debug(pnp_model* model, const pnp_state* st, int32_t B, double* dbg, void* stream) {
  if (!dbg) { pnp_set_error("pnp_forward_debug: null dbg"); return PNP_ERR_ARG; }
  return launch_step<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), B, 0, stream, dbg);
}
extern "C" int32_t pnp_forward_debug_f64(pnp_model* model, const pnp_state_f64* st, int32_t B, double* dbg,
                                         void* stream) {
  if (!dbg) { pnp_set_error("pnp_forward_debug: null dbg"); return PNP_ERR_ARG; }
  return launch_step<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), B, 0, stream, dbg);
}
extern "C" int32_t pnp_step_profile(pnp_model* model, const pnp_state* st, int32_t B, int32_t nsub,
                                    unsigned long long* stage_cycles, void* stream) {
  if (!stage_cycles) { pnp_set_error("pnp_step_profile: null stage_cycles"); return PNP_ERR_ARG; }
  return launch_step<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), B, nsub, stream, nullptr,
                            stage_cycles);
}

extern "C" int32_t pnp_step_lds_bytes(int32_t fp64) {
  return fp64 ? (int32_t)sizeof(Env<double>) : (int32_t)sizeof(Env<float>);
}

// ============================================================================ gym env (fused)
// (full build only: the gym step runs the full-capacity kernel.  A compact gym path -- set_action,
// compact physics launches with resume passes, observation -- was built and measured at eadc013:
// bit-exact, but random-action workloads keep > 20 contacts in about a third of the envs (closed
// finger pads), so it ran slower than one full launch (275 vs 304-337 ms per 4096-env gym step),
// and compiling the gym kernels into the compact build grew the compact step kernel's call
// frames (scratch 384 -> 464 B per lane, 5x the HBM write-back traffic).)
#include "env_dev.h"
static_assert(PH_MAXCON == PNP_GF_MAXCON && PH_MAXEFC == PNP_GF_MAXEFC && PH_MAXJSLOT == PNP_GF_MAXJSLOT &&
                  PH_JTCAP == PNP_GF_JTCAP,
              "env_dev.h's routing estimate (tier_need) must see the full tier's capacities");
#endif  // !PNP_COMPACT
