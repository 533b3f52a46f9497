// ik_dls.hip — batched JacobianIKController.solve (reference skills/ik_solver.py:35-101).
//
// One thread per env, the whole solve (<= max_iters iterations) inside one launch, all per-env
// state in VGPRs: the 7 joint angles, the chain frames, the 3x7 Jacobian and the 3x3 DLS
// system never leave registers.  HBM traffic is the 92 B/solve of the batch arrays
// (q_init 28 + target 12 in; q 28 + final_pos 12 + err 4 + iters 4 + flags 1 out).
//
// Kinematics: the 10-body root->ee_center_site path is folded on the host (pnp_capi.cpp) into
// 7 hinge "segments" {fixed transform to the joint body, rotation about +-z} plus a fixed site
// offset, so the FK loop is a fully unrolled chain of 3x3 products with static register
// indices.  The numerics follow MuJoCo's mj_kinematics / mj_jacSite semantics (see oracle.c).
//
// Control flow is the reference's, line for line:
//   for i < max_iters: p = FK(q); e = target - p; if |e| < thr: converged, iters = i+1, break
//                      J = jacp; dq = J^T (J J^T + damping I)^-1 e   (LU, partial pivoting)
//                      q = clip(q + clip(dq, +-step), lo, hi); iters = i+1
//   final = FK(q); err = |final - target|; success = converged && err < 2 thr
#include "pnp_internal.h"

#include "gen/panda_chain.h"

template <typename T>
struct IKSeg {
  T Rpre[7][9];   // fixed rotation from the previous joint frame to joint j's body frame
  T ppre[7][3];   // fixed translation (in the previous joint frame)
  T sgn[7];       // hinge axis = sgn * z
  T psite[3];     // site position in the frame of the last joint body
  T lo[7], hi[7];
  T qpos0[7];
};

// Chain constants: compile-time (baked Panda chain, gen/panda_chain.h) or kernel-argument.
// After full unrolling every index is static, so the baked values fold into the FMAs and the
// 0 / +-1 entries of the +-90 deg body rotations disappear.
#define IK_CONST(field, cfield, ...) \
  (BAKED ? (T)panda_chain::field __VA_ARGS__ : c.cfield __VA_ARGS__)

// ---------------------------------------------------------------------------- fp32 fast math
// sin/cos for the arm's joint-angle range (|x| < 2^7): Cody-Waite reduction by pi/2 in three
// parts + Cephes minimax polynomials on [-pi/4, pi/4] (<= 1 ulp there).  The library sincosf
// carries a Payne-Hanek large-argument path that more than doubled the kernel's instruction
// count; joint angles never need it.
__device__ __forceinline__ void fast_sincos(float x, float* s, float* c) {
  const float k = __builtin_rintf(x * 0.636619772367581343f);
  float r = __builtin_fmaf(k, -1.5703125f, x);
  r = __builtin_fmaf(k, -4.837512969970703125e-4f, r);
  r = __builtin_fmaf(k, -7.549789954891882e-8f, r);
  const float r2 = r * r;
  float ps = __builtin_fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = __builtin_fmaf(r2, ps, -1.6666654611e-1f);
  const float sn = __builtin_fmaf(r * r2, ps, r);
  float pc = __builtin_fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = __builtin_fmaf(r2, pc, 4.166664568298827e-2f);
  const float cs = __builtin_fmaf(r2 * r2, pc, __builtin_fmaf(r2, -0.5f, 1.0f));
  const int q = (int)k;
  const float ss = (q & 1) ? cs : sn;
  const float cc = (q & 1) ? sn : cs;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}

template <typename T> struct KMath;
template <> struct KMath<float> {
  // The hardware v_sin_f32 / v_cos_f32 (argument in revolutions: x * 1/(2 pi), rounded once, so
  // <= 5e-7 rad absolute over the joint range |x| < 6.3) -- 3 instructions instead of the 27 of
  // fast_sincos's reduction, polynomials and quadrant selects; the IK iteration is issue-bound on
  // one wave per SIMD, so that is 8 % of the launch (69.2 -> 64.0 us per 4096 solves, iteration
  // counts identical on both C2 regimes, profiles/r02/ik_v6_ab.log).  The fp32 parity bars hold:
  // one DLS iteration within 1e-5 of the fp64 oracle, final_pos within 2e-6 m of the kinematics
  // kernel (tests/test_ik_gpu.py).  -DPNP_IK_POLYSIN restores fast_sincos (A/B builds).
#ifdef PNP_IK_POLYSIN
  static __device__ __forceinline__ void sincos(float x, float* s, float* c) { fast_sincos(x, s, c); }
#else
  static __device__ __forceinline__ void sincos(float x, float* s, float* c) { *s = __sinf(x); *c = __cosf(x); }
#endif
  static __device__ __forceinline__ float sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
  static __device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
};
template <> struct KMath<double> {
  static __device__ __forceinline__ void sincos(double x, double* s, double* c) { ::sincos(x, s, c); }
  static __device__ __forceinline__ double sqrt(double x) { return ::sqrt(x); }
  static __device__ __forceinline__ double rcp(double x) { return 1.0 / x; }
};

template <typename T, bool BAKED>
__device__ __forceinline__ void ik_fk(const IKSeg<T>& c, const T q[7], T site[3], T anchor[7][3],
                                      T axis[7][3]) {
  T R[9], p[3];
#pragma unroll
  for (int j = 0; j < 7; j++) {
    if (j == 0) {
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = IK_CONST(kRpre, Rpre, [0][k]);
#pragma unroll
      for (int k = 0; k < 3; k++) p[k] = IK_CONST(kPpre, ppre, [0][k]);
    } else {
#pragma unroll
      for (int r = 0; r < 3; r++)
        p[r] += R[3 * r + 0] * IK_CONST(kPpre, ppre, [j][0]) + R[3 * r + 1] * IK_CONST(kPpre, ppre, [j][1]) +
                R[3 * r + 2] * IK_CONST(kPpre, ppre, [j][2]);
      T N[9];
#pragma unroll
      for (int r = 0; r < 3; r++)
#pragma unroll
        for (int col = 0; col < 3; col++)
          N[3 * r + col] = R[3 * r + 0] * IK_CONST(kRpre, Rpre, [j][0 + col]) +
                           R[3 * r + 1] * IK_CONST(kRpre, Rpre, [j][3 + col]) +
                           R[3 * r + 2] * IK_CONST(kRpre, Rpre, [j][6 + col]);
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = N[k];
    }
    // joint j: anchor at the body origin, world axis = sgn * (R e_z)
    const T sg = IK_CONST(kSgn, sgn, [j]);
    anchor[j][0] = p[0]; anchor[j][1] = p[1]; anchor[j][2] = p[2];
    axis[j][0] = sg * R[2]; axis[j][1] = sg * R[5]; axis[j][2] = sg * R[8];
    T s, co;
    KMath<T>::sincos(q[j] - IK_CONST(kQpos0, qpos0, [j]), &s, &co);
    s *= sg;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const T a = R[3 * r + 0], b = R[3 * r + 1];
      R[3 * r + 0] = a * co + b * s;
      R[3 * r + 1] = b * co - a * s;
    }
  }
#pragma unroll
  for (int r = 0; r < 3; r++)
    site[r] = p[r] + R[3 * r + 0] * IK_CONST(kPsite, psite, [0]) + R[3 * r + 1] * IK_CONST(kPsite, psite, [1]) +
              R[3 * r + 2] * IK_CONST(kPsite, psite, [2]);
}

// fp64: 3x3 LU with partial pivoting (LAPACK getrf/getrs order, as numpy.linalg.solve), so
// the debugging instantiation tracks the reference's arithmetic.
__device__ __forceinline__ void solve3(double A[9], double b[3]) {
#pragma unroll
  for (int k = 0; k < 3; k++) {
    int p = k;
    double mx = fabs(A[3 * k + k]);
#pragma unroll
    for (int i = k + 1; i < 3; i++) {
      const double v = fabs(A[3 * i + k]);
      if (v > mx) { mx = v; p = i; }
    }
#pragma unroll
    for (int i = k + 1; i < 3; i++) {   // branch-free swap keeps register indices static
      const bool sw = (p == i);
#pragma unroll
      for (int col = 0; col < 3; col++) {
        const double x = A[3 * k + col], y = A[3 * i + col];
        A[3 * k + col] = sw ? y : x;
        A[3 * i + col] = sw ? x : y;
      }
      const double x = b[k], y = b[i];
      b[k] = sw ? y : x;
      b[i] = sw ? x : y;
    }
    const double r = 1.0 / A[3 * k + k];
#pragma unroll
    for (int i = k + 1; i < 3; i++) {
      const double l = A[3 * i + k] * r;
#pragma unroll
      for (int col = k + 1; col < 3; col++) A[3 * i + col] -= l * A[3 * k + col];
      b[i] -= l * b[k];
    }
  }
#pragma unroll
  for (int i = 2; i >= 0; i--) {
    double s = b[i];
#pragma unroll
    for (int col = i + 1; col < 3; col++) s -= A[3 * i + col] * b[col];
    b[i] = s / A[3 * i + i];
  }
}

// fp32: A = J J^T + damping I is symmetric positive definite (damping > 0), so an LDL^T
// factorisation needs no pivoting: 3 reciprocals + ~20 FMAs, backward stable.
__device__ __forceinline__ void solve3(float A[9], float b[3]) {
  const float d0 = A[0], i0 = __builtin_amdgcn_rcpf(d0);
  const float l10 = A[3] * i0, l20 = A[6] * i0;
  const float d1 = __builtin_fmaf(-l10, A[3], A[4]), i1 = __builtin_amdgcn_rcpf(d1);
  const float l21 = __builtin_fmaf(-l20, A[3], A[7]) * i1;
  const float d2 = A[8] - l20 * A[6] - l21 * l21 * d1, i2 = __builtin_amdgcn_rcpf(d2);
  const float z0 = b[0], z1 = __builtin_fmaf(-l10, z0, b[1]);
  const float z2 = b[2] - l20 * z0 - l21 * z1;
  const float x2 = z2 * i2;
  const float x1 = __builtin_fmaf(-l21, x2, z1 * i1);
  const float x0 = z0 * i0 - l10 * x1 - l20 * x2;
  b[0] = x0; b[1] = x1; b[2] = x2;
}

template <typename T, bool BAKED>
__global__ void __launch_bounds__(64) ik_dls_kernel(IKSeg<T> c, int max_iters, T thr, T damping,
                                                    T step, const T* __restrict__ q_init,
                                                    const T* __restrict__ target,
                                                    T* __restrict__ q_out, T* __restrict__ final_pos,
                                                    T* __restrict__ pos_error,
                                                    int32_t* __restrict__ iterations,
                                                    uint8_t* __restrict__ flags, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  T q[7], tg[3];
#pragma unroll
  for (int j = 0; j < 7; j++) q[j] = q_init[(size_t)b * 7 + j];
  tg[0] = target[(size_t)b * 3]; tg[1] = target[(size_t)b * 3 + 1]; tg[2] = target[(size_t)b * 3 + 2];

  T site[3], anchor[7][3], axis[7][3];
  ik_fk<T, BAKED>(c, q, site, anchor, axis);
  int converged = 0, iters = 0;
  for (int i = 0; i < max_iters; i++) {
    const T e0 = tg[0] - site[0], e1 = tg[1] - site[1], e2 = tg[2] - site[2];
    const T n = KMath<T>::sqrt(e0 * e0 + e1 * e1 + e2 * e2);
    if (n < thr) {
      converged = 1;
      iters = i + 1;
      break;
    }
    // jacp columns: axis_j x (site - anchor_j)
    T J[3][7];
#pragma unroll
    for (int j = 0; j < 7; j++) {
      const T r0 = site[0] - anchor[j][0], r1 = site[1] - anchor[j][1], r2 = site[2] - anchor[j][2];
      J[0][j] = axis[j][1] * r2 - axis[j][2] * r1;
      J[1][j] = axis[j][2] * r0 - axis[j][0] * r2;
      J[2][j] = axis[j][0] * r1 - axis[j][1] * r0;
    }
    T A[9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int col = r; col < 3; col++) {
        T acc = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) acc += J[r][k] * J[col][k];
        A[3 * r + col] = acc;
        A[3 * col + r] = acc;
      }
    A[0] += damping; A[4] += damping; A[8] += damping;
    T y[3] = {e0, e1, e2};
    solve3(A, y);
#pragma unroll
    for (int j = 0; j < 7; j++) {
      T dq = J[0][j] * y[0] + J[1][j] * y[1] + J[2][j] * y[2];
      dq = fmin(fmax(dq, -step), step);
      q[j] = fmin(fmax(q[j] + dq, IK_CONST(kLo, lo, [j])), IK_CONST(kHi, hi, [j]));
    }
    ik_fk<T, BAKED>(c, q, site, anchor, axis);
    iters = i + 1;
  }
  const T d0 = site[0] - tg[0], d1 = site[1] - tg[1], d2 = site[2] - tg[2];
  const T err = KMath<T>::sqrt(d0 * d0 + d1 * d1 + d2 * d2);
#pragma unroll
  for (int j = 0; j < 7; j++) q_out[(size_t)b * 7 + j] = q[j];
  final_pos[(size_t)b * 3] = site[0];
  final_pos[(size_t)b * 3 + 1] = site[1];
  final_pos[(size_t)b * 3 + 2] = site[2];
  pos_error[b] = err;
  iterations[b] = iters;
  flags[b] = (uint8_t)((converged ? PNP_IK_CONVERGED : 0u) |
                       ((converged && err < thr * T(2)) ? PNP_IK_SUCCESS : 0u));
}

// ---------------------------------------------------------------------------- lane groups
// ik_dls_group_kernel: one solve per 16-lane DPP row (4 solves per wave), lane j < 7 owns joint
// j, lane 7 the site, lanes 8..15 run along unused.  (v4 packed 8 solves per wave on 8-lane
// groups; then the row_shr of the scan leaked the neighbouring group's frames into lanes 8..8+O-1
// and every one of the 12 received entries needed a select.  With a group per row the lanes
// without a source are exactly j < O and the DPP's zero fill supplies the identity's zeros: 27
// fewer instructions per iteration, and 4096 solves make 1024 waves -- one per SIMD -- instead of
// 512 on half the SIMDs.)
// The thread-per-solve kernel above is latency-bound: a batch of 4096 solves is 64 waves on
// 64 CUs, and the launch lasts as long as the slowest solve (up to max_iters iterations), each
// iteration one long dependent chain (7 joint rotations composed in order, then the Jacobian, the
// 3 x 3 solve and the update).  Here every iteration is shallow:
//   * lane j forms its joint's local transform A_j = [Rpre_j Rz(q_j) | ppre_j] (its own sincos);
//     lane 7 carries the site offset [I | psite];
//   * the world frames G_j = A_0 ... A_j are an inclusive prefix product over the group
//     (Hillis-Steele, 3 DPP row_shr steps); lane 7 ends up holding the site position;
//   * anchor_j = p(G_j), axis_j = sgn_j R(G_j) e_z (Rz leaves both unchanged, as in ik_fk);
//   * J J^T is 6 three-step DPP sums over lanes 0..7 (J column j on lane j), the 3 x 3 solve runs
//     redundantly on every lane, and dq_j = J_j^T y is lane-local.
// The reference's control flow is kept per group (convergence test before the update, the final
// position measured after the last update); groups that have stopped are predicated off.  Same
// formulas as the serial kernel; the frame products associate differently (prefix tree instead
// of the left-to-right chain), so results agree to rounding (fp64: ~1e-16 relative).
// ZERO: a lane whose DPP source is outside its row (row_shr:O, lanes 0..O-1) reads 0 (bound_ctrl)
template <int CTRL, typename T, bool ZERO = false>
__device__ __forceinline__ T gdpp(T v) {
  if constexpr (sizeof(T) == 4) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, ZERO));
  } else {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, ZERO);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, ZERO);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
  }
}
// sum over the 8-lane group, identical bits in every lane
template <typename T>
__device__ __forceinline__ T gsum8(T v) {
  v += gdpp<0xB1>(v);    // quad_perm [1,0,3,2]
  v += gdpp<0x4E>(v);    // quad_perm [2,3,0,1]
  v += gdpp<0x141>(v);   // row_half_mirror: the other quad of the group
  return v;
}
// six group sums at once, level by level: the three DPP steps of one sum each wait on the previous
// add (a VALU write read by DPP needs two wait states), which the compiler filled with s_nop when
// the sums were written one after the other; interleaved, each sum's wait is the others' issue.
// Same additions per value, so the same bits as six gsum8 calls.
template <typename T>
__device__ __forceinline__ void gsum8x6(T v[6]) {
  T t[6];
#pragma unroll
  for (int k = 0; k < 6; k++) t[k] = gdpp<0xB1>(v[k]);
#pragma unroll
  for (int k = 0; k < 6; k++) v[k] += t[k];
#pragma unroll
  for (int k = 0; k < 6; k++) t[k] = gdpp<0x4E>(v[k]);
#pragma unroll
  for (int k = 0; k < 6; k++) v[k] += t[k];
#pragma unroll
  for (int k = 0; k < 6; k++) t[k] = gdpp<0x141>(v[k]);
#pragma unroll
  for (int k = 0; k < 6; k++) v[k] += t[k];
}
// lane 7 of the group (= of its DPP row) to every lane of the row (row_newbcast:7)
template <typename T>
__device__ __forceinline__ T gbcast7(T v) {
  return gdpp<0x157>(v);
}
// one Hillis-Steele step: G_j <- G_{j-O} G_j for j >= O (row_shr:O inside the group's row of
// 16).  A lane j < O has no DPP source in its row and composes with the identity instead (1 x +
// 0 y + 0 z + 0 is x exactly for finite values), so every lane runs the same straight-line code:
// the identity's zeros come from the DPP's bound_ctrl zero fill, only its three ones need a select.
template <int O, typename T>
__device__ __forceinline__ void gscan_step(T R[9], T p[3], int j) {
  const bool take = j >= O;
  T X[9], xp[3];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    if (k == 0 || k == 4 || k == 8) {
      const T v = gdpp<0x110 + O>(R[k]);
      X[k] = take ? v : T(1);
    } else {
      X[k] = gdpp<0x110 + O, T, true>(R[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) xp[k] = gdpp<0x110 + O, T, true>(p[k]);
  T N[9], np[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int c = 0; c < 3; c++) N[3 * r + c] = X[3 * r] * R[c] + X[3 * r + 1] * R[3 + c] + X[3 * r + 2] * R[6 + c];
    np[r] = X[3 * r] * p[0] + X[3 * r + 1] * p[1] + X[3 * r + 2] * p[2] + xp[r];
  }
#pragma unroll
  for (int k = 0; k < 9; k++) R[k] = N[k];
#pragma unroll
  for (int k = 0; k < 3; k++) p[k] = np[k];
}

// frames of the group at its joint angles: lane j -> (anchor_j, axis_j); every lane -> site
template <typename T>
__device__ __forceinline__ void gfk(const T Rp[9], const T pp[3], T sg, T q0, T qj, bool joint, int j,
                                    T anchor[3], T axis[3], T site[3]) {
  T s, c;
  KMath<T>::sincos(qj - q0, &s, &c);   // lane 7: sincos(0), and sg = 0
  s *= sg;
  (void)joint;
  T R[9], p[3] = {pp[0], pp[1], pp[2]};
#pragma unroll
  for (int r = 0; r < 3; r++) {     // Rpre_j Rz(q_j): rotate columns 0 and 1
    R[3 * r + 0] = Rp[3 * r + 0] * c + Rp[3 * r + 1] * s;
    R[3 * r + 1] = Rp[3 * r + 1] * c - Rp[3 * r + 0] * s;
    R[3 * r + 2] = Rp[3 * r + 2];
  }
  gscan_step<1>(R, p, j);
  gscan_step<2>(R, p, j);
  gscan_step<4>(R, p, j);
  anchor[0] = p[0]; anchor[1] = p[1]; anchor[2] = p[2];
  axis[0] = sg * R[2]; axis[1] = sg * R[5]; axis[2] = sg * R[8];
#pragma unroll
  for (int k = 0; k < 3; k++) site[k] = gbcast7(p[k]);
}

template <typename T>
__global__ void __launch_bounds__(64) ik_dls_group_kernel(IKSeg<T> c, int max_iters, T thr, T damping, T step,
                                                          const T* __restrict__ q_init, const T* __restrict__ target,
                                                          T* __restrict__ q_out, T* __restrict__ final_pos,
                                                          T* __restrict__ pos_error, int32_t* __restrict__ iterations,
                                                          uint8_t* __restrict__ flags, int B) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = t >> 4, j = t & 15;
  const bool valid = b < B;          // (a partial group past B runs along, predicated off)
  const bool joint = j < 7;
  // this lane's joint constants (lane 7: the site offset, no rotation; lanes 8..15 likewise --
  // they run along and are never read: the group sums cover lanes 0..7 of the row)
  T Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pp[3] = {c.psite[0], c.psite[1], c.psite[2]};
  T sg = 0, lo = 0, hi = 0, q0 = 0;
#pragma unroll
  for (int jj = 0; jj < 7; jj++) {
    if (j == jj) {
#pragma unroll
      for (int k = 0; k < 9; k++) Rp[k] = c.Rpre[jj][k];
#pragma unroll
      for (int k = 0; k < 3; k++) pp[k] = c.ppre[jj][k];
      sg = c.sgn[jj]; lo = c.lo[jj]; hi = c.hi[jj]; q0 = c.qpos0[jj];
    }
  }
  T q = (valid && joint) ? q_init[(size_t)b * 7 + j] : T(0);
  T tg[3] = {0, 0, 0};
  if (valid) { tg[0] = target[(size_t)b * 3]; tg[1] = target[(size_t)b * 3 + 1]; tg[2] = target[(size_t)b * 3 + 2]; }
  T anchor[3], axis[3], site[3];
  bool active = valid;
  int converged = 0, iters = 0;
  // the frames are formed at the top of each iteration (and once more after the loop for the
  // final position), so only q and the flags are carried around the loop: formed at the bottom,
  // anchor / axis / site were loop-carried values the compiler copied on every back edge
  for (int i = 0; i < max_iters; i++) {
    gfk(Rp, pp, sg, q0, q, joint, j, anchor, axis, site);
    const T e0 = tg[0] - site[0], e1 = tg[1] - site[1], e2 = tg[2] - site[2];
    const T n = KMath<T>::sqrt(e0 * e0 + e1 * e1 + e2 * e2);
    if (active && n < thr) {
      converged = 1;
      iters = i + 1;
      active = false;
    }
    if (!__ballot(active)) break;
    // jacp column j: axis_j x (site - anchor_j); lane 7's axis is sg R e_z = 0 (sg = 0), so its
    // column is exactly zero without a select
    const T r0 = site[0] - anchor[0], r1 = site[1] - anchor[1], r2 = site[2] - anchor[2];
    const T J0 = axis[1] * r2 - axis[2] * r1;
    const T J1 = axis[2] * r0 - axis[0] * r2;
    const T J2 = axis[0] * r1 - axis[1] * r0;
    T A[9], jj[6] = {J0 * J0, J0 * J1, J0 * J2, J1 * J1, J1 * J2, J2 * J2};
    gsum8x6(jj);
    A[0] = jj[0] + damping;
    A[1] = A[3] = jj[1];
    A[2] = A[6] = jj[2];
    A[4] = jj[3] + damping;
    A[5] = A[7] = jj[4];
    A[8] = jj[5] + damping;
    T y[3] = {e0, e1, e2};
    solve3(A, y);
    T dq = J0 * y[0] + J1 * y[1] + J2 * y[2];
    dq = fmin(fmax(dq, -step), step);
    const T qn = fmin(fmax(q + dq, lo), hi);
    q = (active && joint) ? qn : q;
    iters = active ? i + 1 : iters;
  }
  gfk(Rp, pp, sg, q0, q, joint, j, anchor, axis, site);
  if (!valid) return;
  const T d0 = site[0] - tg[0], d1 = site[1] - tg[1], d2 = site[2] - tg[2];
  const T err = KMath<T>::sqrt(d0 * d0 + d1 * d1 + d2 * d2);
  if (joint) q_out[(size_t)b * 7 + j] = q;
  if (j < 3) final_pos[(size_t)b * 3 + j] = site[j == 0 ? 0 : (j == 1 ? 1 : 2)];
  if (j == 0) {
    pos_error[b] = err;
    iterations[b] = iters;
    flags[b] = (uint8_t)((converged ? PNP_IK_CONVERGED : 0u) |
                         ((converged && err < thr * T(2)) ? PNP_IK_SUCCESS : 0u));
  }
}

// ---------------------------------------------------------------------------- host side
static void mat_mul3(double r[9], const double a[9], const double b[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  for (int k = 0; k < 9; k++) r[k] = t[k];
}

static void quat_to_mat(double m[9], const double q[4]) {
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[4] = q00 - q11 + q22 - q33; m[8] = q00 - q11 - q22 + q33;
  m[1] = 2 * (q12 - q03); m[2] = 2 * (q13 + q02); m[3] = 2 * (q12 + q03);
  m[5] = 2 * (q23 - q01); m[6] = 2 * (q13 - q02); m[7] = 2 * (q23 + q01);
}

// Fold the root -> site body path into 7 hinge segments.  Requirements (the Panda satisfies
// them; anything else is PNP_ERR_UNSUPPORTED): no mocap/free/slide/ball joint on the path,
// exactly the hinges 0..6 in order, each hinge through its body origin about +-z.
static int32_t build_segments(const pnp_model* M, int site, IKSeg<double>* out) {
  const DevModel<double>& m = M->h;
  int path[PNP_MAXBODY], n = 0;
  for (int b = m.site_bodyid[site]; b > 0; b = m.body_parentid[b]) {
    if (n >= PNP_MAXBODY) return PNP_ERR_MODEL;
    path[n++] = b;
  }
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
  int nj = 0;
  for (int k = n - 1; k >= 0; k--) {
    const int b = path[k];
    if (m.body_mocapid[b] >= 0) return PNP_ERR_UNSUPPORTED;
    double Rb[9], d[3];
    quat_to_mat(Rb, m.body_quat[b]);
    for (int r = 0; r < 3; r++) d[r] = R[3 * r] * m.body_pos[b][0] + R[3 * r + 1] * m.body_pos[b][1] + R[3 * r + 2] * m.body_pos[b][2];
    p[0] += d[0]; p[1] += d[1]; p[2] += d[2];
    mat_mul3(R, R, Rb);
    for (int j = m.body_jntadr[b]; j >= 0 && j < m.body_jntadr[b] + m.body_jntnum[b]; j++) {
      if (m.jnt_type[j] != 3 || j != nj || nj >= 7) return PNP_ERR_UNSUPPORTED;
      if (m.jnt_pos[j][0] != 0 || m.jnt_pos[j][1] != 0 || m.jnt_pos[j][2] != 0) return PNP_ERR_UNSUPPORTED;
      if (m.jnt_axis[j][0] != 0 || m.jnt_axis[j][1] != 0 || fabs(fabs(m.jnt_axis[j][2]) - 1) > 1e-12)
        return PNP_ERR_UNSUPPORTED;
      for (int t = 0; t < 9; t++) out->Rpre[nj][t] = R[t];
      for (int t = 0; t < 3; t++) out->ppre[nj][t] = p[t];
      out->sgn[nj] = m.jnt_axis[j][2] > 0 ? 1.0 : -1.0;
      out->lo[nj] = M->jnt_range[j][0];
      out->hi[nj] = M->jnt_range[j][1];
      out->qpos0[nj] = m.qpos0[m.jnt_qposadr[j]];
      nj++;
      // the next segment starts in this joint's (unrotated) body frame
      R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
      p[0] = p[1] = p[2] = 0;
    }
  }
  if (nj != 7) return PNP_ERR_UNSUPPORTED;
  for (int r = 0; r < 3; r++)
    out->psite[r] = p[r] + R[3 * r] * m.site_pos[site][0] + R[3 * r + 1] * m.site_pos[site][1] +
                    R[3 * r + 2] * m.site_pos[site][2];
  return PNP_OK;
}

// The baked kernel is used only when the runtime chain is the generated one (same site body,
// every constant within 1e-12); any other model/site runs the kernel-argument path.
static bool matches_baked(const IKSeg<double>& s, int site_body) {
  using namespace panda_chain;
  if (site_body != kSiteBody) return false;
  auto near = [](double a, double b) { return fabs(a - b) <= 1e-12; };
  for (int j = 0; j < 7; j++) {
    for (int t = 0; t < 9; t++) if (!near(s.Rpre[j][t], kRpre[j][t])) return false;
    for (int t = 0; t < 3; t++) if (!near(s.ppre[j][t], kPpre[j][t])) return false;
    if (!near(s.sgn[j], kSgn[j]) || !near(s.lo[j], kLo[j]) || !near(s.hi[j], kHi[j]) ||
        !near(s.qpos0[j], kQpos0[j]))
      return false;
  }
  for (int t = 0; t < 3; t++) if (!near(s.psite[t], kPsite[t])) return false;
  return true;
}

// PNP_IK_SERIAL=1: the thread-per-solve kernel (A/B runs); default: 8-lane groups
static bool serial_ik() {
  const char* e = getenv("PNP_IK_SERIAL");
  return e && e[0] == '1';
}

template <typename T>
static int32_t launch_ik(pnp_model* model, int32_t site, pnp_ik_params prm, const T* q_init,
                         const T* target, T* q_out, T* final_pos, T* pos_error, int32_t* iterations,
                         uint8_t* flags, int32_t B, void* stream) {
  if (!model || B < 0 || site < 0 || site >= model->h.nsite || prm.max_iters < 0) {
    pnp_set_error("pnp_ik_dls: bad argument (model=%p site=%d B=%d max_iters=%d)", (void*)model,
                  site, B, prm.max_iters);
    return PNP_ERR_ARG;
  }
  if (B == 0) return PNP_OK;
  if (!q_init || !target || !q_out || !final_pos || !pos_error || !iterations || !flags) {
    pnp_set_error("pnp_ik_dls: null buffer");
    return PNP_ERR_ARG;
  }
  IKSeg<double> s64;
  int32_t rc = build_segments(model, site, &s64);
  if (rc) {
    pnp_set_error("pnp_ik_dls: site %d is not below a 7-hinge +-z chain", site);
    return rc;
  }
  IKSeg<T> s;
  for (int j = 0; j < 7; j++) {
    for (int t = 0; t < 9; t++) s.Rpre[j][t] = (T)s64.Rpre[j][t];
    for (int t = 0; t < 3; t++) s.ppre[j][t] = (T)s64.ppre[j][t];
    s.sgn[j] = (T)s64.sgn[j];
    s.lo[j] = (T)s64.lo[j];
    s.hi[j] = (T)s64.hi[j];
    s.qpos0[j] = (T)s64.qpos0[j];
  }
  for (int t = 0; t < 3; t++) s.psite[t] = (T)s64.psite[t];
  if (serial_ik()) {
    const bool baked = matches_baked(s64, model->h.site_bodyid[site]);
    auto kern = baked ? ik_dls_kernel<T, true> : ik_dls_kernel<T, false>;
    hipLaunchKernelGGL(kern, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, s,
                       prm.max_iters, (T)prm.pos_thresh, (T)prm.damping, (T)prm.step_limit, q_init,
                       target, q_out, final_pos, pos_error, iterations, flags, B);
    return pnp_check_launch("ik_dls_kernel");
  }
  // one DPP row (16 lanes) per solve: 4 solves per 64-lane block
  hipLaunchKernelGGL(ik_dls_group_kernel<T>, dim3((B + 3) / 4), dim3(64), 0, (hipStream_t)stream, s,
                     prm.max_iters, (T)prm.pos_thresh, (T)prm.damping, (T)prm.step_limit, q_init, target,
                     q_out, final_pos, pos_error, iterations, flags, B);
  return pnp_check_launch("ik_dls_group_kernel");
}

extern "C" int32_t pnp_ik_dls(pnp_model* model, int32_t site_id, pnp_ik_params params,
                              const float* q_init, const float* target, float* q_out,
                              float* final_pos, float* pos_error, int32_t* iterations,
                              uint8_t* flags, int32_t B, void* stream) {
  return launch_ik<float>(model, site_id, params, q_init, target, q_out, final_pos, pos_error,
                          iterations, flags, B, stream);
}

extern "C" int32_t pnp_ik_dls_f64(pnp_model* model, int32_t site_id, pnp_ik_params params,
                                  const double* q_init, const double* target, double* q_out,
                                  double* final_pos, double* pos_error, int32_t* iterations,
                                  uint8_t* flags, int32_t B, void* stream) {
  return launch_ik<double>(model, site_id, params, q_init, target, q_out, final_pos, pos_error,
                           iterations, flags, B, stream);
}
