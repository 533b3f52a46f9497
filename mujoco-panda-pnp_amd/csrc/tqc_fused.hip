// tqc_fused.hip — one TQC gradient step (sb3-contrib tqc.py train(), the reference's learner in
// scripts/train.py:74-93) as four launches on the matrix cores, for C5 at train.py's update ratio.
//
// The PyTorch restatement (pnp_amd/tqc.py TQC._update) replays ~400 kernels per gradient step from
// a HIP graph: 512-row GEMMs of 256-wide layers, each a few microseconds, plus the elementwise and
// reduction kernels between them -- launch and latency bound (1.9 ms per step).  Here the batch is
// cut into slabs of 16 rows, one workgroup (4 waves) per slab, and each workgroup runs a whole
// network chain for its rows with v_mfma_f32_16x16x4_f32 tiles (fp32 in, fp32 accumulate: the
// precision of the PyTorch step); the per-slab weight gradients are reduced in a fixed order by
// the Adam kernels (deterministic):
//   K1 tqc_critic_kernel   per slab: actor(obs) -> a_pi, log_prob (kept for K2); actor(next_obs);
//                          target critics(next_obs, next_action) -> the 50 quantiles sorted, the top
//                          4 dropped, the TD target; critics(obs, action) and the quantile Huber
//                          loss; its backward pass through both critics -> per-slab gradients
//   K2 tqc_adam_kernel     critic Adam (+ Polyak update of the target critics), entropy Adam
//   K3 tqc_actor_kernel    per slab: critics(obs, a_pi) with the updated critics -> actor loss;
//                          backward through the critics (input gradient), the squashed Gaussian and
//                          the actor -> per-slab actor gradients
//   K4 tqc_adam_kernel     actor Adam
// The order is sb3-contrib's: entropy coefficient (its pre-update value in both losses), critic
// step, actor loss against the updated critics, Polyak.  Adam is torch.optim.Adam's fused /
// capturable update (per-parameter step tensors, incremented first; bias corrections from them),
// on the PyTorch optimisers' own state tensors, so the fused and the PyTorch steps interchange.
// Supported shape: train.py's -- obs 25 (achieved_goal, desired_goal, observation), action 7,
// [256, 256, 256] ReLU MLPs, 2 critics x 25 quantiles, batch a multiple of 16.
#include "pnp_internal.h"

#include <type_traits>

namespace {

constexpr int R = 16;              // rows per slab (one MFMA tile of rows)
constexpr int NW = 8;              // waves per workgroup (two per SIMD)
constexpr int NTH = 64 * NW;
constexpr int KC = 32;             // reduction rows per staged weight chunk
constexpr int OBS = 25, ACT = 7, HID = 256, NC = 2, NQ = 25, NIN = OBS + ACT, NALL = NC * NQ;
constexpr int LD = HID + 4;        // LDS row stride of the slab buffers (floats; = 4 mod 64: the A
                                   // operand's b128 reads and the row-permuted wgrad reads are
                                   // conflict-free)
constexpr int LDT = KC + 4;        // staged weight chunk, [column][reduction row] layout (CR)
constexpr int LDW = HID + 4;       // staged weight chunk, [reduction row][column] layout (RC)
constexpr int WCH = HID * LDT > KC * LDW ? HID * LDT : KC * LDW;   // one chunk buffer (floats)
constexpr float LOG_STD_MIN = -20.0f, LOG_STD_MAX = 2.0f, SQUASH_EPS = 1e-6f;
constexpr float HALF_LOG_2PI = 0.91893853320467274178f;

// per-slab workspace (floats): the actor's hidden activations and per-row values K3 needs, and
// the critics' hidden activations (K1 and K3 scratch)
constexpr int WS_H = R * HID;
constexpr int WS_ACTOR = 0;                       // 3 x [16][256]
constexpr int WS_CRIT = WS_ACTOR + 3 * WS_H;      // [2 critics][3][16][256]
constexpr int WS_ROW = WS_CRIT + NC * 3 * WS_H;   // a_pi, std, eps, log_std raw [16][7] each; log_prob [16]
constexpr int WS_SLAB = WS_ROW + 4 * R * ACT + R;

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- slab matrix products (X, Y, dY, dX: LDS [16][LD]; W: global, staged through LDS)
// acc = X[16][GK] B[GK][GN]: B(r, c) (r the reduction index, c the output column) is the weight
// element W[c * GK + r] (CR: contiguous in r) or W[r * GN + c] (RC).  The weight streams through
// two LDS chunk buffers of KC reduction rows, stored [c][r] (stride LDT) for CR and [r][c] (stride
// LDW) for RC so that the global fetches are float4 and coalesced: every thread fetches its share
// of chunk ch + 1 into registers while the waves run chunk ch's MFMAs from LDS, then stores it and
// the workgroup syncs -- the MFMA chains never wait on a global load.  Wave w owns the output
// tiles w and w + NW (16 columns each; every MFMA runs with the whole wave).
// The reduction index is permuted within each block of 16: at step s lane (kq = lane / 16, i)
// supplies A[i][16 kb + 4 kq + s] and B[16 kb + 4 kq + s][c] -- one b128 LDS read of A per four
// MFMAs (and of B in the CR layout); the sum is the same, the fp32 accumulation order differs.
// Reduction rows past GK read zeros from the staged chunk and are masked in A; columns past GN
// compute garbage in output columns nobody keeps.  Every thread of the workgroup must call it.
template <bool CR, int GK, int GN>
__device__ void slab_gemm(const float* X, const float* __restrict__ W, float* Ws, f32x4 acc[2]) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, i = lane & 15, kq = lane >> 4;
  constexpr int NTILE = (GN + 15) / 16, NCH = (GK + KC - 1) / KC;
  constexpr int LDG = CR ? GK : GN;                          // global row stride
  constexpr bool VEC = LDG % 4 == 0;
  constexpr int NUNIT = VEC ? KC * GN / 4 : KC * GN;          // float4 (or float) units per chunk
  constexpr int PER = (NUNIT + NTH - 1) / NTH;
  static_assert(NTILE <= 2 * NW && (CR ? GN * LDT : KC * LDW) <= WCH, "slab_gemm shape");
  acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  using U = typename std::conditional<VEC, f32x4, float>::type;
  U pre[PER];
  // unit u of chunk ch: its global address, its LDS slot, whether it lies inside the matrix
  auto unit = [&](int u, int ch, const float*& src, int& dst, bool& in) {
    if (VEC) {
      if (CR) {
        const int c = u / (KC / 4), j = u % (KC / 4), r = ch * KC + 4 * j;
        src = W + (size_t)c * LDG + r; dst = c * LDT + 4 * j; in = r < GK;
      } else {
        const int rr = u / (GN / 4), j = u % (GN / 4), r = ch * KC + rr;
        src = W + (size_t)r * LDG + 4 * j; dst = rr * LDW + 4 * j; in = r < GK;
      }
    } else {
      if (CR) {
        const int c = u / KC, rr = u % KC, r = ch * KC + rr;
        src = W + (size_t)c * LDG + r; dst = c * LDT + rr; in = r < GK;
      } else {
        const int rr = u / GN, c = u % GN, r = ch * KC + rr;
        src = W + (size_t)r * LDG + c; dst = rr * LDW + c; in = r < GK;
      }
    }
  };
  auto fetch = [&](int ch) {
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int u = t + j * NTH;
      const float* src; int dst; bool in;
      unit(u, ch, src, dst, in);
      pre[j] = U{};
      if (u < NUNIT && in) pre[j] = *reinterpret_cast<const U*>(src);
    }
  };
  auto put = [&](int buf, int ch) {
    float* D = Ws + buf * WCH;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int u = t + j * NTH;
      const float* src; int dst; bool in;
      unit(u, ch, src, dst, in);
      if (u < NUNIT) *reinterpret_cast<U*>(D + dst) = pre[j];
    }
  };
  fetch(0);
  put(0, 0);
  __syncthreads();
  for (int ch = 0; ch < NCH; ch++) {
    if (ch + 1 < NCH) fetch(ch + 1);
    const float* D = Ws + (ch & 1) * WCH;
#pragma unroll
    for (int kb = 0; kb < KC; kb += 16) {
      const int k0 = kb + 4 * kq, k = ch * KC + k0;
      f32x4 a = *reinterpret_cast<const f32x4*>(X + i * LD + k);
      if (GK % KC != 0)
#pragma unroll
        for (int s = 0; s < 4; s++) a[s] = k + s < GK ? a[s] : 0.f;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int tile = wv + q * NW;
        if (tile < NTILE) {
          const int c = tile * 16 + i;
          f32x4 b;
          if (CR) {
            b = *reinterpret_cast<const f32x4*>(D + c * LDT + k0);
          } else {
#pragma unroll
            for (int s = 0; s < 4; s++) b[s] = D[(k0 + s) * LDW + c];
          }
#pragma unroll
          for (int s = 0; s < 4; s++) acc[q] = mfma4(a[s], b[s], acc[q]);
        }
      }
    }
    if (ch + 1 < NCH) put((ch + 1) & 1, ch + 1);
    __syncthreads();
  }
}
// Y = act(X Wk + b) with Wk(k, n) from nn.Linear's [out][in] (TR: CR view) or the stacked critics'
// [in][out] (RC view)
template <bool TR, int K, int N>
__device__ __attribute__((noinline)) void lin_fwd(const float* X, const float* __restrict__ W, const float* __restrict__ bias,
                                                  float* Y, bool relu, float* Ws) {
  f32x4 acc[2];
  slab_gemm<TR, K, N>(X, W, Ws, acc);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int n = (wv + q * NW) * 16 + i;
    if (n < N) {
      const float bn = bias[n];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float v = bn + acc[q][r];
        Y[(4 * kq + r) * LD + n] = relu ? fmaxf(v, 0.f) : v;
      }
    }
  }
}
// dX[16][K] (+)= dY[16][N] Wk^T, masked by relu'(H) (H: the layer input's post-ReLU activation,
// or null).  Wk as in lin_fwd: the reduction runs over the layer's outputs n, B(n, k) = Wk(k, n)
// -- nn.Linear [out][in]: W[n * K + k] (RC view); critics [in][out]: W[k * N + n] (CR view)
template <bool TR, int N, int K>
__device__ __attribute__((noinline)) void lin_dgrad(const float* dY, const float* __restrict__ W, float* dX, const float* H,
                                                    bool accumulate, float* Ws) {
  f32x4 acc[2];
  slab_gemm<!TR, N, K>(dY, W, Ws, acc);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int k = (wv + q * NW) * 16 + i;
    if (k < K)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 4 * kq + r;
        float v = acc[q][r];
        if (accumulate) v += dX[row * LD + k];
        if (H && !(H[row * LD + k] > 0.f)) v = 0.f;
        dX[row * LD + k] = v;
      }
  }
}
// per-slab weight gradient P(k, n) = sum over the 16 rows of X[r][k] dY[r][n] (P in Wk's storage
// layout) and the bias gradient Pb[n] = sum_r dY[r][n].  Rows permuted as in slab_gemm (step s,
// lane kq: row 4 kq + s): the b32 reads of X and dY are then conflict-free with LD = 4 mod 64.
template <bool TR, int K, int N>
__device__ __attribute__((noinline)) void lin_wgrad(const float* X, const float* dY, float* __restrict__ P, float* __restrict__ Pb) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, i = lane & 15, kq = lane >> 4;
  constexpr int tk = (K + 15) >> 4, tn = (N + 15) >> 4, nt = tk * tn;
  for (int t0 = wv * 4; t0 < nt; t0 += 4 * NW) {
    f32x4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; q++) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int r = 4 * kq + s;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int t = t0 + q;
        if (t < nt) {
          const int k = (t / tn) * 16 + i, n = (t % tn) * 16 + i;
          const float a = k < K ? X[r * LD + k] : 0.f;
          const float b = n < N ? dY[r * LD + n] : 0.f;
          acc[q] = mfma4(a, b, acc[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int t = t0 + q;
      if (t < nt) {
        const int n = (t % tn) * 16 + i;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int k = (t / tn) * 16 + 4 * kq + r;
          if (k < K && n < N) P[TR ? (size_t)n * K + k : (size_t)k * N + n] = acc[q][r];
        }
      }
    }
  }
  for (int n = threadIdx.x; n < N; n += NTH) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < R; r++) s += dY[r * LD + n];
    Pb[n] = s;
  }
}

// global <-> LDS slab copies (save/load: float4 both sides)
template <int COLS>
__device__ void load_rows(float* D, const float* __restrict__ src, int row0, int ld_src, int col0 = 0) {
  for (int e = threadIdx.x; e < R * COLS; e += NTH) {
    const int r = e / COLS, c = e - r * COLS;
    D[r * LD + col0 + c] = src[(size_t)(row0 + r) * ld_src + c];
  }
}
template <int COLS>
__device__ void save_slab(float* __restrict__ dst, const float* S) {
  static_assert(COLS % 4 == 0, "save_slab");
  for (int e = threadIdx.x; e < R * COLS / 4; e += NTH) {
    const int r = e / (COLS / 4), c = 4 * (e - r * (COLS / 4));
    *reinterpret_cast<f32x4*>(dst + 4 * e) = *reinterpret_cast<const f32x4*>(S + r * LD + c);
  }
}
template <int COLS>
__device__ void load_slab(float* D, const float* __restrict__ src) {
  static_assert(COLS % 4 == 0, "load_slab");
  for (int e = threadIdx.x; e < R * COLS / 4; e += NTH) {
    const int r = e / (COLS / 4), c = 4 * (e - r * (COLS / 4));
    *reinterpret_cast<f32x4*>(D + r * LD + c) = *reinterpret_cast<const f32x4*>(src + 4 * e);
  }
}

struct TqcArgs {
  const float* actor[10];    // W0 b0 W1 b1 W2 b2 Wmu bmu Wls bls (nn.Linear: W [out][in])
  const float* critic[8];    // w0 b0 .. w3 b3 ([n_critics][in][out], [n_critics][1][out])
  const float* target[8];
  const float* obs; const float* act; const float* nobs; const float* done; const float* rew;
  const float* eps_pi; const float* eps_next;
  const float* log_ent_coef;
  float* ws;                 // [slabs][WS_SLAB]
  float* part_c;             // [slabs][critic params]
  float* part_a;             // [slabs][actor params]
  float* part_s;             // [slabs][4]: critic loss sum, sum(log_prob + target entropy), actor loss sum
  float* logs;               // [4]: ent_coef (pre-update), critic loss, actor loss, entropy-coefficient loss
  float gamma, target_entropy;
  int B;
};
// critic parameter offsets (per tensor, both critics) in the flat critic gradient vector; actor
// likewise
__host__ __device__ constexpr int crit_size(int t) {
  return t == 0 ? NC * NIN * HID : t == 2 || t == 4 ? NC * HID * HID : t == 6 ? NC * HID * NQ : t == 7 ? NC * NQ : NC * HID;
}
__host__ __device__ constexpr int crit_off(int t) { return t == 0 ? 0 : crit_off(t - 1) + crit_size(t - 1); }
constexpr int CRIT_P = crit_off(8);
__host__ __device__ constexpr int act_size(int t) {
  return t == 0 ? HID * OBS : t == 2 || t == 4 ? HID * HID : t == 6 || t == 8 ? ACT * HID : t == 7 || t == 9 ? ACT : HID;
}
__host__ __device__ constexpr int act_off(int t) { return t == 0 ? 0 : act_off(t - 1) + act_size(t - 1); }
constexpr int ACT_P = act_off(10);

struct alignas(16) Lds {   // 136 KB (a workgroup may hold all 160 KB of a CU's LDS)
  float A[R * LD], Bf[R * LD], C[R * LD];
  float W[2 * WCH];
  float row[R][NALL + 14], q[R][NALL], tq[R][NALL];
  float red[NTH];
};

// the actor's forward pass on the slab's rows of x (LDS A): a = tanh(mu + std eps), log_prob;
// hidden activations saved to hs (or not, null); leaves a in aout[16][7] (LDS), log_prob in lpo[16]
__device__ void actor_fwd(Lds& L, const TqcArgs& g, const float* __restrict__ eps, int row0, float* hs, float (*aout)[8],
                          float* lpo, float* row_ws) {
  const float* const* P = g.actor;
  lin_fwd<true, OBS, HID>(L.A, P[0], P[1], L.Bf, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs, L.Bf);
  lin_fwd<true, HID, HID>(L.Bf, P[2], P[3], L.C, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs + WS_H, L.C);
  lin_fwd<true, HID, HID>(L.C, P[4], P[5], L.Bf, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs + 2 * WS_H, L.Bf);
  // heads: mu and log_std into C's first 16 columns (N = 7 each)
  lin_fwd<true, HID, ACT>(L.Bf, P[6], P[7], L.C, false, L.W);
  lin_fwd<true, HID, ACT>(L.Bf, P[8], P[9], L.C + 8, false, L.W);
  __syncthreads();
  const int t = threadIdx.x;
  if (t < R * ACT) {
    const int r = t / ACT, j = t - r * ACT;
    const float mu = L.C[r * LD + j], lsr = L.C[r * LD + 8 + j];
    const float ls = fminf(fmaxf(lsr, LOG_STD_MIN), LOG_STD_MAX);
    const float sd = expf(ls), e = eps[(size_t)(row0 + r) * ACT + j];
    const float a = tanhf(mu + sd * e);
    aout[r][j] = a;
    L.row[r][j] = -0.5f * e * e - ls - HALF_LOG_2PI;
    L.row[r][7 + j] = logf(1.f - a * a + SQUASH_EPS);
    if (row_ws) {
      row_ws[t] = a;                     // a_pi
      row_ws[R * ACT + t] = sd;          // std
      row_ws[2 * R * ACT + t] = e;       // eps
      row_ws[3 * R * ACT + t] = lsr;     // raw log_std (the clamp's gradient mask)
    }
  }
  __syncthreads();
  if (t < R) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < ACT; j++) { s1 += L.row[t][j]; s2 += L.row[t][7 + j]; }
    lpo[t] = s1 - s2;
    if (row_ws) row_ws[4 * R * ACT + t] = s1 - s2;
  }
  __syncthreads();
}

// one critic network c on x (LDS A, 32 columns) -> q[16][25] into out (LDS, row stride NALL,
// column offset c * 25); hidden activations saved to hs (or not)
__device__ void critic_fwd(Lds& L, const float* const* P, int c, float* hs, float* out) {
  const float* w0 = P[0] + (size_t)c * NIN * HID;
  const float* w1 = P[2] + (size_t)c * HID * HID;
  const float* w2 = P[4] + (size_t)c * HID * HID;
  const float* w3 = P[6] + (size_t)c * HID * NQ;
  lin_fwd<false, NIN, HID>(L.A, w0, P[1] + c * HID, L.Bf, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs, L.Bf);
  lin_fwd<false, HID, HID>(L.Bf, w1, P[3] + c * HID, L.C, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs + WS_H, L.C);
  lin_fwd<false, HID, HID>(L.C, w2, P[5] + c * HID, L.Bf, true, L.W);
  __syncthreads();
  if (hs) save_slab<HID>(hs + 2 * WS_H, L.Bf);
  lin_fwd<false, HID, NQ>(L.Bf, w3, P[7] + c * NQ, L.C, false, L.W);
  __syncthreads();
  for (int e = threadIdx.x; e < R * NQ; e += NTH) {
    const int r = e / NQ, j = e - r * NQ;
    out[r * NALL + c * NQ + j] = L.C[r * LD + j];
  }
  __syncthreads();
}
// backward through critic c from dq (LDS C, [16][25]) with its saved activations hs and input x
// (global rows, re-staged): weight gradients into pw (the slab's critic gradient vector) when
// non-null; the input gradient d x (32 columns) left in L.A when want_dx
__device__ void critic_bwd(Lds& L, const float* const* P, int c, const float* hs, float* pw, bool want_dx,
                           const TqcArgs& g, int row0, bool x_is_pi, float (*api)[8]) {
  const float* w1 = P[2] + (size_t)c * HID * HID;
  const float* w2 = P[4] + (size_t)c * HID * HID;
  const float* w3 = P[6] + (size_t)c * HID * NQ;
  // layer 3 (linear): dq in C; H3 -> A
  load_slab<HID>(L.A, hs + 2 * WS_H);
  __syncthreads();
  if (pw) lin_wgrad<false, HID, NQ>(L.A, L.C, pw + crit_off(6) + c * HID * NQ, pw + crit_off(7) + c * NQ);
  lin_dgrad<false, NQ, HID>(L.C, w3, L.Bf, L.A, false, L.W);   // dH3 = dq w3^T, relu'(H3)
  __syncthreads();
  // layer 2: dY = dH3 (Bf), X = H2 -> A
  load_slab<HID>(L.A, hs + WS_H);
  __syncthreads();
  if (pw) lin_wgrad<false, HID, HID>(L.A, L.Bf, pw + crit_off(4) + c * HID * HID, pw + crit_off(5) + c * HID);
  lin_dgrad<false, HID, HID>(L.Bf, w2, L.C, L.A, false, L.W);   // dH2
  __syncthreads();
  // layer 1: dY = dH2 (C), X = H1 -> A
  load_slab<HID>(L.A, hs);
  __syncthreads();
  if (pw) lin_wgrad<false, HID, HID>(L.A, L.C, pw + crit_off(2) + c * HID * HID, pw + crit_off(3) + c * HID);
  lin_dgrad<false, HID, HID>(L.C, w1, L.Bf, L.A, false, L.W);   // dH1
  __syncthreads();
  // layer 0: dY = dH1 (Bf), X = [obs, action] -> A
  load_rows<OBS>(L.A, g.obs, row0, OBS);
  if (x_is_pi) {
    for (int e = threadIdx.x; e < R * ACT; e += NTH) L.A[(e / ACT) * LD + OBS + e % ACT] = api[e / ACT][e % ACT];
  } else {
    load_rows<ACT>(L.A, g.act, row0, ACT, OBS);
  }
  __syncthreads();
  if (pw) lin_wgrad<false, NIN, HID>(L.A, L.Bf, pw + crit_off(0) + c * NIN * HID, pw + crit_off(1) + c * HID);
  __syncthreads();
  if (want_dx) {
    lin_dgrad<false, HID, NIN>(L.Bf, P[0] + (size_t)c * NIN * HID, L.A, nullptr, false, L.W);
    __syncthreads();
  }
}

// block sum of v (all threads), result on every thread
__device__ float block_sum(Lds& L, float v) {
  L.red[threadIdx.x] = v;
  __syncthreads();
  for (int s = NTH / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) L.red[threadIdx.x] += L.red[threadIdx.x + s];
    __syncthreads();
  }
  const float r = L.red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(NTH) tqc_critic_kernel(TqcArgs g) {
  __shared__ Lds L;
  const int slab = blockIdx.x, row0 = slab * R, t = threadIdx.x;
  float* ws = g.ws + (size_t)slab * WS_SLAB;
  float* pw = g.part_c + (size_t)slab * CRIT_P;
  const float ent_coef = expf(g.log_ent_coef[0]);
  // actor(obs): a_pi, log_prob (kept for the actor step)
  __shared__ float api[R][8], lp[R], na[R][8], nlp[R];
  load_rows<OBS>(L.A, g.obs, row0, OBS);
  __syncthreads();
  actor_fwd(L, g, g.eps_pi, row0, ws + WS_ACTOR, api, lp, ws + WS_ROW);
  // actor(next_obs): next action and its log_prob
  load_rows<OBS>(L.A, g.nobs, row0, OBS);
  __syncthreads();
  actor_fwd(L, g, g.eps_next, row0, nullptr, na, nlp, nullptr);
  // target critics on (next_obs, next_action)
  for (int c = 0; c < NC; c++) {
    load_rows<OBS>(L.A, g.nobs, row0, OBS);
    for (int e = t; e < R * ACT; e += NTH) L.A[(e / ACT) * LD + OBS + e % ACT] = na[e / ACT][e % ACT];
    __syncthreads();
    critic_fwd(L, g.target, c, nullptr, &L.q[0][0]);
  }
  // sort the 50 target quantiles per row (rank by counting; ties broken by index), keep the
  // lowest 46, TD target
  for (int e = t; e < R * NALL; e += NTH) {
    const int r = e / NALL, j = e - r * NALL;
    const float v = L.q[r][j];
    int rank = 0;
    for (int i = 0; i < NALL; i++) {
      const float u = L.q[r][i];
      rank += (u < v || (u == v && i < j)) ? 1 : 0;
    }
    L.row[r][rank] = v;
  }
  __syncthreads();
  constexpr int KEEP = NALL - 2 * NC;
  for (int e = t; e < R * KEEP; e += NTH) {
    const int r = e / KEEP, j = e - r * KEEP;
    const float d = g.done[row0 + r], rw = g.rew[row0 + r];
    const float tq = L.row[r][j] - ent_coef * nlp[r];
    L.tq[r][j] = rw + (1.f - d) * g.gamma * tq;
  }
  __syncthreads();
  // critics on (obs, action), activations saved
  for (int c = 0; c < NC; c++) {
    load_rows<OBS>(L.A, g.obs, row0, OBS);
    load_rows<ACT>(L.A, g.act, row0, ACT, OBS);
    __syncthreads();
    critic_fwd(L, g.critic, c, ws + WS_CRIT + c * 3 * WS_H, &L.q[0][0]);
  }
  // quantile Huber loss (mean over rows x critics x quantiles x targets) and its gradient dq
  const float scale = 1.f / ((float)g.B * NC * NQ * KEEP);
  float lsum = 0.f;
  for (int e = t; e < R * NALL; e += NTH) {
    const int r = e / NALL, ci = e - r * NALL, i = ci % NQ;
    const float cq = L.q[r][ci], tau = ((float)i + 0.5f) / NQ;
    float gsum = 0.f;
    for (int j = 0; j < KEEP; j++) {
      const float d = L.tq[r][j] - cq, ad = fabsf(d);
      const float w = fabsf(tau - (d < 0.f ? 1.f : 0.f));
      lsum += w * (ad > 1.f ? ad - 0.5f : 0.5f * d * d);
      gsum += w * (ad > 1.f ? (d > 0.f ? 1.f : -1.f) : d);
    }
    L.row[r][ci] = -gsum * scale;   // dL / dq
  }
  lsum = block_sum(L, lsum);
  // per-row log_prob + target entropy (entropy-coefficient gradient)
  const float esum = block_sum(L, t < R ? lp[t] + g.target_entropy : 0.f);
  if (t == 0) {
    g.part_s[slab * 4 + 0] = lsum;
    g.part_s[slab * 4 + 1] = esum;
  }
  // backward through each critic: weight gradients
  for (int c = 0; c < NC; c++) {
    for (int e = t; e < R * NQ; e += NTH) L.C[(e / NQ) * LD + e % NQ] = L.row[e / NQ][c * NQ + e % NQ];
    __syncthreads();
    critic_bwd(L, g.critic, c, ws + WS_CRIT + c * 3 * WS_H, pw, false, g, row0, false, nullptr);
  }
}

__global__ void __launch_bounds__(NTH) tqc_actor_kernel(TqcArgs g) {
  __shared__ Lds L;
  const int slab = blockIdx.x, row0 = slab * R, t = threadIdx.x;
  const float* ws = g.ws + (size_t)slab * WS_SLAB;
  float* pw = g.part_a + (size_t)slab * ACT_P;
  const float ent_coef = g.logs[0];   // sb3: the coefficient before this step's entropy update
  __shared__ float api[R][8], dap[R][8];
  const float* rw = ws + WS_ROW;
  for (int e = t; e < R * ACT; e += NTH) { api[e / ACT][e % ACT] = rw[e]; dap[e / ACT][e % ACT] = 0.f; }
  __syncthreads();
  // critics (updated) on (obs, a_pi): q_pi, then d loss / d a_pi through both critics
  float qsum = 0.f;
  for (int c = 0; c < NC; c++) {
    load_rows<OBS>(L.A, g.obs, row0, OBS);
    for (int e = t; e < R * ACT; e += NTH) L.A[(e / ACT) * LD + OBS + e % ACT] = api[e / ACT][e % ACT];
    __syncthreads();
    float* hs = g.ws + (size_t)slab * WS_SLAB + WS_CRIT + c * 3 * WS_H;
    critic_fwd(L, g.critic, c, hs, &L.q[0][0]);
    for (int e = t; e < R * NQ; e += NTH) qsum += L.q[e / NQ][c * NQ + e % NQ];
    // actor loss = mean_rows(ent_coef log_prob - mean_{c,q} q): d / dq = -1 / (B NC NQ)
    const float dq = -1.f / ((float)g.B * NC * NQ);
    for (int e = t; e < R * NQ; e += NTH) L.C[(e / NQ) * LD + e % NQ] = dq;
    __syncthreads();
    critic_bwd(L, g.critic, c, hs, nullptr, true, g, row0, true, api);
    for (int e = t; e < R * ACT; e += NTH) dap[e / ACT][e % ACT] += L.A[(e / ACT) * LD + OBS + e % ACT];
    __syncthreads();
  }
  const float lpsum = block_sum(L, t < R ? rw[4 * R * ACT + t] : 0.f);
  qsum = block_sum(L, qsum);
  if (t == 0) g.part_s[slab * 4 + 2] = ent_coef * lpsum - qsum / (NC * NQ);
  // the squashed Gaussian: a = tanh(mu + std eps), std = exp(clamp(log_std)),
  // log_prob = sum(-eps^2 / 2 - log_std - log(2 pi) / 2) - sum(log(1 - a^2 + 1e-6))
  const float dlp = ent_coef / (float)g.B;
  if (t < R * ACT) {
    const int r = t / ACT, j = t - r * ACT;
    const float a = rw[t], sd = rw[R * ACT + t], e = rw[2 * R * ACT + t], lsr = rw[3 * R * ACT + t];
    const float da = dap[r][j] + dlp * (2.f * a / (1.f - a * a + SQUASH_EPS));
    const float dgg = da * (1.f - a * a);
    const bool inside = lsr >= LOG_STD_MIN && lsr <= LOG_STD_MAX;
    L.C[r * LD + j] = dgg;                                       // d mu
    L.C[r * LD + 8 + j] = inside ? dgg * sd * e - dlp : 0.f;     // d log_std (raw)
  }
  __syncthreads();
  const float* const* P = g.actor;
  // heads: X = H3 (A), dY = d mu / d log_std (C columns 0.. / 8..)
  load_slab<HID>(L.A, ws + WS_ACTOR + 2 * WS_H);
  for (int e = t; e < R * 8; e += NTH) { L.Bf[(e / 8) * LD + e % 8] = L.C[(e / 8) * LD + 8 + e % 8]; }
  __syncthreads();
  lin_wgrad<true, HID, ACT>(L.A, L.C, pw + act_off(6), pw + act_off(7));
  lin_wgrad<true, HID, ACT>(L.A, L.Bf, pw + act_off(8), pw + act_off(9));
  __syncthreads();
  // d H3 = dmu Wmu + dls Wls, relu'(H3): into the free buffer (C's columns > 15 are unused:
  // stage d mu in Bf's high columns first)
  for (int e = t; e < R * 8; e += NTH) L.Bf[(e / 8) * LD + 16 + e % 8] = L.C[(e / 8) * LD + e % 8];
  __syncthreads();
  lin_dgrad<true, ACT, HID>(L.Bf + 16, P[6], L.C, nullptr, false, L.W);
  __syncthreads();
  lin_dgrad<true, ACT, HID>(L.Bf, P[8], L.C, L.A, true, L.W);
  __syncthreads();
  // layer 2: X = H2, dY = dH3 (C)
  load_slab<HID>(L.A, ws + WS_ACTOR + WS_H);
  __syncthreads();
  lin_wgrad<true, HID, HID>(L.A, L.C, pw + act_off(4), pw + act_off(5));
  lin_dgrad<true, HID, HID>(L.C, P[4], L.Bf, L.A, false, L.W);
  __syncthreads();
  // layer 1: X = H1, dY = dH2 (Bf)
  load_slab<HID>(L.A, ws + WS_ACTOR);
  __syncthreads();
  lin_wgrad<true, HID, HID>(L.A, L.Bf, pw + act_off(2), pw + act_off(3));
  lin_dgrad<true, HID, HID>(L.Bf, P[2], L.C, L.A, false, L.W);
  __syncthreads();
  // layer 0: X = obs, dY = dH1 (C)
  load_rows<OBS>(L.A, g.obs, row0, OBS);
  __syncthreads();
  lin_wgrad<true, OBS, HID>(L.A, L.C, pw + act_off(0), pw + act_off(1));
}

// ---- reduction of the per-slab gradients + Adam (torch.optim.Adam fused / capturable semantics)
struct AdamArgs {
  float* p[10]; float* m[10]; float* v[10]; float* tgt[10]; float* step[10];
  int off[11];               // flat offsets (off[nt] = total)
  int nt;
  const float* part; int nparts; int stride;   // per-slab gradient vectors
  const float* lr;
  float beta1, beta2, eps, tau;
  float* grad_out;           // optional: the reduced gradients (tests)
  // entropy coefficient (the critic pass): log_ent_coef, its Adam state, the gradient's source
  float* ent; float* ent_m; float* ent_v; float* ent_step;
  const float* part_s; int nslab; float target_entropy; int B;
  float* logs; float critic_scale;
};
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float gr, float lr, float b1, float b2, float eps,
                                          float step) {
  const float bc1 = 1.f - powf(b1, step), bc2 = 1.f - powf(b2, step);
  m = b1 * m + (1.f - b1) * gr;
  v = b2 * v + (1.f - b2) * gr * gr;
  const float denom = sqrtf(v) / sqrtf(bc2) + eps;
  p -= (lr / bc1) * m / denom;
}
__global__ void tqc_adam_kernel(AdamArgs a) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const float lr = a.lr[0];
  if (e < a.off[a.nt]) {
    int ti = 0;
    while (ti + 1 < a.nt && e >= a.off[ti + 1]) ti++;
    const int k = e - a.off[ti];
    float gr = 0.f;
    for (int s = 0; s < a.nparts; s++) gr += a.part[(size_t)s * a.stride + e];
    if (a.grad_out) a.grad_out[e] = gr;
    const float step = a.step[ti][0] + 1.f;
    float p = a.p[ti][k], m = a.m[ti][k], v = a.v[ti][k];
    adam_elem(p, m, v, gr, lr, a.beta1, a.beta2, a.eps, step);
    a.p[ti][k] = p; a.m[ti][k] = m; a.v[ti][k] = v;
    if (a.tgt[ti]) {   // Polyak (torch._foreach_mul_ then _foreach_add_ with alpha = tau)
      const float t1 = a.tgt[ti][k] * (1.f - a.tau);
      a.tgt[ti][k] = t1 + a.tau * p;
    }
  }
  if (a.ent && e == 0) {   // entropy coefficient: loss = -(log_ent_coef * mean(log_prob + target)).mean()
    float s = 0.f, l = 0.f;
    for (int i = 0; i < a.nslab; i++) { s += a.part_s[i * 4 + 1]; l += a.part_s[i * 4 + 0]; }
    const float mean = s / (float)a.B;
    const float le = a.ent[0];
    a.logs[0] = expf(le);
    a.logs[1] = l * a.critic_scale;
    a.logs[3] = -(le * mean);
    float p = le, m = a.ent_m[0], v = a.ent_v[0];
    const float step = a.ent_step[0] + 1.f;
    adam_elem(p, m, v, -mean, lr, a.beta1, a.beta2, a.eps, step);
    a.ent[0] = p; a.ent_m[0] = m; a.ent_v[0] = v;
  }
  if (!a.ent && a.logs && e == 0) {
    float s = 0.f;
    for (int i = 0; i < a.nslab; i++) s += a.part_s[i * 4 + 2];
    a.logs[2] = s / (float)a.B;
  }
}
// the optimisers' step tensors, after their update (torch increments every parameter's own)
__global__ void tqc_step_inc(AdamArgs a) {
  const int t = threadIdx.x;
  if (t < a.nt) a.step[t][0] += 1.f;
  if (t == 0 && a.ent_step) a.ent_step[0] += 1.f;
}

}  // namespace

// ---------------------------------------------------------------------------------- C ABI
static bool tqc_shape_ok(const pnp_tqc_desc* d) {
  return d && d->batch > 0 && d->batch % R == 0 && d->obs_dim == OBS && d->act_dim == ACT && d->hidden == HID &&
         d->n_critics == NC && d->n_quantiles == NQ && d->n_drop_per_net == 2;
}
static bool tqc_desc_ok(const pnp_tqc_desc* d) {
  if (!tqc_shape_ok(d) || !d->lr || !d->log_ent_coef) return false;
  for (int i = 0; i < 10; i++)
    if (!d->actor[i] || !d->actor_m[i] || !d->actor_v[i] || !d->actor_step[i]) return false;
  for (int i = 0; i < 8; i++)
    if (!d->critic[i] || !d->critic_m[i] || !d->critic_v[i] || !d->critic_step[i] || !d->target[i]) return false;
  return d->ent_m && d->ent_v && d->ent_step && d->workspace && d->logs;
}

extern "C" int64_t pnp_tqc_workspace_floats(const pnp_tqc_desc* d) {
  if (!tqc_shape_ok(d)) { pnp_set_error("pnp_tqc_workspace_floats: unsupported TQC shape"); return PNP_ERR_UNSUPPORTED; }
  const int64_t S = d->batch / R;
  return S * ((int64_t)WS_SLAB + CRIT_P + ACT_P + 4);
}
extern "C" int32_t pnp_tqc_param_counts(int32_t* actor_params, int32_t* critic_params) {
  if (!actor_params || !critic_params) { pnp_set_error("pnp_tqc_param_counts: null"); return PNP_ERR_ARG; }
  *actor_params = ACT_P;
  *critic_params = CRIT_P;
  return PNP_OK;
}

extern "C" int32_t pnp_tqc_update(const pnp_tqc_desc* d, const pnp_tqc_batch* b, float* grads_out, void* stream) {
  if (!tqc_desc_ok(d)) { pnp_set_error("pnp_tqc_update: unsupported TQC shape or null pointer"); return PNP_ERR_UNSUPPORTED; }
  if (!b || !b->obs || !b->act || !b->next_obs || !b->done || !b->reward || !b->eps_pi || !b->eps_next) {
    pnp_set_error("pnp_tqc_update: null batch buffer");
    return PNP_ERR_ARG;
  }
  const int S = d->batch / R;
  if (d->workspace_floats < (int64_t)S * (WS_SLAB + CRIT_P + ACT_P + 4)) {
    pnp_set_error("pnp_tqc_update: workspace too small");
    return PNP_ERR_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  TqcArgs g{};
  for (int i = 0; i < 10; i++) g.actor[i] = d->actor[i];
  for (int i = 0; i < 8; i++) { g.critic[i] = d->critic[i]; g.target[i] = d->target[i]; }
  g.obs = b->obs; g.act = b->act; g.nobs = b->next_obs; g.done = b->done; g.rew = b->reward;
  g.eps_pi = b->eps_pi; g.eps_next = b->eps_next;
  g.log_ent_coef = d->log_ent_coef;
  g.ws = d->workspace;
  g.part_c = g.ws + (size_t)S * WS_SLAB;
  g.part_a = g.part_c + (size_t)S * CRIT_P;
  g.part_s = g.part_a + (size_t)S * ACT_P;
  g.logs = d->logs;
  g.gamma = d->gamma;
  g.target_entropy = d->target_entropy;
  g.B = d->batch;
  hipLaunchKernelGGL(tqc_critic_kernel, dim3(S), dim3(NTH), 0, st, g);
  if (const int32_t rc = pnp_check_launch("tqc_critic_kernel")) return rc;
  AdamArgs ac{};
  for (int i = 0; i < 8; i++) {
    ac.p[i] = d->critic[i]; ac.m[i] = d->critic_m[i]; ac.v[i] = d->critic_v[i]; ac.tgt[i] = d->target[i];
    ac.step[i] = d->critic_step[i]; ac.off[i] = crit_off(i);
  }
  ac.off[8] = CRIT_P; ac.nt = 8;
  ac.part = g.part_c; ac.nparts = S; ac.stride = CRIT_P;
  ac.lr = d->lr; ac.beta1 = d->beta1; ac.beta2 = d->beta2; ac.eps = d->adam_eps; ac.tau = d->tau;
  ac.grad_out = grads_out ? grads_out + ACT_P : nullptr;
  ac.ent = d->log_ent_coef; ac.ent_m = d->ent_m; ac.ent_v = d->ent_v; ac.ent_step = d->ent_step;
  ac.part_s = g.part_s; ac.nslab = S; ac.target_entropy = d->target_entropy; ac.B = d->batch; ac.logs = d->logs;
  ac.critic_scale = 1.f / ((float)d->batch * NC * NQ * (NALL - 2 * NC));
  hipLaunchKernelGGL(tqc_adam_kernel, dim3((CRIT_P + 255) / 256), dim3(256), 0, st, ac);
  if (const int32_t rc = pnp_check_launch("tqc_adam_kernel (critics)")) return rc;
  hipLaunchKernelGGL(tqc_step_inc, dim3(1), dim3(64), 0, st, ac);
  if (const int32_t rc = pnp_check_launch("tqc_step_inc (critics)")) return rc;
  hipLaunchKernelGGL(tqc_actor_kernel, dim3(S), dim3(NTH), 0, st, g);
  if (const int32_t rc = pnp_check_launch("tqc_actor_kernel")) return rc;
  AdamArgs aa{};
  for (int i = 0; i < 10; i++) {
    aa.p[i] = d->actor[i]; aa.m[i] = d->actor_m[i]; aa.v[i] = d->actor_v[i]; aa.tgt[i] = nullptr;
    aa.step[i] = d->actor_step[i]; aa.off[i] = act_off(i);
  }
  aa.off[10] = ACT_P; aa.nt = 10;
  aa.part = g.part_a; aa.nparts = S; aa.stride = ACT_P;
  aa.lr = d->lr; aa.beta1 = d->beta1; aa.beta2 = d->beta2; aa.eps = d->adam_eps; aa.tau = d->tau;
  aa.grad_out = grads_out;
  aa.part_s = g.part_s; aa.nslab = S; aa.B = d->batch; aa.logs = d->logs;
  hipLaunchKernelGGL(tqc_adam_kernel, dim3((ACT_P + 255) / 256), dim3(256), 0, st, aa);
  if (const int32_t rc = pnp_check_launch("tqc_adam_kernel (actor)")) return rc;
  hipLaunchKernelGGL(tqc_step_inc, dim3(1), dim3(64), 0, st, aa);
  return pnp_check_launch("tqc_step_inc (actor)");
}
