// pnp_internal.h — device-side model image and small spatial helpers shared by the kernels.
//
// The model lives in device global memory as one DevModel<T> per precision (fp32 for the
// product path, fp64 for parity debugging).  Every env of a batch reads the same constants, so
// the loads are wave-uniform and come from the scalar/L1 path; per-env state is SoA [B, n].
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/pnp.h"

#define PNP_MAXBODY 24
#define PNP_MAXJNT 16
#define PNP_MAXQ 40
#define PNP_MAXV 36
#define PNP_MAXSITE 12
#define PNP_MAXMOCAP 2
#define PNP_IK_MAXCHAIN 12

template <typename T>
struct DevModel {
  int nq, nv, nbody, njnt, nsite, nmocap;
  int body_parentid[PNP_MAXBODY];
  int body_mocapid[PNP_MAXBODY];
  int body_jntadr[PNP_MAXBODY];
  int body_jntnum[PNP_MAXBODY];
  int body_simple[PNP_MAXBODY];  // 1: body quat is identity (skip the rotation)
  T body_pos[PNP_MAXBODY][3];
  T body_quat[PNP_MAXBODY][4];
  int jnt_type[PNP_MAXJNT];
  int jnt_qposadr[PNP_MAXJNT];
  int jnt_dofadr[PNP_MAXJNT];
  T jnt_pos[PNP_MAXJNT][3];
  T jnt_axis[PNP_MAXJNT][3];
  T qpos0[PNP_MAXQ];
  int site_bodyid[PNP_MAXSITE];
  T site_pos[PNP_MAXSITE][3];
  T site_quat[PNP_MAXSITE][4];
};

// Root -> site kinematic chain for the IK kernel, passed BY VALUE as a kernel argument (lands in
// SGPRs via s_load: wave-uniform constants, no VGPR or LDS cost).  Built on the host from the
// compiled model; every body rotation is stored as a row-major matrix, every chain joint is a
// hinge about +-z through the body origin (checked on the host, PNP_ERR_UNSUPPORTED otherwise).
template <typename T>
struct IKChain {
  int nbody;
  int jnt[PNP_IK_MAXCHAIN];      // arm joint index (0..6) of the hinge on this body, or -1
  T axis_sign[PNP_IK_MAXCHAIN];  // +1 for axis +z, -1 for -z
  T R[PNP_IK_MAXCHAIN][9];       // body rotation in the parent frame
  T p[PNP_IK_MAXCHAIN][3];       // body position in the parent frame
  T site_pos[3];                 // site offset in the last body frame
  T lo[7], hi[7];                // jnt_range[0..6]
  T qpos0[7];
};

template <typename T> struct DevPhys;

struct pnp_model {
  int device;
  DevModel<float>* d_f32;   // device images
  DevModel<double>* d_f64;
  DevModel<double> h;       // host copy (fp64) used to build chains
  double jnt_range[PNP_MAXJNT][2];
  DevPhys<float>* p_f32;    // step-kernel images (null if the model is outside its capacity)
  DevPhys<double>* p_f64;
  char phys_err[160];
  int nu;                   // actuators (gym env ABI validation)
};

template <typename T> struct pnp_state_t {  // same layout as pnp_state / pnp_state_f64
  T* qpos; T* qvel; T* ctrl; T* mocap_pos; T* mocap_quat; T* qacc_warmstart; T* time; uint32_t* warn;
};

template <typename T> const DevPhys<T>* phys_image(const pnp_model* m);
template <> inline const DevPhys<float>* phys_image<float>(const pnp_model* m) { return m->p_f32; }
template <> inline const DevPhys<double>* phys_image<double>(const pnp_model* m) { return m->p_f64; }
template <typename T> int build_phys(const pnp_model_desc* s, DevPhys<T>* d, char* err, int errlen);
// resident.cpp: stream-ordered residency of a physics image in a device's constant segment.
// acquire() makes `model`'s image the one the symbol holds for launches on `stream` (copying it
// in, after every earlier reader of the old image, when another model was resident) and holds
// the slot until launched() has recorded the launch that reads it; see the top of resident.cpp.
enum ResidentImage { RES_FULL_F32 = 0, RES_FULL_F64, RES_COMPACT_F32, RES_COMPACT_GYM_F32, RES_WIDE_F32, RES_WIDE64_F64,
                     RES_NKIND };
class ResidentLease {
 public:
  ResidentLease() = default;
  ResidentLease(const ResidentLease&) = delete;
  ResidentLease& operator=(const ResidentLease&) = delete;
  ~ResidentLease();
  int32_t acquire(ResidentImage kind, const pnp_model* model, const void* symbol, const void* src, size_t bytes,
                  void* stream);
  int32_t launched();  // call once the kernels reading the image are enqueued on the stream
 private:
  void release();
  void* slot_ = nullptr;
  void* stream_ = nullptr;
  std::unique_lock<std::mutex> lock_;
};
void resident_forget(const pnp_model* model);
// step.hip: acquire the model's full-build physics image for a launch on `stream`
template <typename T> int32_t phys_resident(const pnp_model* model, void* stream, ResidentLease& lease);
// step_compact.hip: the compact-capacity fp32 step kernel (see the top of step.hip)
int32_t launch_step_compact(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, int32_t nsub,
                            void* stream, unsigned long long* prof);
int32_t step_compact_lds_bytes();
// step_wide.hip: the wide-capacity fp32 tier (resume passes of pnp_step and pnp_env_step)
int32_t launch_step_wide(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, int32_t nsub,
                         void* stream, unsigned long long* prof, int resume);
// hq / hq_target: the gym step's hand-over queue (env_dev.h, PNP_HQ_*): the resume pass then
// consumes the envs the full-tier passes publish, concurrently with them, on hq_grid workgroups
// (each gives up after hq_timeout ticks of the 100 MHz clock; <= 0: the default).  count_out
// (list-based passes): receives the number of envs the pass selected (device int).
int32_t launch_env_step_wide(const pnp_model* model, const pnp_state_t<float>* st, const pnp_env_params* p,
                             const pnp_env_state* e, const float* action, const pnp_env_out* o, int32_t B,
                             void* stream, int resume, int only_tier, int* hq = nullptr, int hq_target = 0,
                             int hq_grid = 0, long long hq_timeout = 0, int* count_out = nullptr);
int32_t step_wide_lds_bytes();
// forward_debug's wide tier: the envs whose full-tier forward outgrew it (record COUNTS + 3 = -1)
int32_t launch_forward_debug_wide(const pnp_model* model, const pnp_state_t<float>* st, int32_t B, double* dbg,
                                  void* stream);
int32_t launch_forward_debug_wide64(const pnp_model* model, const pnp_state_t<double>* st, int32_t B, double* dbg,
                                    void* stream);
// step_wide64.hip: the fp64 wide tier (resume passes of pnp_step_f64 and pnp_env_step_f64)
int32_t launch_step_wide64(const pnp_model* model, const pnp_state_t<double>* st, int32_t B, int32_t nsub,
                           void* stream);
int32_t launch_env_step_wide64(const pnp_model* model, const pnp_state_t<double>* st, const pnp_env_params* p,
                               const pnp_env_state* e, const double* action, const pnp_env_out* o, int32_t B,
                               void* stream);
int32_t step_wide64_lds_bytes();
// env_compact.hip: the compact tier of the fp32 gym step (every env from sub-step 0)
int32_t launch_env_step_compact(const pnp_model* model, const pnp_state_t<float>* st, const pnp_env_params* p,
                                const pnp_env_state* e, const float* action, const pnp_env_out* o, int32_t B,
                                void* stream, int only_tier);
int32_t env_compact_lds_bytes();
// env_compact.hip: the routing probe of a routed fp32 gym step (env_dev.h route_probe_kernel)
int32_t launch_env_route_probe(const pnp_model* model, const pnp_state_t<float>* st, uint8_t* tier, int32_t B,
                               void* stream);

// ---------------------------------------------------------------------------- error plumbing
void pnp_set_error(const char* fmt, ...);
int32_t pnp_check_launch(const char* what);

// ---------------------------------------------------------------------------- device helpers
// Same formulas as MuJoCo's engine_util_spatial.c (and oracle/oracle.c), templated on T.
template <typename T>
__device__ __forceinline__ void d_mulquat(T r[4], const T a[4], const T b[4]) {
  T t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  T t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  T t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  T t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

template <typename T>
__device__ __forceinline__ void d_normalize4(T q[4]) {
  T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < T(1e-15)) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - T(1)) > T(1e-15)) {
    T s = T(1) / n;
    q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
  }
}

template <typename T>
__device__ __forceinline__ void d_rotvecquat(T r[3], const T v[3], const T q[4]) {
  T t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
  T t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
  T t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
  r[0] = v[0] + 2 * (q[2] * t2 - q[3] * t1);
  r[1] = v[1] + 2 * (q[3] * t0 - q[1] * t2);
  r[2] = v[2] + 2 * (q[1] * t1 - q[2] * t0);
}

template <typename T>
__device__ __forceinline__ void d_quat2mat(T m[9], const T q[4]) {
  T q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  T q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  T q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
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

template <typename T>
__device__ __forceinline__ void d_mulmatvec3(T r[3], const T m[9], const T v[3]) {
  T t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  T t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  T t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

__device__ __forceinline__ void d_sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void d_sincos(double x, double* s, double* c) { sincos(x, s, c); }
