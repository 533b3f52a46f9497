// skills.hip — device math of the scripted-skill layer (reference panda_mujoco_gym/skills/).
//
//   slerp_track_kernel  RotateSkill.reset's trajectory (reference skills/rotate.py:39-46):
//                       target = R(start) * R(delta), then scipy Slerp([0, 1], [start, target])
//                       sampled at np.linspace(0, 1, steps) -- for B skills at once (the batched
//                       behaviour tree resets many RotateSkills in one tick).
//
// scipy.spatial.transform (the reference's dependency, absent from the GPU path) is restated from
// its published definitions: quaternions scalar-last (x, y, z, w) and normalised on construction;
// composition p * q (Hamilton product) renormalised; inv = conjugate; as_rotvec with the
// w >= 0 branch and its small-angle series (angle <= 1e-3); from_rotvec likewise; Slerp's keyframe
// step as the rotation vector of start^-1 * target, applied as start * exp(t * rotvec).
// tests/test_skills_gpu.py compares the kernel with scipy itself (1e-14).  One thread per
// (skill, sample): 50 samples x B skills, fp64 (the skill layer computes in float64 like numpy).
#include "pnp_internal.h"

namespace {

__device__ __forceinline__ void q_norm(double q[4]) {
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; k++) q[k] /= n;
}
// scipy _compose_quat (x, y, z, w), then Rotation(..., normalize=True)
__device__ __forceinline__ void q_compose(const double p[4], const double q[4], double r[4]) {
  const double cx = p[1] * q[2] - p[2] * q[1], cy = p[2] * q[0] - p[0] * q[2], cz = p[0] * q[1] - p[1] * q[0];
  r[0] = p[3] * q[0] + q[3] * p[0] + cx;
  r[1] = p[3] * q[1] + q[3] * p[1] + cy;
  r[2] = p[3] * q[2] + q[3] * p[2] + cz;
  r[3] = p[3] * q[3] - (p[0] * q[0] + p[1] * q[1] + p[2] * q[2]);
  q_norm(r);
}

__global__ void slerp_track_kernel(const double* __restrict__ q0, const double* __restrict__ delta, int steps,
                                   double* __restrict__ target, double* __restrict__ track, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * steps) return;
  const int b = i / steps, k = i - b * steps;
  double a[4], d[4], t[4], ai[4], rel[4];
  for (int c = 0; c < 4; c++) { a[c] = q0[4 * b + c]; d[c] = delta[4 * b + c]; }
  q_norm(a);
  q_norm(d);
  q_compose(a, d, t);                       // target = R(start) * R(delta)
  if (k == 0 && target)
    for (int c = 0; c < 4; c++) target[4 * b + c] = t[c];
  ai[0] = -a[0]; ai[1] = -a[1]; ai[2] = -a[2]; ai[3] = a[3];
  q_compose(ai, t, rel);                    // start^-1 * target
  if (rel[3] < 0)                           // as_rotvec: the w >= 0 representative
    for (int c = 0; c < 4; c++) rel[c] = -rel[c];
  const double vn = sqrt(rel[0] * rel[0] + rel[1] * rel[1] + rel[2] * rel[2]);
  const double ang = 2.0 * atan2(vn, rel[3]);
  const double sc = ang <= 1e-3 ? 2.0 + ang * ang / 12.0 + 7.0 * ang * ang * ang * ang / 2880.0 : ang / sin(ang / 2.0);
  // np.linspace(0, 1, steps): k * (1 / (steps - 1)), the last sample exactly 1
  const double tk = steps == 1 ? 0.0 : (k == steps - 1 ? 1.0 : (double)k * (1.0 / (double)(steps - 1)));
  double rv[3];
  for (int c = 0; c < 3; c++) rv[c] = sc * rel[c] * tk;
  const double an = sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
  const double s2 = an <= 1e-3 ? 0.5 - an * an / 48.0 + an * an * an * an / 3840.0 : sin(an / 2.0) / an;
  const double e[4] = {s2 * rv[0], s2 * rv[1], s2 * rv[2], cos(an / 2.0)};
  double out[4];
  q_compose(a, e, out);                     // start * exp(t * rotvec)
  for (int c = 0; c < 4; c++) track[((size_t)b * steps + k) * 4 + c] = out[c];
}

}  // namespace

extern "C" int32_t pnp_slerp_track_f64(const double* start_xyzw, const double* delta_xyzw, int32_t steps,
                                       double* target_xyzw, double* track_xyzw, int32_t B, void* stream) {
  if (!start_xyzw || !delta_xyzw || !track_xyzw || steps < 1 || B < 0) {
    pnp_set_error("pnp_slerp_track_f64: bad argument");
    return PNP_ERR_ARG;
  }
  if (B == 0) return PNP_OK;
  const int n = B * steps, nt = 256;
  hipLaunchKernelGGL(slerp_track_kernel, dim3((n + nt - 1) / nt), dim3(nt), 0, (hipStream_t)stream, start_xyzw,
                     delta_xyzw, steps, target_xyzw, track_xyzw, B);
  return pnp_check_launch("slerp_track_kernel");
}
