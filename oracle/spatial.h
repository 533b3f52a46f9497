/* spatial.h — MuJoCo 2.3.3 spatial-algebra helpers (engine_util_spatial.c, engine_util_blas.c),
 * fp64.  TEST INFRASTRUCTURE ONLY (see oracle.c header). 6D motion vectors are [ang; lin],
 * com-based inertias are the 10-vector [Ixx Iyy Izz Ixy Ixz Iyz  m*dx m*dy m*dz  m]. */
#ifndef ORC_SPATIAL_H
#define ORC_SPATIAL_H

#include <math.h>
#include <string.h>

#define ORC_MINVAL 1e-15

static inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline double normalize3(double* v) {
  double n = sqrt(dot3(v, v));
  if (n < ORC_MINVAL) { v[0] = 1; v[1] = 0; v[2] = 0; return 0; }
  double s = 1.0 / n;
  v[0] *= s; v[1] *= s; v[2] *= s;
  return n;
}
static inline void sp_mulquat(double r[4], const double a[4], const double b[4]) {
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}
static inline void sp_negquat(double r[4], const double q[4]) { r[0] = q[0]; r[1] = -q[1]; r[2] = -q[2]; r[3] = -q[3]; }
/* res = q * (0, axis) */
static inline void sp_mulquataxis(double r[4], const double q[4], const double ax[3]) {
  double t[4];
  t[0] = -q[1] * ax[0] - q[2] * ax[1] - q[3] * ax[2];
  t[1] = q[0] * ax[0] + q[2] * ax[2] - q[3] * ax[1];
  t[2] = q[0] * ax[1] + q[3] * ax[0] - q[1] * ax[2];
  t[3] = q[0] * ax[2] + q[1] * ax[1] - q[2] * ax[0];
  memcpy(r, t, sizeof(t));
}
static inline void sp_normalize4(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < ORC_MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else if (fabs(n - 1) > ORC_MINVAL) { double s = 1.0 / n; q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s; }
}
static inline void sp_quat2mat(double m[9], const double q[4]) {
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    memset(m, 0, 9 * sizeof(double)); m[0] = m[4] = m[8] = 1; return;
  }
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[4] = q00 - q11 + q22 - q33; m[8] = q00 - q11 - q22 + q33;
  m[1] = 2 * (q12 - q03); m[2] = 2 * (q13 + q02); m[3] = 2 * (q12 + q03);
  m[5] = 2 * (q23 - q01); m[6] = 2 * (q13 - q02); m[7] = 2 * (q23 + q01);
}
static inline void sp_rotvecquat(double r[3], const double v[3], const double q[4]) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) { r[0] = r[1] = r[2] = 0; return; }
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) { r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; return; }
  double t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
  double t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
  double t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
  r[0] = v[0] + 2 * (q[2] * t2 - q[3] * t1);
  r[1] = v[1] + 2 * (q[3] * t0 - q[1] * t2);
  r[2] = v[2] + 2 * (q[1] * t1 - q[2] * t0);
}
static inline void sp_axisangle2quat(double r[4], const double ax[3], double ang) {
  if (ang == 0) { r[0] = 1; r[1] = r[2] = r[3] = 0; return; }
  double s = sin(ang * 0.5);
  r[0] = cos(ang * 0.5); r[1] = ax[0] * s; r[2] = ax[1] * s; r[3] = ax[2] * s;
}
static inline void mulmatvec3(double r[3], const double m[9], const double v[3]) {
  double t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline void mulmattvec3(double r[3], const double m[9], const double v[3]) {
  double t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  double t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  double t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline void mulmat3(double r[9], const double a[9], const double b[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof(t));
}
/* mju_quatIntegrate: quat <- quat * exp(vel*scale/2) (vel in the local frame) */
static inline void sp_quatintegrate(double q[4], const double vel[3], double scale) {
  double ax[3] = {vel[0], vel[1], vel[2]}, qr[4];
  double ang = scale * normalize3(ax);
  sp_axisangle2quat(qr, ax, ang);
  sp_normalize4(q);
  sp_mulquat(q, q, qr);
}
/* mju_inertCom: com-based 6D inertia from principal inertia, orientation, offset and mass */
static inline void sp_inertcom(double res[10], const double inert[3], const double mat[9],
                               const double dif[3], double mass) {
  double tmp[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      tmp[3 * i + j] = mat[3 * i] * inert[0] * mat[3 * j] + mat[3 * i + 1] * inert[1] * mat[3 * j + 1] +
                       mat[3 * i + 2] * inert[2] * mat[3 * j + 2];
  res[0] = tmp[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
  res[1] = tmp[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
  res[2] = tmp[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
  res[3] = tmp[1] - mass * dif[0] * dif[1];
  res[4] = tmp[2] - mass * dif[0] * dif[2];
  res[5] = tmp[5] - mass * dif[1] * dif[2];
  res[6] = mass * dif[0]; res[7] = mass * dif[1]; res[8] = mass * dif[2];
  res[9] = mass;
}
/* mju_mulInertVec: res = inert * vec (6D) */
static inline void sp_mulinertvec(double r[6], const double i[10], const double v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
/* mju_crossMotion: res = vel x v (motion) */
static inline void sp_crossmotion(double r[6], const double vel[6], const double v[6]) {
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
/* mju_crossForce: res = vel x* f (force) */
static inline void sp_crossforce(double r[6], const double vel[6], const double f[6]) {
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
/* mju_dofCom: cdof of a rotational dof = [axis; axis x offset] */
static inline void sp_dofcom(double r[6], const double axis[3], const double off[3]) {
  r[0] = axis[0]; r[1] = axis[1]; r[2] = axis[2];
  cross3(r + 3, axis, off);
}
/* mju_makeFrame: complete an orthonormal frame from its x axis (frame rows: x, y, z) */
static inline void sp_makeframe(double f[9]) {
  double t[3];
  normalize3(f);
  if (sqrt(dot3(f + 3, f + 3)) < 0.5) {
    if (fabs(f[1]) < 0.5) { f[3] = 0; f[4] = 1; f[5] = 0; }
    else { f[3] = 0; f[4] = 0; f[5] = 1; }
  }
  double d = dot3(f, f + 3);
  t[0] = f[0] * d; t[1] = f[1] * d; t[2] = f[2] * d;
  f[3] -= t[0]; f[4] -= t[1]; f[5] -= t[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

#endif
