// pnp_capi.cpp — model lifetime and error plumbing of libpnp.so (include/pnp.h).
//
// pnp_model_create replaces MjModel.from_xml_path (reference envs/panda_env.py:108): it takes
// the compiled MJCF constants (host, fp64) and uploads one fp32 and one fp64 DevModel image to
// the current HIP device.  Batch state never lives here: it is caller-owned device memory.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>

#include "phys_model.h"
#include "pnp_internal.h"

static thread_local char g_err[512] = "";

void pnp_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int32_t pnp_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    pnp_set_error("%s: %s", what, hipGetErrorString(e));
    return PNP_ERR_HIP;
  }
  return PNP_OK;
}

extern "C" int32_t pnp_abi_version(void) { return PNP_ABI_VERSION; }
extern "C" int32_t pnp_model_desc_size(void) { return (int32_t)sizeof(pnp_model_desc); }
extern "C" const char* pnp_last_error(void) { return g_err; }

template <typename T>
static void fill_dev(DevModel<T>* d, const pnp_model_desc* s) {
  memset(d, 0, sizeof(*d));
  d->nq = s->nq; d->nv = s->nv; d->nbody = s->nbody; d->njnt = s->njnt; d->nsite = s->nsite;
  d->nmocap = s->nmocap;
  for (int i = 0; i < s->nbody; i++) {
    d->body_parentid[i] = s->body_parentid[i];
    d->body_mocapid[i] = s->body_mocapid[i];
    d->body_jntadr[i] = s->body_jntadr[i];
    d->body_jntnum[i] = s->body_jntnum[i];
    const double* q = s->body_quat + 4 * i;
    d->body_simple[i] = (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0);
    for (int k = 0; k < 3; k++) d->body_pos[i][k] = (T)s->body_pos[3 * i + k];
    for (int k = 0; k < 4; k++) d->body_quat[i][k] = (T)q[k];
  }
  for (int j = 0; j < s->njnt; j++) {
    d->jnt_type[j] = s->jnt_type[j];
    d->jnt_qposadr[j] = s->jnt_qposadr[j];
    d->jnt_dofadr[j] = s->jnt_dofadr[j];
    for (int k = 0; k < 3; k++) {
      d->jnt_pos[j][k] = (T)s->jnt_pos[3 * j + k];
      d->jnt_axis[j][k] = (T)s->jnt_axis[3 * j + k];
    }
  }
  for (int i = 0; i < s->nq; i++) d->qpos0[i] = (T)s->qpos0[i];
  for (int i = 0; i < s->nsite; i++) {
    d->site_bodyid[i] = s->site_bodyid[i];
    for (int k = 0; k < 3; k++) d->site_pos[i][k] = (T)s->site_pos[3 * i + k];
    for (int k = 0; k < 4; k++) d->site_quat[i][k] = (T)s->site_quat[4 * i + k];
  }
}

// Host-only check of a model description: the kinematics image (fill_dev) and both precisions'
// physics images (build_phys: pair tables, broadphase groups, hulls, fp64 chain tables) are built
// in host memory and discarded -- no HIP call, so it runs (and is sanitised) without a GPU.
extern "C" int32_t pnp_model_check(const pnp_model_desc* desc) {
  if (!desc) {
    pnp_set_error("pnp_model_check: null argument");
    return PNP_ERR_ARG;
  }
  if (desc->nbody > PNP_MAXBODY || desc->njnt > PNP_MAXJNT || desc->nq > PNP_MAXQ ||
      desc->nv > PNP_MAXV || desc->nsite > PNP_MAXSITE || desc->nmocap > PNP_MAXMOCAP ||
      desc->nbody < 1) {
    pnp_set_error("pnp_model_check: model exceeds compiled capacity (nbody=%d njnt=%d nq=%d nv=%d nsite=%d)",
                  desc->nbody, desc->njnt, desc->nq, desc->nv, desc->nsite);
    return PNP_ERR_MODEL;
  }
  DevModel<double>* h = new (std::nothrow) DevModel<double>();
  DevModel<float>* hf = new (std::nothrow) DevModel<float>();
  DevPhys<float>* pf = new (std::nothrow) DevPhys<float>();
  DevPhys<double>* pd = new (std::nothrow) DevPhys<double>();
  int32_t rc = PNP_OK;
  char err[256] = {0};
  if (!h || !hf || !pf || !pd) {
    pnp_set_error("pnp_model_check: out of host memory");
    rc = PNP_ERR_ARG;
  } else {
    fill_dev(h, desc);
    fill_dev(hf, desc);
    if (build_phys(desc, pf, err, sizeof(err)) != 0 || build_phys(desc, pd, err, sizeof(err)) != 0) {
      pnp_set_error("pnp_model_check: %s", err);
      rc = PNP_ERR_MODEL;
    }
  }
  delete h;
  delete hf;
  delete pf;
  delete pd;
  return rc;
}

extern "C" int32_t pnp_model_create(const pnp_model_desc* desc, pnp_model** out) {
  if (!desc || !out) {
    pnp_set_error("pnp_model_create: null argument");
    return PNP_ERR_ARG;
  }
  *out = nullptr;
  if (desc->nbody > PNP_MAXBODY || desc->njnt > PNP_MAXJNT || desc->nq > PNP_MAXQ ||
      desc->nv > PNP_MAXV || desc->nsite > PNP_MAXSITE || desc->nmocap > PNP_MAXMOCAP ||
      desc->nbody < 1) {
    pnp_set_error("pnp_model_create: model exceeds compiled capacity (nbody=%d njnt=%d nq=%d nv=%d nsite=%d)",
                  desc->nbody, desc->njnt, desc->nq, desc->nv, desc->nsite);
    return PNP_ERR_MODEL;
  }
  pnp_model* m = new (std::nothrow) pnp_model();
  if (!m) {
    pnp_set_error("pnp_model_create: out of host memory");
    return PNP_ERR_ARG;
  }
  (void)hipGetDevice(&m->device);
  fill_dev(&m->h, desc);
  for (int j = 0; j < desc->njnt; j++) {
    m->jnt_range[j][0] = desc->jnt_range[2 * j];
    m->jnt_range[j][1] = desc->jnt_range[2 * j + 1];
  }
  DevModel<float> hf;
  fill_dev(&hf, desc);
  hipError_t e1 = hipMalloc(&m->d_f32, sizeof(DevModel<float>));
  hipError_t e2 = hipMalloc(&m->d_f64, sizeof(DevModel<double>));
  if (e1 != hipSuccess || e2 != hipSuccess) {
    pnp_set_error("pnp_model_create: hipMalloc failed: %s", hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    if (e1 == hipSuccess) (void)hipFree(m->d_f32);
    if (e2 == hipSuccess) (void)hipFree(m->d_f64);
    delete m;
    return PNP_ERR_HIP;
  }
  hipError_t e3 = hipMemcpy(m->d_f32, &hf, sizeof(hf), hipMemcpyHostToDevice);
  hipError_t e4 = hipMemcpy(m->d_f64, &m->h, sizeof(m->h), hipMemcpyHostToDevice);
  if (e3 != hipSuccess || e4 != hipSuccess) {
    pnp_set_error("pnp_model_create: hipMemcpy failed: %s", hipGetErrorString(e3 != hipSuccess ? e3 : e4));
    (void)hipFree(m->d_f32);
    (void)hipFree(m->d_f64);
    delete m;
    return PNP_ERR_HIP;
  }
  // physics images for the step kernel; a model outside the kernel's capacity keeps IK and
  // kinematics working and reports the reason from pnp_step
  m->p_f32 = nullptr;
  m->p_f64 = nullptr;
  m->phys_err[0] = 0;
  m->nu = desc->nu;
  DevPhys<float>* pf = new (std::nothrow) DevPhys<float>();
  DevPhys<double>* pd = new (std::nothrow) DevPhys<double>();
  if (pf && pd && build_phys(desc, pf, m->phys_err, sizeof(m->phys_err)) == 0 &&
      build_phys(desc, pd, m->phys_err, sizeof(m->phys_err)) == 0) {
    if (hipMalloc(&m->p_f32, sizeof(*pf)) == hipSuccess && hipMalloc(&m->p_f64, sizeof(*pd)) == hipSuccess &&
        hipMemcpy(m->p_f32, pf, sizeof(*pf), hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(m->p_f64, pd, sizeof(*pd), hipMemcpyHostToDevice) == hipSuccess) {
    } else {
      snprintf(m->phys_err, sizeof(m->phys_err), "device allocation of the physics image failed");
      if (m->p_f32) (void)hipFree(m->p_f32);
      if (m->p_f64) (void)hipFree(m->p_f64);
      m->p_f32 = nullptr;
      m->p_f64 = nullptr;
    }
  }
  delete pf;
  delete pd;
  *out = m;
  return PNP_OK;
}

extern "C" int32_t pnp_model_destroy(pnp_model* model) {
  if (!model) return PNP_OK;
  resident_forget(model);
  (void)hipFree(model->d_f32);
  (void)hipFree(model->d_f64);
  if (model->p_f32) (void)hipFree(model->p_f32);
  if (model->p_f64) (void)hipFree(model->p_f64);
  delete model;
  return PNP_OK;
}
