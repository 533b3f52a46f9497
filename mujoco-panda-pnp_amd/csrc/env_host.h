// env_host.h — host launchers and C ABI of the fused gym kernels (env_dev.h); full build of
// step.hip only.
//
// The gym step runs the full-capacity kernel in one launch (ENV_ALL).  The compact phased path
// (env_dev.h: ENV_PRO / ENV_PHYS + resume pass / ENV_EPI, bit-identical) is opt-in with
// PNP_GYM_COMPACT=1: on random-action gym workloads about a third of the envs carry more than the
// compact build's 20 contacts for long stretches (closed finger pads pressed together), so they
// are handed over in most physics launches and the phased path measured slower than the single
// full launch (tools/gym_ab.py: 275 ms full vs 304 ms one compact launch + resume vs 337 ms
// per-call phases, per 4096-env gym step).  PNP_GYM_CHUNK sets its physics-launch length.
#pragma once

static bool gym_compact_enabled() {
  const char* e = getenv("PNP_GYM_COMPACT");
  return e && e[0] == '1' && compact_enabled();
}

// ---------------------------------------------------------------- host launchers
static int32_t env_check(pnp_model* model, const void* st, const pnp_env_params* p, const pnp_env_state* e,
                         int32_t B, const char* fn) {
  if (!model || !st || !p || !e || B < 0) { pnp_set_error("%s: bad argument", fn); return PNP_ERR_ARG; }
  const DevModel<double>& h = model->h;
  bool ok = p->n_tasks >= 1 && p->n_tasks <= PNP_MAX_TASKS && p->n_substeps >= 1 && p->n_calls >= 1 &&
            p->ee_site >= 0 && p->ee_site < h.nsite && h.nmocap == 1 && model->nu >= 2 &&
            p->arm_ctrl_n >= 0 && p->arm_ctrl_n <= model->nu;
  for (int k = 0; k < p->n_tasks && ok; k++)
    ok = p->obj_site[k] >= 0 && p->obj_site[k] < h.nsite && p->target_site[k] >= 0 && p->target_site[k] < h.nsite &&
         p->obj_qadr[k] >= 0 && p->obj_qadr[k] + 7 <= h.nq;
  for (int k = 0; k < 9 && ok; k++) ok = p->neutral_qadr[k] >= 0 && p->neutral_qadr[k] < h.nq;
  ok = ok && p->finger_qadr[0] >= 0 && p->finger_qadr[0] < h.nq && p->finger_qadr[1] >= 0 &&
       p->finger_qadr[1] < h.nq && p->height_qadr >= 0 && p->height_qadr + 3 <= h.nq;
  if (!ok) { pnp_set_error("%s: env params do not fit the model", fn); return PNP_ERR_ARG; }
  if (B == 0) return PNP_OK;
  if (!e->goal || !e->task || !e->elapsed || !e->qpos_kin || !e->obj_height0 || !e->init_mocap || !e->init_qvel ||
      !e->init_time || !e->episode || !e->env_index) {
    pnp_set_error("%s: null env state buffer", fn);
    return PNP_ERR_ARG;
  }
  return PNP_OK;
}

template <typename T, typename K>
static int32_t env_prep(pnp_model* model, const pnp_state_t<T>* st, K kernel, const DevPhys<T>** dm, const char* fn,
                        void* stream) {
  if (!st->qpos || !st->qvel || !st->ctrl || !st->mocap_pos || !st->mocap_quat || !st->qacc_warmstart || !st->time ||
      !st->warn) {
    pnp_set_error("%s: null state buffer", fn);
    return PNP_ERR_ARG;
  }
  *dm = phys_image<T>(model);
  if (!*dm) { pnp_set_error("%s: model has no physics image (%s)", fn, model->phys_err); return PNP_ERR_MODEL; }
  if (const int32_t rc = phys_resident<T>(model, stream)) return rc;
  (void)kernel;
  return PNP_OK;
}

template <typename T>
static int32_t launch_env_init(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                               const pnp_env_state* e, int32_t B, void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_init");
  if (rc || B == 0) return rc;
  const DevPhys<T>* dm;
  auto k = env_init_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_init", stream))) return rc;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), B);
  return pnp_check_launch("env_init_kernel");
}
template <typename T>
static int32_t launch_env_reset(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                                const pnp_env_state* e, const uint8_t* mask, const pnp_env_out* o, int32_t B,
                                void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_reset");
  if (rc || B == 0) return rc;
  const DevPhys<T>* dm;
  auto k = env_reset_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_reset", stream))) return rc;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), mask,
                     out_view<T>(o), B);
  return pnp_check_launch("env_reset_kernel");
}
template <typename T>
static int32_t launch_env_step(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                               const pnp_env_state* e, const T* action, const pnp_env_out* o, int32_t B,
                               void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_step");
  if (rc || B == 0) return rc;
  if (!action) { pnp_set_error("pnp_env_step: null action"); return PNP_ERR_ARG; }
  const DevPhys<T>* dm;
  auto k = env_step_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_step", stream))) return rc;
  if (sizeof(T) == 4 && (int64_t)p->n_substeps * p->n_calls <= PNP_RESUME_MAXSUB && gym_compact_enabled()) {
    // phased fp32 gym step (env_dev.h: ENV_*): compact kernels, the full kernel's resume pass
    // after every mj_step call
    const pnp_state_t<float>* sf = reinterpret_cast<const pnp_state_t<float>*>(st);
    const float* af = reinterpret_cast<const float*>(action);
    if ((rc = launch_env_step_compact(model, sf, p, e, af, o, B, stream, ENV_PRO, 0, 0))) return rc;
    const int nsub = p->n_substeps * p->n_calls;
    const char* ce = getenv("PNP_GYM_CHUNK");   // experiments: sub-steps per physics launch
    const int chunk = ce && atoi(ce) > 0 ? atoi(ce) : p->n_substeps;
    for (int k0 = 0; k0 < nsub; k0 += chunk) {
      const int k1 = k0 + chunk < nsub ? k0 + chunk : nsub;
      if ((rc = launch_env_step_compact(model, sf, p, e, af, o, B, stream, ENV_PHYS, k0, k1))) return rc;
      if (compact_mode() == 2) continue;
      hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), action,
                         out_view<T>(o), B, 1, (int)ENV_PHYS, k0, k1);
      if ((rc = pnp_check_launch("env_step_kernel (resume)"))) return rc;
    }
    return launch_env_step_compact(model, sf, p, e, af, o, B, stream, ENV_EPI, 0, 0);
  }
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), action,
                     out_view<T>(o), B, 0, (int)ENV_ALL, 0, 0);
  return pnp_check_launch("env_step_kernel");
}

extern "C" int32_t pnp_env_params_size(void) { return (int32_t)sizeof(pnp_env_params); }

extern "C" int32_t pnp_env_init(pnp_model* model, const pnp_state* st, const pnp_env_params* p,
                                const pnp_env_state* e, int32_t B, void* stream) {
  return launch_env_init<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), p, e, B, stream);
}
extern "C" int32_t pnp_env_init_f64(pnp_model* model, const pnp_state_f64* st, const pnp_env_params* p,
                                    const pnp_env_state* e, int32_t B, void* stream) {
  return launch_env_init<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), p, e, B, stream);
}
extern "C" int32_t pnp_env_reset(pnp_model* model, const pnp_state* st, const pnp_env_params* p,
                                 const pnp_env_state* e, const uint8_t* mask, const pnp_env_out* o, int32_t B,
                                 void* stream) {
  return launch_env_reset<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), p, e, mask, o, B, stream);
}
extern "C" int32_t pnp_env_reset_f64(pnp_model* model, const pnp_state_f64* st, const pnp_env_params* p,
                                     const pnp_env_state* e, const uint8_t* mask, const pnp_env_out* o, int32_t B,
                                     void* stream) {
  return launch_env_reset<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), p, e, mask, o, B, stream);
}
extern "C" int32_t pnp_env_step(pnp_model* model, const pnp_state* st, const pnp_env_params* p,
                                const pnp_env_state* e, const float* action, const pnp_env_out* o, int32_t B,
                                void* stream) {
  return launch_env_step<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), p, e, action, o, B, stream);
}
extern "C" int32_t pnp_env_step_f64(pnp_model* model, const pnp_state_f64* st, const pnp_env_params* p,
                                    const pnp_env_state* e, const double* action, const pnp_env_out* o, int32_t B,
                                    void* stream) {
  return launch_env_step<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), p, e, action, o, B, stream);
}
