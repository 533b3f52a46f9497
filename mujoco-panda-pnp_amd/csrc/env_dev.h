// env_dev.h — the reference's gym surface as fused device code (included by step.hip, whose Env,
// stages and mj_step_dev it uses).  One 64-lane wave per env, like the step kernel.
//
//   env_init_kernel   FrankaEnv._env_setup + _initialize_multi_object_task (envs/panda_env.py:100-141)
//   env_reset_kernel  _reset_sim / _sample_object / _sample_goal / _get_obs (:146-158, :279-301, :360-391)
//   env_step_kernel   FrankaEnv.step (:163-196): clip -> _set_action (:250-277) -> 10 x mj_step(nstep=25)
//                     (:355-358) -> _get_obs -> _is_success (:303-306) -> compute_reward (:205-245)
//                     -> task sequencing -> TimeLimit(max_episode_steps=300) (__init__.py:15)
//
// gymnasium_robotics.utils.rotations (euler2quat, quat_mul, mat2euler) and MuJoCo's mju_mat2Quat
// are restated from their published definitions (third-party, absent here).
#pragma once

// Device code in the tier's namespace (step.hip PNP_NS): the full and the wide build both compile
// these kernels, with different Env layouts, so they must not share symbol names.
namespace PNP_NS {

#define PNP_RESET_STREAM 0x40000000u   // Philox stream word of the reset draws: | episode

// ---------------------------------------------------------------- Philox4x32-10 (pnp_amd/rng.py)
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)c[0] * 0xD2511F53ull, p1 = (uint64_t)c[2] * 0xCD9E8D57ull;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// rng.uniform(env, ndraw, seed, stream)[draw]: counter (env_lo, draw / 4, stream, env_hi = 0)
__device__ __forceinline__ double philox_uniform(uint32_t env, int draw, uint32_t stream, uint32_t k0, uint32_t k1) {
  uint32_t c[4] = {env, (uint32_t)(draw >> 2), stream, 0u};
  philox4x32_10(c, k0, k1);
  return (double)c[draw & 3] * (1.0 / 4294967296.0);
}

// ---------------------------------------------------------------- rotations
// gymnasium_robotics rotations.euler2quat (static x-y-z = roll, pitch, yaw), wxyz
template <typename T>
__device__ void g_euler2quat(const T e[3], T q[4]) {
  T si, ci, sj, cj, sk, ck;
  d_sincos(e[2] * T(0.5), &si, &ci);
  d_sincos(-e[1] * T(0.5), &sj, &cj);
  d_sincos(e[0] * T(0.5), &sk, &ck);
  const T cc = ci * ck, cs = ci * sk, sc = si * ck, ss = si * sk;
  q[0] = cj * cc + sj * ss;
  q[1] = cj * cs - sj * sc;
  q[2] = -(cj * ss + sj * cc);
  q[3] = cj * sc - sj * cs;
}
// rotations.quat_mul(q0, q1) (Hamilton product, wxyz)
template <typename T>
__device__ void g_quat_mul(const T a[4], const T b[4], T r[4]) {
  r[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  r[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  r[2] = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
  r[3] = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
}
// rotations.mat2euler (row-major R), with its 4 * float64-eps gimbal test
template <typename T>
__device__ void g_mat2euler(const T R[9], T e[3]) {
  const T cy = PM<T>::sqrt_(R[8] * R[8] + R[5] * R[5]);
  const bool ok = (double)cy > 4.0 * 2.220446049250313e-16;
  e[2] = ok ? -atan2(R[1], R[0]) : -atan2(-R[3], R[4]);
  e[1] = -atan2(-R[2], cy);
  e[0] = ok ? -atan2(R[5], R[8]) : T(0);
}
// MuJoCo mju_mat2Quat (largest-component branch, then normalised)
template <typename T>
__device__ void g_mat2quat(const T m[9], T q[4]) {
  if (m[0] + m[4] + m[8] > 0) {
    q[0] = T(0.5) * PM<T>::sqrt_(1 + m[0] + m[4] + m[8]);
    q[1] = T(0.25) * (m[7] - m[5]) / q[0];
    q[2] = T(0.25) * (m[2] - m[6]) / q[0];
    q[3] = T(0.25) * (m[3] - m[1]) / q[0];
  } else if (m[0] > m[4] && m[0] > m[8]) {
    q[1] = T(0.5) * PM<T>::sqrt_(1 + m[0] - m[4] - m[8]);
    q[0] = T(0.25) * (m[7] - m[5]) / q[1];
    q[2] = T(0.25) * (m[1] + m[3]) / q[1];
    q[3] = T(0.25) * (m[2] + m[6]) / q[1];
  } else if (m[4] > m[8]) {
    q[2] = T(0.5) * PM<T>::sqrt_(1 - m[0] + m[4] - m[8]);
    q[0] = T(0.25) * (m[2] - m[6]) / q[2];
    q[1] = T(0.25) * (m[1] + m[3]) / q[2];
    q[3] = T(0.25) * (m[5] + m[7]) / q[2];
  } else {
    q[3] = T(0.5) * PM<T>::sqrt_(1 - m[0] - m[4] + m[8]);
    q[0] = T(0.25) * (m[3] - m[1]) / q[3];
    q[1] = T(0.25) * (m[2] + m[6]) / q[3];
    q[2] = T(0.25) * (m[5] + m[7]) / q[3];
  }
  t_normalize4(q);
}

// ---------------------------------------------------------------- typed views of the C structs
template <typename T>
struct EnvSoA {
  T* goal; int32_t* task; int32_t* elapsed; T* qpos_kin; T* obj_height0; T* init_mocap; T* init_qvel;
  T* init_time; uint32_t* episode; uint32_t* env_index;
  uint8_t* tier;   // optional (null: no routing): the tier the env's next gym step starts in
};
template <typename T>
struct EnvOutT {
  T* obs; T* ag; T* dg; T* reward; T* success; uint8_t* terminated; uint8_t* truncated;
};

// site frame from the body frames of the last st_kinematics (mj_kinematics site pass)
template <typename T>
__device__ void site_frame(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int site, T pos[3], T mat[9]) {
  const DevPhys<T>& m = phys<T>();
  const int b = m.site_bodyid[site];
  T v[3], q[4];
  d_mulmatvec3(v, s.xmat[b], m.site_pos[site]);
  for (int t = 0; t < 3; t++) pos[t] = s.xpos[b][t] + v[t];
  d_mulquat(q, s.xquat[b], m.site_quat[site]);
  d_quat2mat(mat, q);
}
// mj_jacSite(site) * qvel (gymnasium_robotics get_site_xvelp / xvelr); needs st_compos_crb
// (subtree COM, cdof); lane-uniform result
template <typename T>
__device__ void site_vel(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, int site, const T pt[3], T vp[3], T vr[3]) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  T jp[3] = {0, 0, 0}, jr[3] = {0, 0, 0};
  if (l < m.nv) jac_col(m, s, m.site_bodyid[site], l, pt, jp, jr);
  const T qv = l < m.nv ? s.qvel[l] : T(0);
  for (int t = 0; t < 3; t++) {
    vp[t] = wsum(jp[t] * qv);
    vr[t] = wsum(jr[t] * qv);
  }
}

// forward kinematics (+ comPos for Jacobians) at qk, keeping s.qpos: s.qpos_pre holds s.qpos
template <typename T>
__device__ void kin_at(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, const T* qk, bool jac) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nq) { s.qpos_pre[l] = s.qpos[l]; s.qpos[l] = qk[l]; }
  wsync();
  st_kinematics(m, s);
  if (jac) st_compos_crb(m, s);
  if (l < m.nq) s.qpos[l] = s.qpos_pre[l];
  wsync();
}


// _get_obs on the current kinematics (positions) and s.qvel; width = finger qpos sum of the
// integrated state.  Writes obs / achieved / desired goal of env b; returns ee / object data.
template <typename T>
__device__ void env_observe(const DevPhys<T>& /*image: phys<T>()*/, Env<T>& s, const pnp_env_params& prm, int task, const T goal[3],
                            const EnvOutT<T>& out, int b, T width, T ee_p[3], T ee_R[9], T ob_p[3]) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  const int ti = task < prm.n_tasks ? task : prm.n_tasks - 1;   // current_target_object
  T ob_R[9], ee_vp[3], ee_vr[3], ob_vp[3], ob_vr[3], eul[3];
  site_frame(m, s, prm.ee_site, ee_p, ee_R);
  site_frame(m, s, prm.obj_site[ti], ob_p, ob_R);
  site_vel(m, s, prm.ee_site, ee_p, ee_vp, ee_vr);
  site_vel(m, s, prm.obj_site[ti], ob_p, ob_vp, ob_vr);
  g_mat2euler(ob_R, eul);
  const T dt = m.timestep * T(prm.n_substeps);   // MujocoRobotEnv.dt
  if (l == 0) {
    if (out.obs) {
      T* o = out.obs + (size_t)b * PNP_OBS_DIM;
      for (int t = 0; t < 3; t++) {
        o[t] = ee_p[t];
        o[3 + t] = ee_vp[t] * dt;
        o[7 + t] = ob_p[t];
        o[10 + t] = eul[t];
        o[13 + t] = ob_vp[t] * dt;
        o[16 + t] = ob_vr[t] * dt;
      }
      o[6] = width;
    }
    if (out.ag)
      for (int t = 0; t < 3; t++) out.ag[(size_t)b * 3 + t] = ob_p[t];
    if (out.dg)
      for (int t = 0; t < 3; t++) out.dg[(size_t)b * 3 + t] = goal[t];
  }
}

template <typename T>
__device__ void store_controls(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, const pnp_state_t<T>& st, int b) {
  const DevPhys<T>& m = phys<T>();
  const int l = lane_id();
  if (l < m.nu) st.ctrl[(size_t)b * m.nu + l] = s.ctrl[l];
  if (l < 3 * m.nmocap) st.mocap_pos[(size_t)b * 3 * m.nmocap + l] = s.mocap_pos[l];
  if (l < 4 * m.nmocap) st.mocap_quat[(size_t)b * 4 * m.nmocap + l] = s.mocap_quat[l];
}

// ---------------------------------------------------------------- init (_env_setup)
template <typename T>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) env_init_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st,
                                                      pnp_env_params prm, EnvSoA<T> es, int B) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  const int b = blockIdx.x;
  if (b >= B) return;
  const int l = lane_id();
  load_env(m, s, st, b);
  // set_joint_neutral; ctrl[0:7] = neutral[:7]; (welds already at identity relpose)
  if (l == 0) {
    for (int i = 0; i < 9; i++) s.qpos[prm.neutral_qadr[i]] = (T)prm.neutral[i];
    for (int i = 0; i < prm.arm_ctrl_n; i++) s.ctrl[i] = (T)prm.neutral[i];
  }
  wsync();
  // mj_forward -> initial mocap = ee_center_site pose (get_site_xpos, get_ee_orientation)
  st_kinematics(m, s);
  T ee_p[3], ee_R[9], ee_q[4], goal[3], gR[9];
  site_frame(m, s, prm.ee_site, ee_p, ee_R);
  g_mat2quat(ee_R, ee_q);
  site_frame(m, s, prm.target_site[0], goal, gR);
  if (l == 0) {
    for (int t = 0; t < 3; t++) s.mocap_pos[t] = ee_p[t];
    for (int t = 0; t < 4; t++) s.mocap_quat[t] = ee_q[t];
  }
  wsync();
  // _mujoco_step(): 10 x mj_step(nstep = n_substeps)
  NoClock clk;
  const int nsub = prm.n_substeps * prm.n_calls;
  for (int k = 0; k < nsub; k++) mj_step_dev(m, s, clk, k == nsub - 1 ? s.qpos_pre : nullptr);
  store_env(m, s, st, b);
  store_controls(m, s, st, b);
  if (l < m.nq) es.qpos_kin[(size_t)b * m.nq + l] = s.qpos_pre[l];
  if (l < m.nv) es.init_qvel[(size_t)b * m.nv + l] = s.qvel[l];
  if (l < 3) es.init_mocap[(size_t)b * 7 + l] = s.mocap_pos[l];
  if (l < 4) es.init_mocap[(size_t)b * 7 + 3 + l] = s.mocap_quat[l];
  if (l < 3) es.goal[(size_t)b * 3 + l] = goal[l];
  if (l == 0) {
    es.obj_height0[b] = s.qpos[prm.height_qadr + 2];
    es.init_time[b] = s.time;
    es.task[b] = 0;
    es.elapsed[b] = 0;
    es.episode[b] = 0;
    if (es.tier) es.tier[b] = 0;
  }
}

// ---------------------------------------------------------------- reset (_reset_sim + _get_obs)
template <typename T>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) env_reset_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st,
                                                       pnp_env_params prm, EnvSoA<T> es,
                                                       const uint8_t* __restrict__ mask, EnvOutT<T> out, int B) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  const int b = blockIdx.x;
  if (b >= B || (mask && !mask[b])) return;
  const int l = lane_id();
  load_env(m, s, st, b);
  // _sample_object centres: the objects' site_xpos as of the last forward (not refreshed by
  // set_joint_neutral / set_mocap_pose, which only write qpos / mocap)
  kin_at(m, s, es.qpos_kin + (size_t)b * m.nq, false);
  T ctr[PNP_MAX_TASKS][3];
#pragma unroll
  for (int k = 0; k < PNP_MAX_TASKS; k++) {
    T R[9];
    if (k < prm.n_tasks) site_frame(m, s, prm.obj_site[k], ctr[k], R);
  }
  const uint32_t ep = es.episode[b], env = es.env_index[b];
  if (l == 0) {
    s.time = es.init_time[b];
    for (int i = 0; i < 9; i++) s.qpos[prm.neutral_qadr[i]] = (T)prm.neutral[i];
    for (int t = 0; t < 3; t++) s.mocap_pos[t] = es.init_mocap[(size_t)b * 7 + t];
    for (int t = 0; t < 4; t++) s.mocap_quat[t] = es.init_mocap[(size_t)b * 7 + 3 + t];
    for (int k = 0; k < prm.n_tasks; k++) {
      // x = centre + np.random.uniform(-r, r) = centre + (-r + (r - -r) * u)
      const double ux = philox_uniform(env, 2 * k, PNP_RESET_STREAM | ep, prm.seed_lo, prm.seed_hi);
      const double uy = philox_uniform(env, 2 * k + 1, PNP_RESET_STREAM | ep, prm.seed_lo, prm.seed_hi);
      const double xr = prm.obj_x_range, yr = prm.obj_y_range;
      T* q = s.qpos + prm.obj_qadr[k];
      q[0] = ctr[k][0] + (T)(-xr + (xr - -xr) * ux);
      q[1] = ctr[k][1] + (T)(-yr + (yr - -yr) * uy);
      q[2] = ctr[k][2];
      q[3] = 1; q[4] = 0; q[5] = 0; q[6] = 0;
    }
    es.task[b] = 0;
    es.elapsed[b] = 0;
    es.episode[b] = ep + 1;
    if (es.tier) es.tier[b] = 0;
  }
  if (l < m.nv) s.qvel[l] = es.init_qvel[(size_t)b * m.nv + l];
  wsync();
  // _initialize_multi_object_task + mj_forward
  st_kinematics(m, s);
  st_compos_crb(m, s);
  T goal[3], gR[9];
  site_frame(m, s, prm.target_site[0], goal, gR);
  if (l < 3) es.goal[(size_t)b * 3 + l] = goal[l];
  if (l < m.nq) es.qpos_kin[(size_t)b * m.nq + l] = s.qpos[l];
  T ee_p[3], ee_R[9], ob_p[3];
  env_observe(m, s, prm, 0, goal, out, b, s.qpos[prm.finger_qadr[0]] + s.qpos[prm.finger_qadr[1]], ee_p, ee_R, ob_p);
  store_env(m, s, st, b);
  store_controls(m, s, st, b);
}

// ---------------------------------------------------------------- reward (compute_reward)
// FrankaEnv.compute_reward (panda_env.py:205-245) + _is_success (:303-306) for achieved goal ag and
// desired goal dg, at the ee frame (ee_p, ee_R) of the last forward, finger width `width`,
// initial_object_height h0 and current_task_index `task`; *placed = _is_success.
template <typename T>
__device__ T env_reward(const pnp_env_params& prm, const T ee_p[3], const T ee_R[9], const T ag[3], const T dg[3],
                        T width, T h0, int task, bool* placed) {
  const T dr[3] = {ee_p[0] - ag[0], ee_p[1] - ag[1], ee_p[2] - ag[2]};
  const T dp[3] = {ag[0] - dg[0], ag[1] - dg[1], ag[2] - dg[2]};
  const T d_reach = PM<T>::sqrt_(dr[0] * dr[0] + dr[1] * dr[1] + dr[2] * dr[2]);
  const T d_place = PM<T>::sqrt_(dp[0] * dp[0] + dp[1] * dp[1] + dp[2] * dp[2]);
  *placed = d_place < (T)prm.distance_threshold;
  const bool gripped = width < (T)prm.grip_width && d_reach < (T)prm.reach_thresh;
  const bool lifted = gripped && ag[2] - h0 > (T)prm.lift_height;
  T eq[4];
  g_mat2quat(ee_R, eq);
  T need[4] = {1, 0, 0, 0};   // VERTICAL_QUAT = euler2quat(0)
  if (ag[2] > (T)prm.high_pick_z) {
    const T hz[3] = {T(-1.5707963267948966), 0, 0};   // HORIZONTAL_QUAT = euler2quat([-pi/2, 0, 0])
    g_euler2quat(hz, need);
  }
  const T ori_err = T(1) - fabs(eq[0] * need[0] + eq[1] * need[1] + eq[2] * need[2] + eq[3] * need[3]);
  if (!prm.reward_dense) return *placed ? T(0) : T(-1);
  T reward = T(-0.003) - fmin(d_reach, (T)prm.reach_thresh);
  if (gripped) reward += T(2) + (T(1) - ori_err);
  if (lifted) reward += T(4);
  if (*placed) reward += T(10);
  reward += T(0.5) * (T(task) / T(prm.n_tasks));
  return reward;
}

// ---------------------------------------------------------------- evaluate (_get_obs + compute_reward)
// FrankaEnv._get_obs (panda_env.py:279-301) at the current state -- data.site_* of the last
// forward (qpos_kin), the current qvel and finger qpos -- and compute_reward / _is_success
// (:205-245, :303-306) for the given goals (ag / dg: [B*3], NULL = the observed ones).  Reads the
// state only: no sub-step, no task update, no TimeLimit count.
template <typename T>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) env_eval_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st,
                                                      pnp_env_params prm, EnvSoA<T> es, const T* __restrict__ ag_in,
                                                      const T* __restrict__ dg_in, EnvOutT<T> out, int B) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  const int b = blockIdx.x;
  if (b >= B) return;
  const int l = lane_id();
  load_env(m, s, st, b);
  kin_at(m, s, es.qpos_kin + (size_t)b * m.nq, true);
  const T width = s.qpos[prm.finger_qadr[0]] + s.qpos[prm.finger_qadr[1]];
  const int task = es.task[b];
  T goal[3], ee_p[3], ee_R[9], ob_p[3];
  for (int t = 0; t < 3; t++) goal[t] = es.goal[(size_t)b * 3 + t];
  env_observe(m, s, prm, task, goal, out, b, width, ee_p, ee_R, ob_p);
  T ag[3], dg[3];
  for (int t = 0; t < 3; t++) {
    ag[t] = ag_in ? ag_in[(size_t)b * 3 + t] : ob_p[t];
    dg[t] = dg_in ? dg_in[(size_t)b * 3 + t] : goal[t];
  }
  bool placed;
  const T reward = env_reward(prm, ee_p, ee_R, ag, dg, width, es.obj_height0[b], task, &placed);
  if (l == 0) {
    if (out.reward) out.reward[b] = (T)(float)reward;   // compute_reward returns np.float32
    if (out.success) out.success[b] = placed ? T(1) : T(0);
  }
}

// ---------------------------------------------------------------- step (FrankaEnv.step)
// Routing (env_state.tier): the smallest tier whose capacities hold a sub-step with a margin --
// compact (0), full (1), wide (2).  The full and wide kernels record the largest over the
// sub-steps they ran as the tier the env's next gym step starts in, so envs that stay heavy
// (pads pressed, a grasped cube) skip the compact tier and its hand-over wait.  A hint only: a
// wrong guess costs time (a hand-over, or a light env in a bigger tier), never results.
// tier byte: bits 0-1 the tier this step started in (read by every pass, stable for the whole
// step: the routed passes run concurrently), bits 2-3 the next one with bit 4 set once a pass
// has written it; route_commit_kernel moves it down after the step's last pass.
// Compact gym capacities (env_compact.hip) and full ones (phys_model.h), checked in those TUs.
#define PNP_GC_MAXCON 20
#define PNP_GC_MAXEFC 96
#define PNP_GC_MAXJSLOT 800
#define PNP_GC_JTCAP 768
#define PNP_GC_HCAP 288
#define PNP_GF_MAXCON 64
#define PNP_GF_MAXEFC 272
#define PNP_GF_MAXJSLOT 2688
#define PNP_GF_JTCAP 2560
template <typename T>
__device__ __forceinline__ int tier_need(const DevPhys<T>& m, const Env<T>& s) {
  const int ne = s.nefc, nc = s.ncon_raw;
  const int slots = ne ? s.efc_off[ne - 1] + row_width(m, s.efc_t0[ne - 1], s.efc_t1[ne - 1]) : 0;
  const int nis = ne ? s.nisland : 0;
  const int l = lane_id();
  const bool big = __ballot(l < nis && s.isl_roff[l + 1] - s.isl_roff[l] > PNP_BIG_ROWS - 4) != 0;
  const int jt = nis ? s.isl_joff[nis] : 0, he = nis ? s.isl_eoff[nis] : 0;
  if (5 * nc <= 4 * PNP_GC_MAXCON && 5 * ne <= 4 * PNP_GC_MAXEFC && 5 * slots <= 4 * PNP_GC_MAXJSLOT && !big &&
      5 * jt <= 4 * PNP_GC_JTCAP && 5 * he <= 4 * PNP_GC_HCAP)
    return 0;
  if (6 * nc <= 5 * PNP_GF_MAXCON && 6 * ne <= 5 * PNP_GF_MAXEFC && 6 * slots <= 5 * PNP_GF_MAXJSLOT &&
      6 * jt <= 5 * PNP_GF_JTCAP)
    return 1;
  return 2;
}

// Tiers (step.hip): the full build runs the whole gym step; with hand = 1 a physics sub-step that
// would overflow its capacity stops the env before that sub-step changes the state (controls and
// state stored, resume bits in warn, no epilogue), and the wide build's resume pass (resume = 1)
// finishes the physics from that sub-step and runs the epilogue.
// One env's gym step on its workgroup's wave 0 (env_step_kernel: one env per workgroup; the wide
// build's env_step_wide_kernel: a persistent loop over the selected envs).  k0: the sub-step to
// resume from (resume passes); cur: the env's current tier; mw: the workgroup's waves.
// hand_pct: bit 0 = hand overflowing sub-steps over, bits 8.. = the routing's wide share (below).
template <typename T>
__device__ __forceinline__ void env_step_one(const DevPhys<T>& m, Env<T>& s, const pnp_state_t<T>& st,
                                             const pnp_env_params& prm, const EnvSoA<T>& es, const T* __restrict__ action,
                                             const EnvOutT<T>& out, int b, int cur, int k0, int resume, int hand_pct, int mw) {
  (void)mw;
  const int l = lane_id();
  const int hand = hand_pct & 1, wide_pct = (hand_pct >> 8) & 255, full_pct = hand_pct >> 16;
  load_env(m, s, st, b, hand);
#if PNP_MW
  if (l == 0) s.mw = mw;
  wsync();
#endif
  T ee_p[3], ee_R[9], ee_q[4];
  if (!resume) {
  // ---- _set_action: ee pose from the last forward's site frame
  kin_at(m, s, es.qpos_kin + (size_t)b * m.nq, false);
  site_frame(m, s, prm.ee_site, ee_p, ee_R);
  g_mat2quat(ee_R, ee_q);
  if (l == 0) {
    // the action space is float32: np.clip(action, low, high) and the scalings 0.05 * a, 0.2 * a,
    // clip(a, -1, 1) * 0.1 happen in float32 in the reference (NumPy scalar promotion), before
    // meeting the float64 state; __fmul_rn keeps the product out of any FMA contraction
    float a[7];
    for (int k = 0; k < 7; k++) a[k] = fminf(fmaxf((float)action[(size_t)b * 7 + k], -1.0f), 1.0f);
    const T width = s.qpos[prm.finger_qadr[0]] + s.qpos[prm.finger_qadr[1]] + (T)__fmul_rn(a[6], (float)prm.finger_scale);
    const T half = fmin(fmax(width / T(2), m.act_ctrlrange[m.nu - 1][0]), m.act_ctrlrange[m.nu - 1][1]);
    s.ctrl[m.nu - 2] = half;
    s.ctrl[m.nu - 1] = half;
    T de[3], dq[4], tq[4];
    for (int t = 0; t < 3; t++) {
      s.mocap_pos[t] = ee_p[t] + (T)__fmul_rn((float)prm.pos_scale, a[t]);
      de[t] = (T)__fmul_rn(fminf(fmaxf(a[3 + t], -1.0f), 1.0f), (float)prm.rot_scale);
    }
    s.mocap_pos[2] = fmax(T(0), s.mocap_pos[2]);
    g_euler2quat(de, dq);
    g_quat_mul(dq, ee_q, tq);
    for (int t = 0; t < 4; t++) s.mocap_quat[t] = tq[t];
  }
  wsync();
  }
  // ---- _mujoco_step: n_calls x mj_step(nstep = n_substeps)
  NoClock clk;
  const int nsub = prm.n_substeps * prm.n_calls;
  int k = k0;
  const bool track = !PNP_COMPACT && es.tier;
  int need_tier = 0, nwide = 0, nfull = 0, nrun = 0;
  for (; k < nsub && !(PNP_HANDS && s.ovf); k++) {
    mj_step_dev(m, s, clk, k == nsub - 1 ? s.qpos_pre : nullptr);
    if (track && !(PNP_HANDS && s.ovf)) {
      const int t = tier_need(m, s);
      need_tier = max(need_tier, t);
      nwide += t == 2;
      nfull += t >= 1;
      nrun++;
    }
  }
  // an env that needed the wide tier on fewer than wide_pct % of the sub-steps it ran here starts
  // its next step in the full tier (3 envs per CU instead of 1) and is handed over -- through the
  // hand-over queue, at once -- when a sub-step needs it (closed fingers: pad contacts flicker in
  // and out, most sub-steps light)
  if (need_tier == 2 && 100 * nwide < wide_pct * nrun) need_tier = 1;
  // likewise compact -> full (PNP_GYM_FULL_PCT; the compact pass's hand-overs wait for it to end)
  if (need_tier == 1 && 100 * nfull < full_pct * nrun) need_tier = 0;
  if (PNP_HANDS && s.ovf) {   // sub-step k - 1 overflowed before changing the state: hand over
    if (l == 0)
      s.warn |= PNP_RESUME_FLAG | ((uint32_t)s.ovf << PNP_RESUME_WHY_SHIFT) | ((uint32_t)(k - 1) << PNP_RESUME_SHIFT);
    wsync();
    store_env(m, s, st, b);
    store_controls(m, s, st, b);
    return;
  }
  store_env(m, s, st, b);
  store_controls(m, s, st, b);
  if (track && l == 0) es.tier[b] = (uint8_t)(cur | need_tier << 2 | 0x10);
  const T width = s.qpos[prm.finger_qadr[0]] + s.qpos[prm.finger_qadr[1]];
  if (l < m.nq) es.qpos_kin[(size_t)b * m.nq + l] = s.qpos_pre[l];
  // ---- _get_obs at data.site_* (kinematics of qpos_pre) with the integrated qvel
  if (l < m.nq) { const T t = s.qpos[l]; s.qpos[l] = s.qpos_pre[l]; s.qpos_pre[l] = t; }
  wsync();
  st_kinematics(m, s);
  st_compos_crb(m, s);
  const int task = es.task[b];
  T dg[3];
  for (int t = 0; t < 3; t++) dg[t] = es.goal[(size_t)b * 3 + t];
  T ob_p[3];
  env_observe(m, s, prm, task, dg, out, b, width, ee_p, ee_R, ob_p);
  // ---- _is_success / compute_reward (before the task update)
  bool placed;
  const T reward = env_reward(prm, ee_p, ee_R, ob_p, dg, width, es.obj_height0[b], task, &placed);
  // ---- task sequencing, TimeLimit
  bool terminated = false;
  int ntask = task;
  T goal[3] = {dg[0], dg[1], dg[2]};
  if (placed) {
    ntask = task + 1;
    if (ntask < prm.n_tasks) {
      T gR[9];
      site_frame(m, s, prm.target_site[ntask], goal, gR);
    } else {
      terminated = true;
    }
  }
  const int elapsed = es.elapsed[b] + 1;
  const bool truncated = prm.max_episode_steps > 0 && elapsed >= prm.max_episode_steps;
  if (l == 0) {
    es.task[b] = ntask;
    es.elapsed[b] = elapsed;
    for (int t = 0; t < 3; t++) es.goal[(size_t)b * 3 + t] = goal[t];
    if (out.reward) out.reward[b] = (T)(float)reward;   // compute_reward returns np.float32
    if (out.success) out.success[b] = placed ? T(1) : T(0);
    if (out.terminated) out.terminated[b] = terminated;
    if (out.truncated) out.truncated[b] = truncated;
  }
}

// ---- hand-over queue of the fp32 gym step (the full-tier passes -> the wide tier's resume pass)
// The wide resume pass used to start after the full resume pass had finished every env, so an env
// handed compact -> full -> wide waited for the slowest env of the full pass before its wide
// sub-steps began (the gym step's span was the sum of three passes' slowest envs).  With the
// queue, each full-tier workgroup that hands its env over publishes it at once, and a persistent
// wide consumer grid (on a few CUs, launched after the producers in host order) resumes it while
// the full passes still run.  Layout (ints): count of entries, producer workgroups done, the
// consumers' claim counter, the consumers that timed out, the envs the fallback pass finished,
// then the entries (-1 until published).  Every env's computation is unchanged: only when its
// wide sub-steps start.
// A consumer that waits longer than its timeout for a producer gives up (counted in PNP_HQ_ERR)
// instead of holding the GPU; the env it waited for keeps its resume bits, and after the join the
// list-based wide resume pass finishes every env still carrying them (their count lands in
// PNP_HQ_LATE; one selection kernel when there are none).  So no env is ever left mid-step, and
// pnp_env_queue_status reports both counts.
#define PNP_HQ_COUNT 0
#define PNP_HQ_DONE 1
#define PNP_HQ_NEXT 2
#define PNP_HQ_ERR 3
#define PNP_HQ_LATE 4
#define PNP_HQ_PREV 7   // the last queued step's published count (kept across steps: the consumer grid's size)
#define PNP_HQ_ENTRY 8
// default consumer timeout: 20 s of the 100 MHz constant clock (PNP_GYM_QUEUE_TIMEOUT_US)
#define PNP_HQ_TIMEOUT 2000000000ll
// producer side: after the workgroup's last state store, publish its env if it handed over, and
// count the workgroup done (every workgroup of the grid, so the consumers know when to stop)
__device__ __forceinline__ void hq_publish(int* hq, int b, bool handed) {
  wsync();           // every lane's state stores issued ...
  __threadfence();   // ... and visible device-wide before the entry and the done count
  if (lane_id() == 0) {
    if (handed) {
      const int i = __hip_atomic_fetch_add(&hq[PNP_HQ_COUNT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&hq[PNP_HQ_ENTRY + i], b, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_fetch_add(&hq[PNP_HQ_DONE], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// consumer side: entry i (claimed by this workgroup) once published, or -1 once every producer
// workgroup is done and fewer than i + 1 entries exist (or on the timeout); wave-uniform
__device__ __forceinline__ int hq_take(int* hq, int i, int target, int cap, long long timeout) {
  if (i >= cap) return -1;   // (at most one entry per env)
  int b = -1;
  if (lane_id() == 0) {
    const long long t0 = wall_clock64();
    for (;;) {
      b = __hip_atomic_load(&hq[PNP_HQ_ENTRY + i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (b >= 0) break;
      if (__hip_atomic_load(&hq[PNP_HQ_DONE], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target &&
          __hip_atomic_load(&hq[PNP_HQ_COUNT], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) <= i)
        break;
      if (wall_clock64() - t0 > timeout) {
        __hip_atomic_fetch_add(&hq[PNP_HQ_ERR], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  return __builtin_amdgcn_readfirstlane(__shfl(b, 0));
}

template <typename T>
__global__ void __launch_bounds__(NT, sizeof(T) == 4 ? PNP_STEP_WAVES : 1) env_step_kernel(const DevPhys<T>* __restrict__ mp, pnp_state_t<T> st,
                                                      pnp_env_params prm, EnvSoA<T> es, const T* __restrict__ action,
                                                      EnvOutT<T> out, int B, int resume, int hand, int only_tier,
                                                      int* __restrict__ hq, const int* __restrict__ order) {
  __shared__ __attribute__((aligned(16))) Env<T> s_env;   // static LDS: see env_lds_note
  Env<T>& s = s_env;
  const DevPhys<T>& m = phys<T>();
  (void)mp;
  int b = blockIdx.x;
  if (b >= B) return;   // (grid = B)
  // order (resume passes): workgroup i runs the env at list position i (resume_order_kernel: the
  // longest remaining chains first), the workgroups past the list none
  if (order) b = b < order[0] ? order[1 + b] : -1;
  const int cur = b >= 0 && es.tier ? (es.tier[b] & 3) : 0;
  bool run = b >= 0 && !(only_tier >= 0 && es.tier && cur != only_tier);   // else routed to another tier's pass
  int k0 = 0;
  if (run && resume) {
    const uint32_t w = st.warn[b];
    run = (w & PNP_RESUME_FLAG) != 0;
    k0 = (int)((w >> PNP_RESUME_SHIFT) & PNP_RESUME_MAXSUB);
  }
  if (run) env_step_one(m, s, st, prm, es, action, out, b, cur, k0, resume, hand, 1);
  if (hq) hq_publish(hq, b, run && PNP_HANDS && s.ovf);
}

#if PNP_MW
// Wide and full tiers, persistent: the selection kernel lists the envs the pass runs (list[0] = count), and
// a grid of as many workgroups per CU as the LDS holds (one at 192 contacts) loops over the list.  Each workgroup is MW_WAVES waves: wave 0
// steps its env, the others are helper waves for the convex pass (step.hip, mw_helper).  Multi-wave
// workgroups launched one per env (4096 per pass, nearly all exiting at once) made the gym step
// 25 % slower even with the helpers idle; a resident grid over the selected envs does not.
__global__ void __launch_bounds__(1024) wide_select_kernel(const uint8_t* __restrict__ tier,
                                                           const uint32_t* __restrict__ warn, int B, int resume,
                                                           int only_tier, int* __restrict__ list,
                                                           int* __restrict__ count_out) {
  __shared__ int wcount[16];
  __shared__ int base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) base = 0;
  __syncthreads();
  for (int c = 0; c < B; c += 1024) {
    const int b = c + t;
    bool sel = false;
    if (b < B)
      sel = (only_tier < 0 || !tier || (tier[b] & 3) == only_tier) && (!resume || (warn[b] & PNP_RESUME_FLAG));
    const uint64_t bal = __ballot(sel);
    if (lane == 0) wcount[w] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int i = 0; i < w; i++) off += wcount[i];
    if (sel) list[1 + off + __popcll(bal & ((1ull << lane) - 1ull))] = b;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int i = 0; i < 16; i++) tot += wcount[i];
      base += tot;
    }
    __syncthreads();
  }
  if (t == 0) {
    list[0] = base;
    if (count_out) *count_out = base;
  }
}
// hq (resume passes of the gym step): consume the hand-over queue instead of the list -- claim
// entries one at a time until hq_take reports the producers done (hq_target workgroups) and
// the queue drained; B bounds the entries
__global__ void __launch_bounds__(NT * MW_WAVES, PNP_WIDE ? 1 : PNP_FULL_MW_EU) env_step_wide_kernel(pnp_state_t<float> st, pnp_env_params prm,
                                                                          EnvSoA<float> es, const float* __restrict__ action,
                                                                          EnvOutT<float> out, const int* __restrict__ list,
                                                                          int resume, int hand, int* __restrict__ hq,
                                                                          int hq_target, int B, long long hq_timeout,
                                                                          int hq_min, int hq_pct) {
  __shared__ __attribute__((aligned(16))) Env<float> s_env;   // static LDS: see env_lds_note
  Env<float>& s = s_env;
  const DevPhys<float>& m = phys<float>();
  if (threadIdx.x >= NT) {   // helper waves: wave 0's commands until MW_EXIT
    mw_helper(s);
    return;
  }
  auto one = [&](int b) {
    const int cur = es.tier ? (es.tier[b] & 3) : 0;
    const int k0 = resume ? (int)((st.warn[b] >> PNP_RESUME_SHIFT) & PNP_RESUME_MAXSUB) : 0;
    env_step_one(m, s, st, prm, es, action, out, b, cur, k0, resume, hand, MW_WAVES);
  };
  // the consumers this step keeps: about as many as the last step published (hand-overs arrive over
  // the whole step, and a consumer holds its CU's LDS while it waits, away from the producers);
  // the others end at once
  bool active = true;
  if (hq) {
    const int prev = __hip_atomic_load(&hq[PNP_HQ_PREV], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    active = (int)blockIdx.x < max(hq_min, (int)((long long)prev * hq_pct / 100));
  }
  if (hq && active) {
    for (;;) {
      int i = 0;
      if (lane_id() == 0) i = __hip_atomic_fetch_add(&hq[PNP_HQ_NEXT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      i = __builtin_amdgcn_readfirstlane(__shfl(i, 0));
      const int b = hq_take(hq, i, hq_target, B, hq_timeout);
      if (b < 0) break;
      one(b);
    }
  } else if (!hq) {
    const int count = list[0];
    for (int i = blockIdx.x; i < count; i += gridDim.x) one(list[1 + i]);
  }
  if (lane_id() == 0) s.mw_cmd = MW_EXIT;   // every path of wave 0 ends here
  __syncthreads();
}
#endif

#if PNP_COMPACT && PNP_GYM
// Routing probe (routed fp32 gym steps, before the passes): the compact tier's collision stage at
// each compact-routed env's current state -- the contacts of its step's first sub-step, which the
// action does not change.  An env that would overflow there is routed to the full tier for this
// step, so it starts on the routed full pass at once instead of waiting out the whole compact pass
// before its hand-over is resumed.  A hint: only where an env runs changes, never what it computes.
__global__ void __launch_bounds__(NT, PNP_STEP_WAVES) route_probe_kernel(pnp_state_t<float> st,
                                                                         uint8_t* __restrict__ tier, int B) {
  __shared__ __attribute__((aligned(16))) Env<float> s_env;   // static LDS: see env_lds_note
  Env<float>& s = s_env;
  const DevPhys<float>& m = phys<float>();
  const int b = blockIdx.x;
  if (b >= B || (tier[b] & 3) != 0) return;   // (grid = B) routed past the compact tier already
  NoClock clk;
  load_env(m, s, st, b, 1);
  st_kinematics(m, s);
  st_compos_crb(m, s);
  st_factor_M(m, s);
  st_collision(m, s, clk);
  if (s.nconvex && !s.ovf) st_collision_convex(m, s);
  if (lane_id() == 0 && s.ovf) tier[b] = 1;
}
#endif

#if !PNP_COMPACT && !PNP_WIDE && !PNP_WIDE64
// The full tier's resume pass in order of remaining sub-steps, most first (a counting sort of the
// selected envs by resume sub-step; ties in any order -- only which workgroup runs an env changes,
// never what it computes).  The dispatcher starts workgroups in index order, so the envs with the
// longest chains left start first and the pass does not end on one started late.
__global__ void __launch_bounds__(1024) resume_order_kernel(const uint8_t* __restrict__ tier,
                                                            const uint32_t* __restrict__ warn, int B, int only_tier,
                                                            int* __restrict__ list) {
  constexpr int NB = PNP_RESUME_MAXSUB + 1;
  __shared__ int cnt[NB];
  __shared__ int wtot[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = t; i < NB; i += 1024) cnt[i] = 0;
  __syncthreads();
  auto sel = [&](int b) {
    return (only_tier < 0 || !tier || (tier[b] & 3) == only_tier) && (warn[b] & PNP_RESUME_FLAG);
  };
  auto key = [&](int b) { return (int)((warn[b] >> PNP_RESUME_SHIFT) & PNP_RESUME_MAXSUB); };
  for (int b = t; b < B; b += 1024)
    if (sel(b)) atomicAdd(&cnt[key(b)], 1);
  __syncthreads();
  // exclusive scan of the NB bins: thread t owns NB / 1024 consecutive bins
  constexpr int PER = NB / 1024;
  static_assert(NB % 1024 == 0, "bins per thread");
  int v[PER], tot = 0;
  for (int j = 0; j < PER; j++) { v[j] = cnt[t * PER + j]; tot += v[j]; }
  int inc = tot;
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(inc, d);
    if (lane >= d) inc += u;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int base = inc - tot;
  for (int i = 0; i < w; i++) base += wtot[i];
  for (int j = 0; j < PER; j++) { cnt[t * PER + j] = base; base += v[j]; }
  __syncthreads();
  for (int b = t; b < B; b += 1024)
    if (sel(b)) list[1 + atomicAdd(&cnt[key(b)], 1)] = b;
  if (t == 1023) list[0] = base;   // the last thread's running offset = the total
}
__global__ void route_commit_kernel(uint8_t* __restrict__ tier, int B, int* __restrict__ hq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (hq && i == 0) hq[PNP_HQ_PREV] = hq[PNP_HQ_COUNT];   // the next queued step's consumer count
  if (i < B) {
    const uint8_t t = tier[i];
    if (t & 0x10) tier[i] = (uint8_t)((t >> 2) & 3);
  }
}
#endif

}  // namespace PNP_NS

// ---------------------------------------------------------------- host launchers
template <typename T>
static EnvSoA<T> env_view(const pnp_env_state* e) {
  return EnvSoA<T>{(T*)e->goal, e->task, e->elapsed, (T*)e->qpos_kin, (T*)e->obj_height0, (T*)e->init_mocap,
                   (T*)e->init_qvel, (T*)e->init_time, e->episode, e->env_index, e->tier};
}
template <typename T>
static EnvOutT<T> out_view(const pnp_env_out* o) {
  if (!o) return EnvOutT<T>{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  return EnvOutT<T>{(T*)o->obs, (T*)o->achieved_goal, (T*)o->desired_goal, (T*)o->reward, (T*)o->is_success,
                    o->terminated, o->truncated};
}

// PNP_GYM_QUEUE_MIN / PNP_GYM_QUEUE_PCT: the hand-over queue's consumers this step = max(MIN,
// PCT % of the envs the last queued step published), at most the launched grid
// (PNP_GYM_QUEUE_CU); the rest of the grid ends at once.  Defaults 8 and 100.
static int gym_queue_min() {
  const char* e = getenv("PNP_GYM_QUEUE_MIN");
  const int v = e ? atoi(e) : 8;
  return v < 0 ? 0 : v;   // (0 with PCT 0: no consumer -- the fallback pass takes every hand-over; tests)
}
static int gym_queue_pct() {
  const char* e = getenv("PNP_GYM_QUEUE_PCT");
  const int v = e ? atoi(e) : 100;
  return v < 0 ? 0 : (v > 10000 ? 10000 : v);
}
#if PNP_MW
struct WideLists {   // kinds: 0 / 1 the persistent passes' lists, 2 the full resume pass's order
  int* list[3] = {nullptr, nullptr, nullptr};
  int cap[3] = {0, 0, 0};
  int ncu = 0;
};
static int32_t wide_list(int kind, int32_t B, int** out, int* ncu) {
  static std::mutex mu;
  static WideLists wl[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { pnp_set_error("pnp_env_step: bad device"); return PNP_ERR_HIP; }
  std::lock_guard<std::mutex> lk(mu);
  WideLists& w = wl[dev];
  hipError_t e = hipSuccess;
  if (!w.ncu) e = hipDeviceGetAttribute(&w.ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess && w.cap[kind] < B + 1) {
    if (w.list[kind]) e = hipFree(w.list[kind]);   // (synchronises: only when a larger batch arrives)
    w.list[kind] = nullptr;
    w.cap[kind] = 0;
    if (e == hipSuccess) e = hipMalloc((void**)&w.list[kind], sizeof(int) * (size_t)(B + 1));
    if (e == hipSuccess) w.cap[kind] = B + 1;
  }
  if (e != hipSuccess) { pnp_set_error("pnp_env_step: wide list: %s", hipGetErrorString(e)); return PNP_ERR_HIP; }
  *out = w.list[kind];
  *ncu = w.ncu > 0 ? w.ncu : 256;
  return PNP_OK;
}
// persistent multi-wave gym pass of this build's tier over the envs the selection kernel lists
static int32_t launch_env_step_mw(const pnp_state_t<float>* st, const pnp_env_params* p, const pnp_env_state* e,
                                  const float* action, const pnp_env_out* o, int32_t B, void* stream, int resume,
                                  int only_tier, int hand, const char* what, int* hq = nullptr, int hq_target = 0,
                                  int hq_grid = 0, long long hq_timeout = PNP_HQ_TIMEOUT, int* count_out = nullptr) {
  if (B <= 0) return PNP_OK;
  int* list = nullptr;
  int ncu = 0;
  if (const int32_t rc = wide_list(resume ? 1 : 0, B, &list, &ncu)) return rc;
  const int per_cu = (int)(163840 / sizeof(Env<float>)) > 0 ? (int)(163840 / sizeof(Env<float>)) : 1;   // envs per CU (LDS)
  int grid = B < per_cu * ncu ? B : per_cu * ncu;
  if (hq) {
    // the consumer grid leaves the other CUs to the producers it waits for (no deadlock: they
    // always have room, and they are enqueued before it on any shared hardware queue); the
    // caller's grid is clamped to that (launch_env_step only takes the queue path when the device
    // has a CU to spare)
    grid = hq_grid < grid ? hq_grid : grid;
    if (grid > per_cu * ncu - 1) grid = per_cu * ncu - 1;
    if (grid < 1) { pnp_set_error("pnp_env_step: hand-over queue grid %d", grid); return PNP_ERR_ARG; }
  } else {
    // PNP_GYM_WIDE_GRID (A/B): at most this many workgroups for a list pass (a wide workgroup holds
    // a CU's LDS; fewer leave CUs to the concurrent full-tier pass)
    if (const char* eg = getenv("PNP_GYM_WIDE_GRID")) {
      const int cap = atoi(eg);
      if (cap > 0 && grid > cap) grid = cap;
    }
    hipLaunchKernelGGL(wide_select_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, e->tier, st->warn, B, resume,
                       only_tier, list, count_out);
    if (const int32_t rc = pnp_check_launch("wide_select_kernel")) return rc;
  }
  hipLaunchKernelGGL(env_step_wide_kernel, dim3(grid), dim3(NT * MW_WAVES), 0, (hipStream_t)stream, *st, *p,
                     env_view<float>(e), action, out_view<float>(o), (const int*)list, resume, hand, hq, hq_target, B,
                     hq_timeout, gym_queue_min(), gym_queue_pct());
  return pnp_check_launch(what);
}
#endif
// PNP_GYM_WIDE_PCT: the routing sends an env to the wide tier for its next step only if at least
// this share (%) of its sub-steps needed it (see env_step_one; 0: any one sub-step, round 3's
// rule).  Random-action gym workload (4096 envs, profiles/r04/gym_route_pct_ab.log): 0: 20.1-20.2 k
// gym-steps/s (~600 envs a step started in the wide tier, one env per CU, most of them closed
// grippers whose pad contacts overflow the full tier on a few sub-steps); 10 .. 100: 22.4-22.8 k.
// Default 50.
// PNP_GYM_FULL_PCT: the same share for starting in the full tier instead of the compact one
// (0: any one sub-step).  Measured on top of the wide share (profiles/r04/gym_route_pct_ab.log):
// 0: 22.1 k gym-steps/s; 20 .. 80: 22.7-23.1 k.  Default 50.
static int gym_full_pct() {
  const char* e = getenv("PNP_GYM_FULL_PCT");
  const int v = e ? atoi(e) : 50;
  return v < 0 ? 0 : (v > 100 ? 100 : v);
}
static int gym_wide_pct() {
  const char* e = getenv("PNP_GYM_WIDE_PCT");
  const int v = e ? atoi(e) : 50;
  return v < 0 ? 0 : (v > 100 ? 100 : v);
}
#if PNP_COMPACT
int32_t launch_env_step_compact(const pnp_model* model, const pnp_state_t<float>* st, const pnp_env_params* p,
                                const pnp_env_state* e, const float* action, const pnp_env_out* o, int32_t B,
                                void* stream, int only_tier) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_COMPACT_GYM_F32, model, (const void*)&g_phys_f32, src,
                                       sizeof(DevPhys<float>), stream))
    return rc;
  hipLaunchKernelGGL(env_step_kernel<float>, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, *p,
                     env_view<float>(e), action, out_view<float>(o), B, 0, 1, only_tier, (int*)nullptr, (const int*)nullptr);
  if (const int32_t rc = pnp_check_launch("env_step_kernel (compact)")) return rc;
  return lease.launched();
}
int32_t env_compact_lds_bytes() { return (int32_t)sizeof(Env<float>); }
int32_t launch_env_route_probe(const pnp_model* model, const pnp_state_t<float>* st, uint8_t* tier, int32_t B,
                               void* stream) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_COMPACT_GYM_F32, model, (const void*)&g_phys_f32, src,
                                       sizeof(DevPhys<float>), stream))
    return rc;
  hipLaunchKernelGGL(route_probe_kernel, dim3(B), dim3(NT), 0, (hipStream_t)stream, *st, tier, B);
  if (const int32_t rc = pnp_check_launch("route_probe_kernel")) return rc;
  return lease.launched();
}
#elif PNP_WIDE
// wide tier: resume pass of the gym step over the envs the full kernel handed over (resume = 1),
// or the routed pass over the envs whose step starts in the wide tier (resume = 0, only_tier = 2);
// launched by the full build's launch_env_step, which holds the full image's lease
// The selection lists (one per pass kind: the routed pass on its side stream and the resume pass
// on the caller's stream can be in flight together), per device; their users are serialised by
// the full image's lease like the route streams.
int32_t launch_env_step_wide(const pnp_model* model, const pnp_state_t<float>* st, const pnp_env_params* p,
                             const pnp_env_state* e, const float* action, const pnp_env_out* o, int32_t B,
                             void* stream, int resume, int only_tier, int* hq, int hq_target, int hq_grid,
                             long long hq_timeout, int* count_out) {
  const DevPhys<float>* src = phys_image<float>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  if (B <= 0) return PNP_OK;
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE_F32, model, (const void*)&g_phys_f32, src, sizeof(DevPhys<float>),
                                       stream))
    return rc;
  if (const int32_t rc = launch_env_step_mw(st, p, e, action, o, B, stream, resume, only_tier, gym_wide_pct() << 8 | gym_full_pct() << 16,
                                            hq ? "env_step_wide_kernel (hand-over queue)" : "env_step_wide_kernel",
                                            hq, hq_target, hq_grid, hq_timeout > 0 ? hq_timeout : PNP_HQ_TIMEOUT,
                                            count_out))
    return rc;
  return lease.launched();
}
#elif PNP_WIDE64
// fp64 wide tier: the resume pass of pnp_env_step_f64 over the envs the full fp64 kernel handed
// over (launched by the full build's launch_env_step, which holds the full fp64 image's lease)
int32_t launch_env_step_wide64(const pnp_model* model, const pnp_state_t<double>* st, const pnp_env_params* p,
                               const pnp_env_state* e, const double* action, const pnp_env_out* o, int32_t B,
                               void* stream) {
  const DevPhys<double>* src = phys_image<double>(model);
  if (!src) { pnp_set_error("model has no physics image (%s)", model->phys_err); return PNP_ERR_MODEL; }
  if (B <= 0) return PNP_OK;
  ResidentLease lease;
  if (const int32_t rc = lease.acquire(RES_WIDE64_F64, model, (const void*)&g_phys_f64, src,
                                       sizeof(DevPhys<double>), stream))
    return rc;
  hipLaunchKernelGGL(env_step_kernel<double>, dim3(B), dim3(NT), 0, (hipStream_t)stream, src, *st, *p,
                     env_view<double>(e), action, out_view<double>(o), B, 1, 0, -1, (int*)nullptr, (const int*)nullptr);
  if (const int32_t rc = pnp_check_launch("env_step_kernel (wide64)")) return rc;
  return lease.launched();
}
#else
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
                        void* stream, ResidentLease& lease) {
  if (!st->qpos || !st->qvel || !st->ctrl || !st->mocap_pos || !st->mocap_quat || !st->qacc_warmstart || !st->time ||
      !st->warn) {
    pnp_set_error("%s: null state buffer", fn);
    return PNP_ERR_ARG;
  }
  *dm = phys_image<T>(model);
  if (!*dm) { pnp_set_error("%s: model has no physics image (%s)", fn, model->phys_err); return PNP_ERR_MODEL; }
  if (const int32_t rc = phys_resident<T>(model, stream, lease)) return rc;
  (void)kernel;
  return PNP_OK;
}

template <typename T>
static int32_t launch_env_init(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                               const pnp_env_state* e, int32_t B, void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_init");
  if (rc || B == 0) return rc;
  const DevPhys<T>* dm;
  ResidentLease lease;
  auto k = env_init_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_init", stream, lease))) return rc;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), B);
  if ((rc = pnp_check_launch("env_init_kernel"))) return rc;
  return lease.launched();
}
template <typename T>
static int32_t launch_env_reset(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                                const pnp_env_state* e, const uint8_t* mask, const pnp_env_out* o, int32_t B,
                                void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_reset");
  if (rc || B == 0) return rc;
  const DevPhys<T>* dm;
  ResidentLease lease;
  auto k = env_reset_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_reset", stream, lease))) return rc;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), mask,
                     out_view<T>(o), B);
  if ((rc = pnp_check_launch("env_reset_kernel"))) return rc;
  return lease.launched();
}
template <typename T>
static int32_t launch_env_eval(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                               const pnp_env_state* e, const T* ag, const T* dg, const pnp_env_out* o, int32_t B,
                               void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_evaluate");
  if (rc || B == 0) return rc;
  const DevPhys<T>* dm;
  ResidentLease lease;
  auto k = env_eval_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_evaluate", stream, lease))) return rc;
  hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), ag, dg,
                     out_view<T>(o), B);
  if ((rc = pnp_check_launch("env_eval_kernel"))) return rc;
  return lease.launched();
}
// PNP_GYM_ROUTE: unset / 1 = with an env_state.tier buffer, envs start their fp32 gym step in the
// tier their last step finished in (default); 0 = every env starts in the compact tier (A/B runs)
static bool gym_route_enabled() {
  const char* e = getenv("PNP_GYM_ROUTE");
  return !(e && e[0] == '0');
}
// PNP_GYM_FULL_RESUME: unset / 1 = the compact pass's hand-overs are resumed by the full tier,
// whose own hand-overs go on to the wide resume pass (default); 0 = routed steps send the compact
// pass's hand-overs straight to the wide resume pass (A/B runs)
static bool gym_full_resume_enabled() {
  const char* e = getenv("PNP_GYM_FULL_RESUME");
  return !(e && e[0] == '0');
}
// PNP_GYM_FULL_MW: 1 = the fp32 gym step's full-tier passes run the persistent two-wave kernel
// (env_step_wide_kernel of the full build: the helper wave takes half of the convex pass); unset /
// 0 = one single-wave workgroup per env (default: the two-wave pass measured 5 % slower on the gym
// step, 18.0 k vs 18.9 k gym-steps/s -- a persistent grid walks the selected envs in list order,
// while one workgroup per env lets the dispatcher balance the CUs; profiles/r03/ab_gym_full_mw.log)
// PNP_GYM_ROUTE_ORDER: 1 (default) = the routed full pass is enqueued before the routed wide pass,
// 0 = wide first (round 5).  A wide workgroup holds a CU's LDS (140 KB) for its env's whole step,
// so the pass enqueued first takes the CUs: full first, the steady-state gym step 442.6 / 435.5 ->
// 423.7 / 422.3 ms (profiles/r06/ab_round6.log r6am); from reset unchanged.
static int gym_route_order() {
  const char* e = getenv("PNP_GYM_ROUTE_ORDER");
  return e ? atoi(e) : 1;
}
static bool gym_full_mw_enabled() {
  const char* e = getenv("PNP_GYM_FULL_MW");
  return PNP_MPR_SV_WAVES >= PNP_NS::MW_WAVES && e && e[0] == '1';
}
// PNP_GYM_QUEUE: unset / 1 = routed fp32 gym steps hand the full tier's hand-overs to the wide
// tier through the device queue (hq_publish / hq_take), consumed concurrently with the full passes
// (default); 0 = the wide resume pass starts after the full passes (A/B runs).  PNP_GYM_QUEUE_CU:
// the consumer grid, one wide workgroup per CU (default: the device's CUs less an eighth -- 224 of
// 256 on an MI355X -- leaving the rest to the producers, whose progress is all the consumers wait
// for; clamped to the CU count - 1, and a device with a single CU takes the non-queue path).  Measured (4096 envs, random actions,
// gym-steps/s; profiles/r04/gym_queue_ab.log), with round 3's routing: queue off 18.5 k; consumers
// 32: 9.5 k, 64: 15.2 k, 128: 19.5 k, 160-255: 19.9-20.4 k; with the routing shares (50 %): off
// 18.8 k, 96: 18.8 k, 160: 22.3 k, 192: 22.9 k, 240: 23.2 k -- the full passes hand envs to the
// wide tier at every point of the step, and each needs a free consumer then
// PNP_GYM_FULL_ORDER: unset / 1 = the full tier's resume pass starts its envs in order of
// remaining sub-steps, most first (resume_order_kernel); 0 = in env order
// PNP_GYM_PROBE: 1 = routed fp32 gym steps probe every compact-routed env's first sub-step's
// contacts and route the ones the compact tier cannot hold to the full tier for this step
// (route_probe_kernel); unset / 0 = the last step's routing alone (default: the probe measured
// +2.5 % on the random-action gym leg and -12 % on C5's policy-driven 8192-env leg, whose envs
// overflowing at sub-step 0 mostly fall back under the compact capacity within the step)
static bool gym_probe_enabled() {
  const char* e = getenv("PNP_GYM_PROBE");
  return e && e[0] == '1';
}
static bool gym_full_order_enabled() {
  const char* e = getenv("PNP_GYM_FULL_ORDER");
  return !(e && e[0] == '0');
}
static bool gym_queue_enabled() {
  const char* e = getenv("PNP_GYM_QUEUE");
  return !(e && e[0] == '0');
}
static int gym_queue_grid(int ncu) {
  const int def = ncu - (ncu / 8 > 1 ? ncu / 8 : 1);
  const char* e = getenv("PNP_GYM_QUEUE_CU");
  const int g = e ? atoi(e) : def;
  const int v = g > 0 ? g : def;
  return v < ncu - 1 ? v : ncu - 1;
}
// PNP_GYM_QUEUE_TIMEOUT_US: how long a consumer waits for a producer before it gives up (the
// fallback resume pass then finishes that env); default 20 s.  Tests set it tiny to exercise the
// fallback.
static long long gym_queue_timeout() {
  const char* e = getenv("PNP_GYM_QUEUE_TIMEOUT_US");
  const long long us = e ? atoll(e) : 0;
  return us > 0 ? us * 100 : PNP_HQ_TIMEOUT;   // 100 MHz constant clock
}
// CUs of the current device (cached per device)
static int device_cus() {
  static std::mutex mu;
  static int ncu[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lk(mu);
  if (!ncu[dev] && hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu[dev] = 0;
  return ncu[dev];
}
// the hand-over queue buffer per device (PNP_HQ_ENTRY header ints + one entry per env); its users
// are serialised by the full image's lease like the route streams
static std::mutex g_hq_mu;
static int* g_hq_buf[64] = {};
static int32_t hand_queue(int32_t B, int** out) {
  std::mutex& mu = g_hq_mu;
  int** buf = g_hq_buf;
  static int cap[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { pnp_set_error("pnp_env_step: bad device"); return PNP_ERR_HIP; }
  std::lock_guard<std::mutex> lk(mu);
  hipError_t e = hipSuccess;
  if (cap[dev] < B + PNP_HQ_ENTRY) {
    if (buf[dev]) e = hipFree(buf[dev]);   // (synchronises: only when a larger batch arrives)
    buf[dev] = nullptr;
    cap[dev] = 0;
    if (e == hipSuccess) e = hipMalloc((void**)&buf[dev], sizeof(int) * (size_t)(B + PNP_HQ_ENTRY));
    if (e == hipSuccess) e = hipMemset(buf[dev], 0, sizeof(int) * PNP_HQ_ENTRY);   // (PNP_HQ_PREV: none yet)
    if (e == hipSuccess) cap[dev] = B + PNP_HQ_ENTRY;
  }
  if (e != hipSuccess) { pnp_set_error("pnp_env_step: hand-over queue: %s", hipGetErrorString(e)); return PNP_ERR_HIP; }
  *out = buf[dev];
  return PNP_OK;
}
// Three side streams per device for the routed passes and the hand-over queue's consumer, forked
// from and joined back into the caller's stream.  Used only while the full image's lease is held
// (launch_env_step), which serialises their users per device; creation has its own lock.
// `last`: recorded on the caller's stream when a routed step is complete; the next routed step
// (possibly on another stream) waits for it, so two steps never share the per-device selection
// lists and hand-over queue on the GPU at the same time.
struct RouteStreams {
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr}, cdone = nullptr, last = nullptr;
  bool last_valid = false;
};
static int32_t route_streams(RouteStreams** out) {
  static std::mutex mu;
  static RouteStreams rs[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { pnp_set_error("pnp_env_step: bad device"); return PNP_ERR_HIP; }
  std::lock_guard<std::mutex> lk(mu);
  RouteStreams& r = rs[dev];
  hipError_t e = hipSuccess;
  // (neither wave priority, s_setprio, for the routed passes nor the highest stream priority
  // shortened the routed wide pass: its span is the heaviest env's own chain of sub-steps)
  for (int i = 0; i < 3 && e == hipSuccess; i++) {
    if (!r.side[i]) e = hipStreamCreateWithFlags(&r.side[i], hipStreamNonBlocking);
    if (e == hipSuccess && !r.join[i]) e = hipEventCreateWithFlags(&r.join[i], hipEventDisableTiming);
  }
  if (e == hipSuccess && !r.fork) e = hipEventCreateWithFlags(&r.fork, hipEventDisableTiming);
  if (e == hipSuccess && !r.cdone) e = hipEventCreateWithFlags(&r.cdone, hipEventDisableTiming);
  if (e == hipSuccess && !r.last) e = hipEventCreateWithFlags(&r.last, hipEventDisableTiming);
  if (e != hipSuccess) { pnp_set_error("pnp_env_step: route streams: %s", hipGetErrorString(e)); return PNP_ERR_HIP; }
  *out = &r;
  return PNP_OK;
}

template <typename T>
static int32_t launch_env_step(pnp_model* model, const pnp_state_t<T>* st, const pnp_env_params* p,
                               const pnp_env_state* e, const T* action, const pnp_env_out* o, int32_t B,
                               void* stream) {
  int32_t rc = env_check(model, st, p, e, B, "pnp_env_step");
  if (rc || B == 0) return rc;
  if (!action) { pnp_set_error("pnp_env_step: null action"); return PNP_ERR_ARG; }
  const DevPhys<T>* dm;
  ResidentLease lease;
  auto k = env_step_kernel<T>;
  if ((rc = env_prep(model, st, k, &dm, "pnp_env_step", stream, lease))) return rc;
  if constexpr (sizeof(T) == 8) {
    // fp64 (the facade, the batched behaviour trees): the full kernel, handing the envs whose
    // sub-steps outgrow it to the fp64 wide tier's resume pass
    const int w64 = p->n_substeps * p->n_calls <= PNP_RESUME_MAXSUB && wide_enabled();
    hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, (hipStream_t)stream, dm, *st, *p, env_view<T>(e), action,
                       out_view<T>(o), B, 0, w64, -1, (int*)nullptr, (const int*)nullptr);
    if ((rc = pnp_check_launch("env_step_kernel (fp64)"))) return rc;
    if (w64 && (rc = launch_env_step_wide64(model, st, p, e, action, o, B, stream))) return rc;
    return lease.launched();
  }
  // fp32 tiers: the compact gym kernel (8 envs per CU) runs every env, the full kernel resumes
  // the envs it hands over, the wide kernel the envs the full kernel hands over
  const bool tiers = sizeof(T) == 4 && p->n_substeps * p->n_calls <= PNP_RESUME_MAXSUB;
  const int wide = tiers && wide_enabled();
  const int hand_pct = wide | gym_wide_pct() << 8 | gym_full_pct() << 16;   // hand flag + routing shares
  const bool compact = tiers && gym_compact_enabled();
  const auto* st32 = reinterpret_cast<const pnp_state_t<float>*>(st);
  const float* a32 = reinterpret_cast<const float*>(action);
  const hipStream_t s0 = (hipStream_t)stream;
  // routed: the envs whose last step finished in the full / wide tier start there, on side streams
  // concurrent with the compact pass; the resume passes then only see this step's new hand-overs
  const bool route = compact && wide && gym_compact_mode() == 1 && e->tier && gym_route_enabled();
  // fp32 full-tier passes: persistent, two waves per env (helper wave for the convex pass)
  const bool full_mw = tiers && gym_full_mw_enabled();
  // the full passes' hand-overs reach the wide tier through the device queue (routed steps)
  const int ncu = device_cus();
  const bool queue = route && !full_mw && gym_full_resume_enabled() && gym_queue_enabled() && ncu >= 2;
  int* hq = nullptr;
  RouteStreams* rs = nullptr;
  // join side stream i back into the caller's stream (its kernels read the full image and write
  // the state: later work on s0, and the next model switch, must be ordered after them)
  auto join_side = [&](int i) -> hipError_t {
    hipError_t he = hipEventRecord(rs->join[i], rs->side[i]);
    if (he == hipSuccess) he = hipStreamWaitEvent(s0, rs->join[i], 0);
    return he;
  };
  // an error after the fork still joins both side streams and records the lease's use on s0
  // before it is reported (the routed passes already enqueued keep running)
  bool forked = false;
  const int nside = queue ? 3 : 2;
  auto fail = [&](int32_t code) -> int32_t {
    if (forked) {
      for (int i = 0; i < nside; i++) join_side(i);
      lease.launched();
    }
    return code;
  };
  if (route) {
    if ((rc = route_streams(&rs))) return rc;
    hipError_t he = rs->last_valid ? hipStreamWaitEvent(s0, rs->last, 0) : hipSuccess;
    // the routing probe (PNP_GYM_PROBE=1): envs whose first sub-step overflows the compact tier
    // start on the routed full pass; ordered after the last routed step, before the fork
    if (he == hipSuccess && gym_probe_enabled() &&
        (rc = launch_env_route_probe(model, st32, e->tier, B, stream)))
      return rc;
    if (queue && he == hipSuccess) {   // a fresh queue, ordered before every pass of this step
      if ((rc = hand_queue(B, &hq))) return rc;
      he = hipMemsetAsync(hq, 0, sizeof(int) * PNP_HQ_PREV, s0);   // the header but PNP_HQ_PREV
      if (he == hipSuccess) he = hipMemsetAsync(hq + PNP_HQ_ENTRY, 0xFF, sizeof(int) * (size_t)B, s0);
    }
    if (he == hipSuccess) he = hipEventRecord(rs->fork, s0);   // after the full image's copy and the last step
    for (int i = 0; i < nside && he == hipSuccess; i++) he = hipStreamWaitEvent(rs->side[i], rs->fork, 0);
    if (he != hipSuccess) { pnp_set_error("pnp_env_step: fork: %s", hipGetErrorString(he)); return PNP_ERR_HIP; }
    forked = true;
    // the routed passes' launch order (PNP_GYM_ROUTE_ORDER: 1 full first, the default; 0 wide first)
    const bool full_first = gym_route_order() == 1;
    if (!full_first && (rc = launch_env_step_wide(model, st32, p, e, a32, o, B, rs->side[1], 0, 2))) return fail(rc);
    if (full_mw) {
      rc = launch_env_step_mw(st32, p, e, a32, o, B, rs->side[0], 0, 1, hand_pct, "env_step_wide_kernel (full, routed)");
    } else {
      hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, rs->side[0], dm, *st, *p, env_view<T>(e), action, out_view<T>(o), B,
                         0, hand_pct, 1, hq, (const int*)nullptr);
      rc = pnp_check_launch("env_step_kernel (full, routed)");
    }
    if (rc) return fail(rc);
    if (full_first && (rc = launch_env_step_wide(model, st32, p, e, a32, o, B, rs->side[1], 0, 2))) return fail(rc);
  }
  if (compact && (rc = launch_env_step_compact(model, st32, p, e, a32, o, B, stream, route ? 0 : -1))) return fail(rc);
  if (compact && gym_compact_mode() == 2) {
    if (forked)
      for (int i = 0; i < nside; i++) join_side(i);
    return lease.launched();
  }
  if (queue) {   // the consumer starts once the compact pass is done (it does not take its CUs)
    if (const hipError_t he = hipEventRecord(rs->cdone, s0)) {
      pnp_set_error("pnp_env_step: compact event: %s", hipGetErrorString(he));
      return fail(PNP_ERR_HIP);
    }
  }
  if (!route || gym_full_resume_enabled()) {
    if (full_mw) {
      rc = launch_env_step_mw(st32, p, e, a32, o, B, stream, compact ? 1 : 0, route ? 0 : -1, hand_pct,
                              "env_step_wide_kernel (full)");
    } else {
      // the resume pass in order of remaining sub-steps (PNP_GYM_FULL_ORDER, default on)
      int* order = nullptr;
      if (compact && sizeof(T) == 4 && gym_full_order_enabled()) {
        int ncu_unused = 0;
        if ((rc = wide_list(2, B, &order, &ncu_unused))) return fail(rc);
        hipLaunchKernelGGL(resume_order_kernel, dim3(1), dim3(1024), 0, s0, e->tier, st->warn, B, route ? 0 : -1, order);
        if ((rc = pnp_check_launch("resume_order_kernel"))) return fail(rc);
      }
      hipLaunchKernelGGL(k, dim3(B), dim3(NT), 0, s0, dm, *st, *p, env_view<T>(e), action, out_view<T>(o), B,
                         compact ? 1 : 0, hand_pct, route ? 0 : -1, hq, (const int*)order);
      rc = pnp_check_launch("env_step_kernel");
    }
    if (rc) return fail(rc);
  }
  if (queue) {
    // the wide consumer of both full passes' hand-overs (2 B producer workgroups), enqueued after
    // both of them in host order
    if (const hipError_t he = hipStreamWaitEvent(rs->side[2], rs->cdone, 0)) {
      pnp_set_error("pnp_env_step: consumer wait: %s", hipGetErrorString(he));
      return fail(PNP_ERR_HIP);
    }
    if ((rc = launch_env_step_wide(model, st32, p, e, a32, o, B, rs->side[2], 1, -1, hq, 2 * B, gym_queue_grid(ncu),
                                   gym_queue_timeout())))
      return fail(rc);
    for (int i = 0; i < 3; i++)
      if (const hipError_t he = join_side(i)) {
        pnp_set_error("pnp_env_step: join: %s", hipGetErrorString(he));
        return fail(PNP_ERR_HIP);
      }
    // fallback: any env a consumer gave up on still carries its resume bits -- the list-based
    // wide resume pass finishes it (its count -> hq[PNP_HQ_LATE]; nothing to do: one selection
    // kernel and an empty grid)
    if ((rc = launch_env_step_wide(model, st32, p, e, a32, o, B, stream, 1, -1, nullptr, 0, 0, 0, hq + PNP_HQ_LATE)))
      return fail(rc);
  } else {
    if (route) {   // the wide resume pass also takes the routed full pass's hand-overs
      if (const hipError_t he = join_side(0)) {
        pnp_set_error("pnp_env_step: join: %s", hipGetErrorString(he));
        return fail(PNP_ERR_HIP);
      }
    }
    if (wide && (rc = launch_env_step_wide(model, st32, p, e, a32, o, B, stream, 1, -1))) return fail(rc);
    if (route) {
      if (const hipError_t he = join_side(1)) {
        pnp_set_error("pnp_env_step: join: %s", hipGetErrorString(he));
        return fail(PNP_ERR_HIP);
      }
    }
  }
  if (e->tier) {   // every pass has run: the next step's tiers become current
    hipLaunchKernelGGL(route_commit_kernel, dim3((B + 255) / 256), dim3(256), 0, s0, e->tier, B, hq);
    if ((rc = pnp_check_launch("route_commit_kernel"))) return fail(rc);
  }
  if (route) {
    if (const hipError_t he = hipEventRecord(rs->last, s0)) {
      pnp_set_error("pnp_env_step: step event: %s", hipGetErrorString(he));
      return fail(PNP_ERR_HIP);
    }
    rs->last_valid = true;
  }
  return lease.launched();   // recorded on the caller's stream, after both joins
}

extern "C" int32_t pnp_env_params_size(void) { return (int32_t)sizeof(pnp_env_params); }

// the hand-over queue's header after the last routed fp32 gym step on the current device
// (synchronises the device): [0] entries published, [1] producer workgroups done, [2] consumer
// claims, [3] consumers that timed out, [4] envs the fallback resume pass finished.  All zero
// before any queued step.
extern "C" int32_t pnp_env_queue_status(int32_t* out5) {
  if (!out5) { pnp_set_error("pnp_env_queue_status: null out"); return PNP_ERR_ARG; }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { pnp_set_error("pnp_env_queue_status: bad device"); return PNP_ERR_HIP; }
  int h[PNP_HQ_ENTRY] = {};
  {
    std::lock_guard<std::mutex> lk(g_hq_mu);
    if (g_hq_buf[dev]) {
      hipError_t e = hipDeviceSynchronize();
      if (e == hipSuccess) e = hipMemcpy(h, g_hq_buf[dev], sizeof(h), hipMemcpyDeviceToHost);
      if (e != hipSuccess) { pnp_set_error("pnp_env_queue_status: %s", hipGetErrorString(e)); return PNP_ERR_HIP; }
    }
  }
  for (int i = 0; i < 5; i++) out5[i] = h[i];
  return PNP_OK;
}

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
extern "C" int32_t pnp_env_evaluate(pnp_model* model, const pnp_state* st, const pnp_env_params* p,
                                    const pnp_env_state* e, const float* ag, const float* dg, const pnp_env_out* o,
                                    int32_t B, void* stream) {
  return launch_env_eval<float>(model, reinterpret_cast<const pnp_state_t<float>*>(st), p, e, ag, dg, o, B, stream);
}
extern "C" int32_t pnp_env_evaluate_f64(pnp_model* model, const pnp_state_f64* st, const pnp_env_params* p,
                                        const pnp_env_state* e, const double* ag, const double* dg,
                                        const pnp_env_out* o, int32_t B, void* stream) {
  return launch_env_eval<double>(model, reinterpret_cast<const pnp_state_t<double>*>(st), p, e, ag, dg, o, B, stream);
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
#endif  // PNP_WIDE
