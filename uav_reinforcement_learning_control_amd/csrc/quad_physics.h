// quad_physics.h -- one env step of the reference hot path, as __host__ __device__ templates.
//
// T = float is what the gfx950 kernels run (state resident in HBM as float32 SoA). The same
// source instantiated with T = double on the host is cross-checked against the independent
// generic float64 oracle (oracle/quad_oracle.c) to 1e-12 in tests/test_physics_host.py, which
// is how the structured closed form below is verified without a GPU.
//
// Reference semantics reproduced (file:line into the reference):
//   RateControlWrapper.action            envs/rate_wrapper.py:69-98
//   denormalize (float32)                utils/normalization.py:20-30   (hover_env.py:169)
//   _mix_to_motors, voltage sag          envs/hover_env.py:102-124, 173-176
//   mujoco.mj_step                       envs/hover_env.py:180 (MuJoCo 3.x Euler step; see below)
//   QuadState.set_from_mujoco (scipy)    utils/state.py:28-46
//   _get_obs + normalize (float32)       envs/hover_env.py:126-136, utils/normalization.py:7-17
//   _get_reward                          envs/hover_env.py:138-141
//   _is_terminated, truncation           envs/hover_env.py:150-157, 182-188
//   reset / random_reset / set_state     envs/hover_env.py:200-238, utils/state.py:48-65,90-98
//   TrajectoryFollowEnv differences      envs/trajectory_follow_env.py:24-26,60-63,220-253
//
// The physics is MuJoCo's Euler step for drone.xml in closed form (quad_model.h explains the
// reduction): generalized speeds u = (v_world, w_body, s_1..4); forces from the motors (site
// transmission), gravity and the inertia-box fluid model on all five bodies; bias from the exact
// Newton-Euler velocity products; qacc from the 3x3 Schur-reduced solve; then semi-implicit Euler
// with MuJoCo's quaternion integration. MuJoCo's mj_checkPos/Vel/Acc resets and its bad-ctrl
// zeroing are reproduced.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "quad_model.h"

#define QD_HD __host__ __device__ __forceinline__

// QD_PROBE (tools/probe/ builds only, never the product): per-wave s_memtime stamps at phase
// boundaries of the step, to see where a lone wave's time goes. QD_STAMP(st, k) records stamp k
// into the wave-uniform array st (nullptr: no-op); the scheduling barriers keep instructions from
// moving across the boundary, so the probe build is slower than the product and only its
// phase proportions are meaningful.
#if defined(QD_PROBE) && defined(__HIP_DEVICE_COMPILE__)
#define QD_STAMP(st, k)                                   \
  do {                                                    \
    if (st) {                                             \
      __builtin_amdgcn_sched_barrier(0);                  \
      (st)[k] = __builtin_amdgcn_s_memtime();             \
      __builtin_amdgcn_sched_barrier(0);                  \
    }                                                     \
  } while (0)
// QD_PIN(x): the probe's stamps must not be crossed by IR-level code motion either; an empty
// volatile asm that reads x forces x to be computed before the next stamp.
#define QD_PIN(x) asm volatile("" ::"v"(x))
#else
#define QD_STAMP(st, k) \
  do {                  \
  } while (0)
#define QD_PIN(x) \
  do {            \
  } while (0)
#endif
#define QD_PIN_N(arr, n)                                  \
  do {                                                    \
    _Pragma("unroll") for (int pin_i_ = 0; pin_i_ < (n); pin_i_++) QD_PIN((arr)[pin_i_]); \
  } while (0)

namespace quadenv {

// ---------------------------------------------------------------------------------------------
// math. The double overloads (host test instantiation) are libm; the float overloads are what
// the kernel runs: short, branch-light sequences with ~1e-7 absolute error, far inside the
// 1e-5 parity bar (see DESIGN.md "Kernel arithmetic"). Full-range sincosf/atan2f/hypotf from
// the device libm cost several times the instructions and most of the registers.
QD_HD float frcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
QD_HD float fsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(x);
#else
  return sqrtf(x);
#endif
}
QD_HD float frsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rsqf(x);
#else
  return 1.0f / sqrtf(x);
#endif
}
QD_HD double q_sqrt(double x) { return sqrt(x); }
QD_HD float q_sqrt(float x) { return fsqrt(x); }
QD_HD double q_rsqrt(double x) { return 1.0 / sqrt(x); }
QD_HD float q_rsqrt(float x) { return frsqrt(x); }
QD_HD double q_atan2(double y, double x) { return atan2(y, x); }
QD_HD double q_hypot(double x, double y) { return hypot(x, y); }
QD_HD float q_hypot(float x, float y) { return fsqrt(x * x + y * y); }  // |args| <= 2 here
QD_HD float q_fma(float a, float b, float c) { return fmaf(a, b, c); }
QD_HD double q_fma(double a, double b, double c) { return fma(a, b, c); }
QD_HD float q_abs(float x) { return fabsf(x); }
QD_HD double q_abs(double x) { return fabs(x); }
QD_HD float q_exp(float x) { return expf(x); }
QD_HD double q_exp(double x) { return exp(x); }
QD_HD void q_sincos(double x, double* s, double* c) { sincos(x, s, c); }

// int(q) & 3 of an integral float with v_cvt_i32_f32's semantics (saturating, NaN -> 0) on the
// host as well: there the plain conversion of a diverged state's huge or NaN angle is undefined
// behaviour (found by UBSan, tools/san); the device keeps the one conversion instruction
QD_HD int quadrant_of(float q) {
#if defined(__HIP_DEVICE_COMPILE__)
  return int(q) & 3;
#else
  if (!(q == q)) return 0;
  if (q >= 2147483648.0f) return 3;  // INT_MAX & 3
  if (q < -2147483648.0f) return 0;  // INT_MIN & 3
  return int(q) & 3;
#endif
}

// sin/cos: Cody-Waite reduction by pi/2 with two constants (exact to ~1e-10 rad for
// |x| < 1e5; hinge angles accumulate but stay far below that), Taylor polynomials on
// [-pi/4, pi/4] (truncation < 2.5e-8), quadrant select.
QD_HD void q_sincos(float x, float* s, float* c) {
  const float q = rintf(x * 0.636619772367581343f);
  float r = fmaf(q, -1.57079637050628662109375f, x);
  r = fmaf(q, 4.37113900018624283e-8f, r);
  const float r2 = r * r;
  const float sp = fmaf(r2, fmaf(r2, fmaf(r2, fmaf(r2, 2.7557319224e-6f, -1.9841269841e-4f),
                                          8.3333333333e-3f), -1.6666666667e-1f), 0.0f);
  const float sn = fmaf(r, sp, r);
  const float cp = fmaf(r2, fmaf(r2, fmaf(r2, fmaf(r2, fmaf(r2, -2.7557319224e-7f, 2.4801587302e-5f),
                                                   -1.3888888889e-3f), 4.1666666667e-2f), -0.5f), 1.0f);
  const int qi = quadrant_of(q);
  const float a = (qi & 1) ? cp : sn;
  const float b = (qi & 1) ? sn : cp;
  *s = (qi & 2) ? -a : a;
  *c = ((qi + 1) & 2) ? -b : b;
}

// sin/cos of a prop hinge angle, which only orients that prop's drag box: on the device the
// hardware v_sin_f32 / v_cos_f32 on the angle in revolutions, reduced to [-1/2, 1/2] (error ~1e-6
// rad plus the reduction's ulp(|x| / 2pi); the float32 angle itself carries ulp(|x|)). ~5 issue
// slots instead of ~22 for q_sincos. The host instantiation keeps libm.
QD_HD void prop_sincos(float x, float* s, float* c) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r = x * 0.159154943091895336f;
  r -= rintf(r);
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
#else
  q_sincos(x, s, c);
#endif
}
QD_HD void prop_sincos(double x, double* s, double* c) { q_sincos(x, s, c); }

// atan2: odd degree-17 polynomial for atan on [0, 1] (float32 evaluation error 1.1e-7),
// octant fix-ups. Matches atan2's conventions for signed zeros and the axes.
QD_HD float q_atan2(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  const float t = mx > 0.0f ? mn * frcp(mx) : 0.0f;
  const float t2 = t * t;
  float p = 0.002456753049045801f;
  p = fmaf(p, t2, -0.01440147403627634f);
  p = fmaf(p, t2, 0.039781421422958374f);
  p = fmaf(p, t2, -0.07234875112771988f);
  p = fmaf(p, t2, 0.10498955100774765f);
  p = fmaf(p, t2, -0.14161232113838196f);
  p = fmaf(p, t2, 0.19985906779766083f);
  p = fmaf(p, t2, -0.33332598209381104f);
  p = fmaf(p, t2, 0.9999998807907104f);
  float r = p * t;
  // |y| == |x| != 0: exactly RN(pi/4), as a correctly rounded atan2 gives (the polynomial is 1 ulp
  // low there, and quat_to_euler's zero-pitch states -- pure roll / yaw -- land on it)
  r = (mn == mx && mx > 0.0f) ? 0.785398185253143310546875f : r;
  if (ay > ax) r = 1.57079632679489662f - r;
  if (copysignf(1.0f, x) < 0.0f) r = 3.14159265358979324f - r;  // atan2(y, -0) conventions too
  return copysignf(r, y);
}

// a / b for a constant b with precomputed rb = RN(1/b): Markstein's correction returns the
// correctly rounded quotient; verified exhaustively over all 2^32 float32 a for the five
// observation spans (every mismatch is a subnormal quotient, unreachable here, or the sign of a
// zero quotient: -0 comes back +0, which its only caller -- norm_obs1, v - 1 -- cannot see).
QD_HD float div_const(float a, float b, float rb) {
#pragma clang fp contract(off)
  const float q = a * rb;
  const float e = fmaf(-q, b, a);
  return fmaf(e, rb, q);
}

// np.clip semantics: NaN propagates
// (two flat selects: NaN fails both compares and passes through; lo <= hi. The nested form with an
// explicit NaN test compiled to divergent branches -- 20 exec-mask regions per step.)
template <typename T>
QD_HD T clipn(T x, T lo, T hi) {
  const T a = x < lo ? lo : x;
  return a > hi ? hi : a;
}
// mju_isBad: NaN or |x| > 1e10 (one compare with an abs modifier)
template <typename T>
QD_HD bool isbad(T x) {
  return !(q_abs(x) <= T(1e10));
}
// any(mju_isBad(x_i)). A rounded sum of non-negative terms is >= each term and NaN if any term
// is, so sum |x_i| <= 1e10 proves no x_i is bad; the per-element tests run only when that screen
// fails. (Per element, each test is a compare plus a scalar mask OR: 2 issue slots vs 1 add.)
// On the device the screen is wave-uniform (a ballot), so the exact tests sit behind a scalar
// branch the compiler cannot if-convert back into the straight-line path.
template <typename T, int N>
QD_HD bool any_bad(const T (&x)[N]) {
  T acc[4] = {q_abs(x[0]), T(0), T(0), T(0)};
#pragma unroll
  for (int i = 1; i < N; i++) acc[i & 3] += q_abs(x[i]);
  const bool ok = (acc[0] + acc[1]) + (acc[2] + acc[3]) <= T(1e10);
#if defined(__HIP_DEVICE_COMPILE__)
  if (__builtin_amdgcn_ballot_w64(!ok) == 0) return false;
#else
  if (ok) return false;
#endif
  bool b = false;
#pragma unroll
  for (int i = 0; i < N; i++) b |= isbad(x[i]);
  return b;
}

// ---------------------------------------------------------------------------------------------
template <typename T>
struct PhysConsts {
  T mt, inv_mt, cbar[3], IO[9], Ainv[9], c_ax, inv_c_ax;
  T pc[4][3], sx[4], sy[4], g5[4];
  T b_kql[3], b_kqa[3], b_kvl, b_kva;
  T p_kql[3], p_kqa[3], p_kvl, p_kva;
  T gz, dt;
  // control path (mixer, voltage, motor wrench) stays float64: four ~13 N motor forces cancel
  // to mN*m torques, which float32 cannot resolve to the 1e-5 parity bar
  double sxd[4], syd[4], g5d[4], ctrl_lo, ctrl_hi;
  double mix[16];
};

template <typename T>
struct KConsts {
  PhysConsts<T> ph;
  // float32 env constants (the reference keeps these as float32 Box bounds)
  float obs_lo[12], obs_span[12];   // span = high - low, computed in float32 like NumPy
  float obs_rspan[12];              // RN(1 / span)
  float term_lo[12], term_hi[12];
  float act_lo[4], act_span[4];
  float init_lo[12], init_span[12];
  float tgt_lo[3], tgt_span[3];
  // float64 in the reference (Python floats / float64 arrays)
  double max_thrust, vnom, vmin, vb, vl, dt;
  double rate_max, rate_ikd[3], rate_kidt, rate_imax, max_torque;
  double r_vnom, r_mx, r_max_torque;  // reciprocals (1-ulp float64 differences, far below 1e-12)
  int32_t max_steps;
  // brax kinds (float32 like the JAX reference)
  float bx_noise, bx_rpos, bx_ract, bx_vlim;
  float bx_tc[3], bx_ta[3], bx_tw[3];  // sinusoid center, amplitude, 2 pi f (float32 products)
  float bx_tdt, bx_tdur;               // linspace step dur / (L - 1), dur
  // TrajectoryFollowEnv info spline
  float sp_clo[3], sp_cspan[3], sp_amp[3], sp_dur;
};

template <typename T>
inline void make_kconsts(const QuadCfg& cfg, const PhysConstsD& d, KConsts<T>& k) {
  PhysConsts<T>& p = k.ph;
  p.mt = T(d.mt); p.inv_mt = T(d.inv_mt); p.c_ax = T(d.c_ax); p.inv_c_ax = T(d.inv_c_ax);
  for (int i = 0; i < 3; i++) {
    p.cbar[i] = T(d.cbar[i]);
    p.b_kql[i] = T(d.b_kql[i]); p.b_kqa[i] = T(d.b_kqa[i]);
    p.p_kql[i] = T(d.p_kql[i]); p.p_kqa[i] = T(d.p_kqa[i]);
  }
  for (int i = 0; i < 9; i++) { p.IO[i] = T(d.IO[i]); p.Ainv[i] = T(d.Ainv[i]); }
  for (int i = 0; i < 4; i++) {
    for (int j = 0; j < 3; j++) p.pc[i][j] = T(d.pc[i][j]);
    p.sx[i] = T(d.sx[i]); p.sy[i] = T(d.sy[i]); p.g5[i] = T(d.g5[i]);
    p.sxd[i] = d.sx[i]; p.syd[i] = d.sy[i]; p.g5d[i] = d.g5[i];
  }
  for (int i = 0; i < 16; i++) p.mix[i] = d.mix[i];
  p.b_kvl = T(d.b_kvl); p.b_kva = T(d.b_kva); p.p_kvl = T(d.p_kvl); p.p_kva = T(d.p_kva);
  p.gz = T(d.gz); p.dt = T(d.dt); p.ctrl_lo = d.ctrl_lo; p.ctrl_hi = d.ctrl_hi;
  for (int i = 0; i < 12; i++) {
    k.obs_lo[i] = cfg.obs_low[i];
    k.obs_span[i] = cfg.obs_high[i] - cfg.obs_low[i];
    k.obs_rspan[i] = 1.0f / k.obs_span[i];
    k.term_lo[i] = cfg.term_low[i];
    k.term_hi[i] = cfg.term_high[i];
    k.init_lo[i] = cfg.init_low[i];
    k.init_span[i] = cfg.init_high[i] - cfg.init_low[i];
  }
  for (int i = 0; i < 4; i++) {
    k.act_lo[i] = cfg.act_low[i];
    k.act_span[i] = cfg.act_high[i] - cfg.act_low[i];
  }
  for (int i = 0; i < 3; i++) {
    k.tgt_lo[i] = cfg.target_low[i];
    k.tgt_span[i] = cfg.target_high[i] - cfg.target_low[i];
  }
  k.max_thrust = cfg.max_motor_thrust;
  k.vnom = cfg.nominal_voltage; k.vmin = cfg.min_voltage;
  k.vb = cfg.vdrop_base; k.vl = cfg.vdrop_load; k.dt = cfg.timestep;
  k.rate_max = cfg.rate_max_rad;
  for (int i = 0; i < 3; i++) k.rate_ikd[i] = cfg.inertia[i] * cfg.rate_kd[i];
  k.rate_kidt = cfg.rate_ki * cfg.timestep;
  k.rate_imax = cfg.rate_imax;
  k.max_torque = cfg.max_torque;
  k.r_vnom = 1.0 / cfg.nominal_voltage;
  k.r_mx = 1.0 / (cfg.max_motor_thrust > 1e-6 ? cfg.max_motor_thrust : 1e-6);
  k.r_max_torque = 1.0 / cfg.max_torque;
  k.max_steps = cfg.max_episode_steps;
  k.bx_noise = cfg.reset_noise;
  k.bx_rpos = cfg.reward_pos_coef;
  k.bx_ract = cfg.reward_action_coef;
  k.bx_vlim = cfg.vel_limit;
  for (int i = 0; i < 3; i++) {
    k.bx_tc[i] = cfg.traj_center[i];
    k.bx_ta[i] = cfg.traj_amp[i];
    k.bx_tw[i] = float(2.0f * float(M_PI)) * cfg.traj_freq[i];  // (2.0 * jp.pi) * freq, float32
  }
  k.bx_tdur = cfg.traj_duration;
  for (int i = 0; i < 3; i++) {
    k.sp_clo[i] = cfg.spline_center_low[i];
    k.sp_cspan[i] = cfg.spline_center_high[i] - cfg.spline_center_low[i];
    k.sp_amp[i] = cfg.spline_amp[i];
  }
  k.sp_dur = cfg.spline_duration;
  k.bx_tdt = cfg.max_episode_steps > 1 ? cfg.traj_duration / float(cfg.max_episode_steps - 1) : 0.f;
}

// Per-env state held in registers for one step.
template <typename T>
struct EnvRegs {
  T pos[3], q[4], th[4];  // qpos
  T v[3], w[3], s[4];     // qvel
  T volt;
  T rint[3];
  float target[3];
  int32_t step;
};

struct StepRes {
  float obs[12];
  float state12[12];
  float reward;
  float motor[4];
  float vscale;
  bool term, trunc;
};

// ---------------------------------------------------------------------------------------------
// physics
template <typename T>
QD_HD void cross(const T a[3], const T b[3], T r[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}

// mj_inertiaBoxFluidModel in the body's own axes: t = -kv_a w - kq_a |w| w, f likewise
template <typename T>
QD_HD void box_drag(const T w[3], const T u[3], const T kqa[3], const T kva, const T kql[3],
                    const T kvl, T t[3], T f[3]) {
#pragma unroll
  for (int j = 0; j < 3; j++) {  // -(kv + kq |x|) x: an fma and a multiply per component
    t[j] = -(kva + kqa[j] * q_abs(w[j])) * w[j];
    f[j] = -(kvl + kql[j] * q_abs(u[j])) * u[j];
  }
}

// qacc of the free base + 4 props at (q, v, w, s, th) under the motor wrench, in two parts so
// that the part which does not depend on the controls can run before (or beside) them:
//   forward_base:   R = quat2mat(q), and the external force (base frame) / torque about the base
//                   origin (base frame) of gravity, the base inertia-box drag and the 4 prop drags,
//                   accumulated from zero in that order; the props' spin-axis drag torques Qs
//   forward_finish: + the motor wrench (total thrust along base z, torque), velocity products,
//                   3x3 solve -> vdot (world), wdot (body), sdot[4]
// Every step form (k_step_h / k_step_hd, k_step_random_h, k_step_relpos, k_rollout) calls both in
// this order, so they compute the same bits whichever wave runs the control path.
template <typename T>
struct ForceAcc {
  T R[9];
  T FB[3], tau[3], Qs[4];
};

// forward_base in pieces (same operations in the same order, so the same bits): the rotation, the
// base-frame velocity, gravity and the base drag; then each prop's drag, accumulated in prop order.
// The fused rollout spreads the pieces over the critic's MFMA issue gaps (rollout.hip).
template <typename T>
struct BaseAcc {
  ForceAcc<T> a;
  T vB[3];
};
template <typename T>
QD_HD void forward_base_begin(const PhysConsts<T>& c, const T qn[4], const T v[3], const T w[3], BaseAcc<T>& b) {
  ForceAcc<T>& o = b.a;
  // R = quat2mat(q) (q already normalized)
  const T qw = qn[0], qx = qn[1], qy = qn[2], qz = qn[3];
  T* R = o.R;
  R[0] = T(1) - T(2) * (qy * qy + qz * qz); R[1] = T(2) * (qx * qy - qw * qz); R[2] = T(2) * (qx * qz + qw * qy);
  R[3] = T(2) * (qx * qy + qw * qz); R[4] = T(1) - T(2) * (qx * qx + qz * qz); R[5] = T(2) * (qy * qz - qw * qx);
  R[6] = T(2) * (qx * qz - qw * qy); R[7] = T(2) * (qy * qz + qw * qx); R[8] = T(1) - T(2) * (qx * qx + qy * qy);
  T* vB = b.vB;
#pragma unroll
  for (int i = 0; i < 3; i++) vB[i] = R[i] * v[0] + R[3 + i] * v[1] + R[6 + i] * v[2];
  T* FB = o.FB;
  T* tau = o.tau;
  // gravity on every body COM: M g at cbar
  {
    const T mg = c.mt * c.gz;
    const T gB[3] = {mg * R[6], mg * R[7], mg * R[8]};
    cross(c.cbar, gB, tau);
#pragma unroll
    for (int i = 0; i < 3; i++) FB[i] = gB[i];
  }
  // base fluid: body frame == principal frame, COM at the origin
  {
    T t[3], f[3];
    box_drag(w, vB, c.b_kqa, c.b_kva, c.b_kql, c.b_kvl, t, f);
#pragma unroll
    for (int i = 0; i < 3; i++) { FB[i] += f[i]; tau[i] += t[i]; }
  }
}
// prop fluid: prop frame = base frame rotated by th_p about z; COM on the axis at pc_p
// (written as explicit fma chains: -ffp-contract=on fuses only within one expression, and the
// cross products, frame rotations and accumulations below are ~1/3 of the physics)
template <typename T>
QD_HD void forward_prop(const PhysConsts<T>& c, int p, T th, const T w[3], T s, BaseAcc<T>& b) {
  T* FB = b.a.FB;
  T* tau = b.a.tau;
  const T* vB = b.vB;
  T sn, cs;
  prop_sincos(th, &sn, &cs);
  const T* r = c.pc[p];
  const T ub[3] = {q_fma(w[1], r[2], q_fma(-w[2], r[1], vB[0])),  // vB + w x r
                   q_fma(w[2], r[0], q_fma(-w[0], r[2], vB[1])),
                   q_fma(w[0], r[1], q_fma(-w[1], r[0], vB[2]))};
  const T wp[3] = {q_fma(cs, w[0], sn * w[1]), q_fma(-sn, w[0], cs * w[1]), w[2] + s};
  const T up[3] = {q_fma(cs, ub[0], sn * ub[1]), q_fma(-sn, ub[0], cs * ub[1]), ub[2]};
  T tp[3], fp[3];
  box_drag(wp, up, c.p_kqa, c.p_kva, c.p_kql, c.p_kvl, tp, fp);
  const T f[3] = {q_fma(cs, fp[0], -sn * fp[1]), q_fma(sn, fp[0], cs * fp[1]), fp[2]};  // back to base
  FB[0] += f[0]; FB[1] += f[1]; FB[2] += f[2];
  // tau += r x f + Rz(th) tp
  tau[0] = q_fma(r[1], f[2], q_fma(-r[2], f[1], q_fma(cs, tp[0], q_fma(-sn, tp[1], tau[0]))));
  tau[1] = q_fma(r[2], f[0], q_fma(-r[0], f[2], q_fma(sn, tp[0], q_fma(cs, tp[1], tau[1]))));
  tau[2] = q_fma(r[0], f[1], q_fma(-r[1], f[0], tau[2] + tp[2]));
  b.a.Qs[p] = tp[2];
}

template <typename T>
QD_HD void forward_base(const PhysConsts<T>& c, const T qn[4], const T th[4], const T v[3], const T w[3],
                        const T s[4], ForceAcc<T>& o) {
  BaseAcc<T> b;
  forward_base_begin(c, qn, v, w, b);
#if defined(QD_ABL_NOPROPS)  // cost ablation (tools only): no prop drag terms
  b.a.Qs[0] = b.a.Qs[1] = b.a.Qs[2] = b.a.Qs[3] = T(0);
  if (false)
#endif
#pragma unroll
  for (int p = 0; p < 4; p++) forward_prop(c, p, th[p], w, s[p], b);
  o = b.a;
}

// The motor wrench of mj_fwdActuation for ctrl F (site transmission; float64 -> T): total thrust
// along base z and the torque about the base origin. `zero`: MuJoCo's bad-ctrl / bad-state
// handling zeroes every ctrl. F_NONNEG: the caller guarantees F >= 0 (or -0, or NaN) -- env_step's
// F * vs -- so the ctrlrange clamp's lower bound (drone.xml's fixed 0, quad_model.h) cannot bind.
template <typename T>
struct Wrench {
  T Fsum, taum[3];
};
template <typename T, bool F_NONNEG>
QD_HD Wrench<T> wrench_of(const PhysConsts<T>& c, const double Fin[4], bool zero) {
  double F[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double f = zero ? 0.0 : Fin[i];
    if (F_NONNEG)  // ctrl_lo <= 0 <= f: only the upper bound can bind
      F[i] = f > c.ctrl_hi ? c.ctrl_hi : f;
    else
      F[i] = clipn(f, c.ctrl_lo, c.ctrl_hi);  // flat selects; a NaN ctrl (CHECKS = false, the brax
                                              // kinds: mjx has no bad-ctrl zeroing) passes through
  }
  Wrench<T> wr;
  wr.Fsum = T(F[0] + F[1] + F[2] + F[3]);
  wr.taum[0] = T(c.syd[0] * F[0] + c.syd[1] * F[1] + c.syd[2] * F[2] + c.syd[3] * F[3]);
  wr.taum[1] = T(-(c.sxd[0] * F[0] + c.sxd[1] * F[1] + c.sxd[2] * F[2] + c.sxd[3] * F[3]));
  wr.taum[2] = T(c.g5d[0] * F[0] + c.g5d[1] * F[1] + c.g5d[2] * F[2] + c.g5d[3] * F[3]);
  return wr;
}

template <typename T>
QD_HD void forward_finish(const PhysConsts<T>& c, const ForceAcc<T>& a, const T w[3], const T s[4],
                          const Wrench<T>& m, T vdot[3], T wdot[3], T sdot[4]) {
  const T* R = a.R;
  const T FB[3] = {a.FB[0], a.FB[1], a.FB[2] + m.Fsum};
  const T tau[3] = {a.tau[0] + m.taum[0], a.tau[1] + m.taum[1], a.tau[2] + m.taum[2]};
  const T* Qs = a.Qs;
  // velocity-product (bias) terms
  T wc[3], wwc[3];
  cross(w, c.cbar, wc);
  cross(w, wc, wwc);
  T fv[3];
#pragma unroll
  for (int i = 0; i < 3; i++) fv[i] = FB[i] - c.mt * wwc[i];
  T Iw[3];
#pragma unroll
  for (int i = 0; i < 3; i++) Iw[i] = c.IO[3 * i] * w[0] + c.IO[3 * i + 1] * w[1] + c.IO[3 * i + 2] * w[2];
  T wIw[3];
  cross(w, Iw, wIw);
  const T ssum = s[0] + s[1] + s[2] + s[3];
  const T Qsum = Qs[0] + Qs[1] + Qs[2] + Qs[3];
  T cxf[3];
  cross(c.cbar, fv, cxf);
  T rhs[3];
  rhs[0] = tau[0] - wIw[0] - c.c_ax * ssum * w[1] - cxf[0];
  rhs[1] = tau[1] - wIw[1] + c.c_ax * ssum * w[0] - cxf[1];
  rhs[2] = tau[2] - wIw[2] - Qsum - cxf[2];
#pragma unroll
  for (int i = 0; i < 3; i++)
    wdot[i] = c.Ainv[3 * i] * rhs[0] + c.Ainv[3 * i + 1] * rhs[1] + c.Ainv[3 * i + 2] * rhs[2];
  T cxw[3];
  cross(c.cbar, wdot, cxw);
  T aB[3];
#pragma unroll
  for (int i = 0; i < 3; i++) aB[i] = fv[i] * c.inv_mt + cxw[i];
#pragma unroll
  for (int i = 0; i < 3; i++) vdot[i] = R[3 * i] * aB[0] + R[3 * i + 1] * aB[1] + R[3 * i + 2] * aB[2];
#pragma unroll
  for (int p = 0; p < 4; p++) sdot[p] = Qs[p] * c.inv_c_ax - wdot[2];
}

template <typename T>
QD_HD void normalize4(T q[4]) {
  const T n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (n2 < T(1e-30)) {
    q[0] = T(1); q[1] = q[2] = q[3] = T(0);
  } else {
    const T inv = q_rsqrt(n2);
    q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
  }
}

// mj_checkPos / mj_checkVel: a bad state (NaN / Inf / |x| > 1e10) is reset to qpos0 with zero
// qvel (mj_resetData); returns whether it was
template <typename T>
QD_HD bool check_state(EnvRegs<T>& e) {
  const T st[21] = {e.pos[0], e.pos[1], e.pos[2], e.q[0], e.q[1], e.q[2], e.q[3], e.th[0], e.th[1], e.th[2], e.th[3],
                    e.v[0], e.v[1], e.v[2], e.w[0], e.w[1], e.w[2], e.s[0], e.s[1], e.s[2], e.s[3]};
  const bool bad = any_bad(st);
  if (bad) {
#pragma unroll
    for (int i = 0; i < 3; i++) { e.pos[i] = T(0); e.v[i] = T(0); e.w[i] = T(0); }
    e.q[0] = T(1); e.q[1] = e.q[2] = e.q[3] = T(0);
#pragma unroll
    for (int i = 0; i < 4; i++) { e.th[i] = T(0); e.s[i] = T(0); }
  }
  return bad;
}

// the rest of mj_step once the state is checked and the wrench known: forward_finish,
// mj_checkAcc, mj_Euler (semi-implicit), MuJoCo's quaternion integration
template <typename T, bool CHECKS>
QD_HD void physics_finish(const PhysConsts<T>& c, EnvRegs<T>& e, T qn[4], const ForceAcc<T>& fa,
                          const Wrench<T>& m) {
  T vdot[3], wdot[3], sdot[4];
  forward_finish(c, fa, e.w, e.s, m, vdot, wdot, sdot);
  const T acc[10] = {vdot[0], vdot[1], vdot[2], wdot[0], wdot[1], wdot[2], sdot[0], sdot[1], sdot[2], sdot[3]};
  const bool badacc = any_bad(acc);
  if (CHECKS && badacc) {  // mj_checkAcc: reset to qpos0 with zero ctrl; at rest there the only force is
                 // gravity, so qacc = (0, 0, gz, 0, ...) exactly (cf. oracle K1)
#pragma unroll
    for (int i = 0; i < 3; i++) { e.pos[i] = T(0); e.v[i] = T(0); e.w[i] = T(0); vdot[i] = T(0); wdot[i] = T(0); }
    vdot[2] = c.gz;
    e.q[0] = T(1); e.q[1] = e.q[2] = e.q[3] = T(0);
#pragma unroll
    for (int i = 0; i < 4; i++) { e.th[i] = T(0); e.s[i] = T(0); sdot[i] = T(0); }
    qn[0] = T(1); qn[1] = qn[2] = qn[3] = T(0);
  }
  // mj_Euler -> mj_advance: qvel += h qacc, then positions with the new qvel
  const T h = c.dt;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    e.v[i] += h * vdot[i];
    e.w[i] += h * wdot[i];
    e.pos[i] += h * e.v[i];
  }
#pragma unroll
  for (int p = 0; p < 4; p++) {
    e.s[p] += h * sdot[p];
    e.th[p] += h * e.s[p];
  }
  // mju_quatIntegrate(quat, w, h): quat = normalize(quat) * (cos x, w/|w| sin x), x = h|w|/2.
  // For |w| < 50 rad/s the rotation uses series in x^2 (no sqrt/division; truncation < 2e-16).
  const T w2 = e.w[0] * e.w[0] + e.w[1] * e.w[1] + e.w[2] * e.w[2];
  const T x2 = T(0.25) * h * h * w2;
  T qr[4];
  if (x2 < T(0.0625)) {
    const T ch = T(1) + x2 * (T(-1.0 / 2) + x2 * (T(1.0 / 24) + x2 * (T(-1.0 / 720) + x2 * (T(1.0 / 40320) + x2 * T(-1.0 / 3628800)))));
    const T sc = T(1) + x2 * (T(-1.0 / 6) + x2 * (T(1.0 / 120) + x2 * (T(-1.0 / 5040) + x2 * (T(1.0 / 362880) + x2 * T(-1.0 / 39916800)))));
    const T k = T(0.5) * h * sc;
    qr[0] = ch; qr[1] = e.w[0] * k; qr[2] = e.w[1] * k; qr[3] = e.w[2] * k;
  } else {
    const T wn = q_sqrt(w2);
    T sh, chh;
    q_sincos(T(0.5) * h * wn, &sh, &chh);
    const T k = sh / wn;
    qr[0] = chh; qr[1] = e.w[0] * k; qr[2] = e.w[1] * k; qr[3] = e.w[2] * k;
  }
  const T a0 = qn[0], a1 = qn[1], a2 = qn[2], a3 = qn[3];
  e.q[0] = a0 * qr[0] - a1 * qr[1] - a2 * qr[2] - a3 * qr[3];
  e.q[1] = a0 * qr[1] + a1 * qr[0] + a2 * qr[3] - a3 * qr[2];
  e.q[2] = a0 * qr[2] - a1 * qr[3] + a2 * qr[0] + a3 * qr[1];
  e.q[3] = a0 * qr[3] + a1 * qr[2] - a2 * qr[1] + a3 * qr[0];
}

template <typename T>
QD_HD bool any_bad_ctrl(const double F[4]) {
  bool b = false;
#pragma unroll
  for (int i = 0; i < 4; i++) b |= isbad(F[i]);
  return b;
}

// mujoco.mj_step for one env. Fin: ctrl in float64 (may be NaN / out of range; MuJoCo semantics).
// CHECKS = false: mjx.step semantics (the brax kinds): no bad-state / bad-ctrl / bad-acc resets,
// NaN propagates. F_NONNEG: see wrench_of.
// (A speculative form -- step first, screen the loaded state afterwards -- measured slower.)
template <typename T, bool CHECKS = true, bool F_NONNEG = false>
QD_HD void physics_step(const PhysConsts<T>& c, EnvRegs<T>& e, const double Fin[4]) {
  // mj_checkPos / mj_checkVel: bad state => mj_resetData (qpos0, zero qvel, zero ctrl)
  const bool bad = CHECKS ? check_state(e) : false;
  // mj_fwdActuation: bad ctrl => all ctrl zeroed; ctrlrange clamp; site-transmission wrench
  const bool zero = CHECKS && (bad || any_bad_ctrl<T>(Fin));
  T qn[4] = {e.q[0], e.q[1], e.q[2], e.q[3]};
  normalize4(qn);
  ForceAcc<T> fa;
  forward_base(c, qn, e.th, e.v, e.w, e.s, fa);
  const Wrench<T> m = wrench_of<T, F_NONNEG>(c, Fin, zero);
  physics_finish<T, CHECKS>(c, e, qn, fa, m);
}

// ---------------------------------------------------------------------------------------------
// scipy Rotation.from_quat(xyzw).as_euler('xyz') (utils/state.py:42): Bernardes & Viollet
// from_quat's normalization is left out in float32: every angle below is a function of ratios
// (atan2, the ratio of the two hypots), so the scale of q cancels, and the raw components keep the
// terms that vanish at gimbal lock exact -- a = qw - qy and b = qx + qz of nearly equal / opposite
// operands are exact by Sterbenz, while the components of a float32-normalized q each carry a
// rounding that a / b, ~cos(pitch) / 2 there, amplified into roll / yaw by 1 / cos(pitch) (3.5e-4 rad
// at cos(pitch) = 3.3e-4). The float64 instantiation keeps scipy's normalize-first sequence.
template <typename T>
QD_HD void quat_to_euler(const T qin[4], T e[3]) {
  T qw = qin[0], qx = qin[1], qy = qin[2], qz = qin[3];
  if constexpr (sizeof(T) == 8) {
    const T inv = q_rsqrt(qw * qw + qx * qx + qy * qy + qz * qz);
    qw *= inv; qx *= inv; qy *= inv; qz *= inv;
  }
  const T a = qw - qy, b = qx + qz, c = qy + qw, d = qz - qx;
  const T PI = T(3.14159265358979323846);
  T mid = T(2) * q_atan2(q_hypot(c, d), q_hypot(a, b));
  const bool case1 = q_abs(mid) <= T(1e-7), case2 = q_abs(mid - PI) <= T(1e-7);
  const T hs = q_atan2(b, a), hd = q_atan2(d, c);
  // (selects, not branches: the if/else forms compiled to seven exec-mask regions per step)
  const bool gimbal = case1 || case2;
  const T e0g = case1 ? T(2) * hs : T(-2) * hd;
  e[0] = gimbal ? e0g : hs - hd;
  e[2] = gimbal ? T(0) : hs + hd;
  e[1] = mid - PI / T(2);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const T up = e[i] + T(2) * PI, dn = e[i] - T(2) * PI;
    e[i] = e[i] < -PI ? up : (e[i] > PI ? dn : e[i]);
  }
}

// scipy Rotation.from_euler('xyz', e).as_quat() (utils/state.py:59) -> wxyz
template <typename T>
QD_HD void euler_to_quat(const T e[3], T q[4]) {
  T sr, cr, sp, cp, sy, cy;
  q_sincos(e[0] * T(0.5), &sr, &cr);
  q_sincos(e[1] * T(0.5), &sp, &cp);
  q_sincos(e[2] * T(0.5), &sy, &cy);
  q[0] = cy * cp * cr + sy * sp * sr;
  q[1] = cy * cp * sr - sy * sp * cr;
  q[2] = cy * sp * cr + sy * cp * sr;
  q[3] = sy * cp * cr - cy * sp * sr;
}

// normalize (utils/normalization.py:7-17) in float32, no contraction, NumPy's operation order
QD_HD float norm_obs1(float x, float lo, float span, float rspan) {
#pragma clang fp contract(off)
  const float t = x - lo;
  const float u = 2.0f * t;
  const float v = div_const(u, span, rspan);
  return v - 1.0f;
}
// denormalize (utils/normalization.py:20-30) in float32
QD_HD float denorm1(float a, float lo, float span) {
#pragma clang fp contract(off)
  const float s = a + 1.0f;
  const float h = s * 0.5f;  // == s / 2.0f exactly
  const float m = h * span;
  return m + lo;
}
QD_HD float sub32(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

template <typename T>
QD_HD void observe(const KConsts<T>& k, const EnvRegs<T>& e, float obs[12], float s12[12]) {
  T eul[3];
  quat_to_euler(e.q, eul);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    s12[i] = float(e.pos[i]);
    s12[3 + i] = float(eul[i]);
    s12[6 + i] = float(e.v[i]);
    s12[9 + i] = float(e.w[i]);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const float x = i < 3 ? sub32(e.target[i], s12[i]) : s12[i];
    obs[i] = norm_obs1(x, k.obs_lo[i], k.obs_span[i], k.obs_rspan[i]);
  }
}

// reward = exp(-|pos - target|^2); the norm is NumPy's float32 sdot (products rounded to float32,
// float64 accumulation) then float32 sqrt -- see oracle/quad_oracle.c.
template <typename T>
QD_HD float reward_of(const float s12[12], const float tgt[3]) {
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float d = sub32(s12[i], tgt[i]);
    float p;
    {
#pragma clang fp contract(off)
      p = d * d;
    }
    acc += double(p);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(T) == sizeof(float)) {
    // hardware sqrt and exp2 (~1 ulp each) instead of the correctly rounded libm sequences (35
    // instructions of range scaling and class tests): reward error <= ~2e-7 * (1 + |pe|^2) relative,
    // and exp(-pe^2) is below the bar's 1e-6 absolute floor once pe^2 > 14
    const float pe = __builtin_amdgcn_sqrtf(float(acc));
    return __builtin_amdgcn_exp2f(-(pe * pe) * 1.44269504088896341f);
  }
#endif
  const T pe = T(sqrtf(float(acc)));
  return float(q_exp(-(pe * pe)));
}

template <typename T>
QD_HD bool terminated_of(const KConsts<T>& k, const float s12[12]) {
  bool t = false;
#pragma unroll
  for (int i = 0; i < 12; i++) t |= !(s12[i] >= k.term_lo[i] && s12[i] <= k.term_hi[i]);
  return t;  // a NaN fails both compares; +-Inf is outside any finite bound
}

// The control path of HoverEnv.step (float64 like the reference): RateControlWrapper.action
// (CTBR: rate command -> torques, the float32 body rate of the last observation; the integral
// state `rint` is updated), denormalize, _mix_to_motors, the voltage sag applied to the motor
// commands, and the voltage update. Depends only on the action, the voltage (and, under CTBR, the
// body rate and the integral) -- not on the rest of the state -- so k_step_h's helper waves run it
// beside the step wave's physics. F[i] = clip(mix, 0, max) * vs >= 0 (or NaN).
template <typename T>
struct Ctl {
  double F[4];  // motor commands (info["motor_commands"]), the ctrl handed to mj_step
  double vs;    // info["voltage_scale"]
  T volt;       // the updated voltage
};
template <typename T, bool CTBR>
QD_HD Ctl<T> env_control(const KConsts<T>& k, T volt, const T w[3], T rint[3], const float act[4]) {
  float a[4];
  a[0] = act[0];
  if (CTBR) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const double des = double(act[1 + j]) * k.rate_max;
      const double err = des - double(float(w[j]));  // _state.angular_velocity is float32
      const double taup = k.rate_ikd[j] * err;
      const double ri = clipn(double(rint[j]) + k.rate_kidt * err, -k.rate_imax, k.rate_imax);
      rint[j] = T(ri);
      const double tau = taup + ri;
      a[1 + j] = float(clipn(tau * k.r_max_torque, -1.0, 1.0));
    }
  } else {
    a[1] = act[1]; a[2] = act[2]; a[3] = act[3];
  }
  double phys[4];
#pragma unroll
  for (int j = 0; j < 4; j++) phys[j] = double(denorm1(a[j], k.act_lo[j], k.act_span[j]));
  Ctl<T> c;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double s = k.ph.mix[4 * i] * phys[0] + k.ph.mix[4 * i + 1] * phys[1] +
                     k.ph.mix[4 * i + 2] * phys[2] + k.ph.mix[4 * i + 3] * phys[3];
    c.F[i] = clipn(s, 0.0, k.max_thrust);
  }
  c.vs = clipn(double(volt) * k.r_vnom, 0.0, 1.0);
  // hover_env.py:175 clips F * vs to [0, max_thrust * vs]; that clip never binds here: F is in
  // [0, max_thrust] (or NaN) after the clip above, vs in [0, 1] (or NaN), max_thrust >= 0 (checked
  // by quad_create), and a rounded product with the same non-negative vs is monotone in F
  // (F * vs <= max_thrust * vs); NaN passes either way.
#pragma unroll
  for (int i = 0; i < 4; i++) c.F[i] = c.F[i] * c.vs;
  const double load = ((c.F[0] + c.F[1] + c.F[2] + c.F[3]) * 0.25) * k.r_mx;
  const double dV = (k.vb + k.vl * load) * k.dt;
  c.volt = T(clipn(double(volt) - dV, k.vmin, k.vnom));
  return c;
}

// After mj_step: step count, QuadState + observation, reward, termination, truncation.
template <typename T>
QD_HD void env_post(const KConsts<T>& k, EnvRegs<T>& e, StepRes& r) {
  e.step += 1;
#if defined(QD_ABL_NOOBS)
#pragma unroll
  for (int i = 0; i < 3; i++) {
    r.state12[i] = float(e.pos[i]); r.state12[3 + i] = float(e.q[1 + i]);
    r.state12[6 + i] = float(e.v[i]); r.state12[9 + i] = float(e.w[i]);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) r.obs[i] = r.state12[i];
#else
  observe(k, e, r.obs, r.state12);
#endif
  r.reward = reward_of<T>(r.state12, e.target);
  r.term = terminated_of(k, r.state12);
  r.trunc = e.step >= k.max_steps;
}

// (RateControlWrapper.action ->) HoverEnv.step for one env: env_control, mujoco.mj_step
// (physics_step, the rigid-body dynamics in T), env_post.
template <typename T, bool CTBR>
QD_HD void env_step(const KConsts<T>& k, EnvRegs<T>& e, const float act[4], StepRes& r,
                    uint64_t* stamps = nullptr) {
  const Ctl<T> c = env_control<T, CTBR>(k, e.volt, e.w, e.rint, act);
  e.volt = c.volt;
  if (stamps) { QD_PIN_N(c.F, 4); QD_PIN(e.volt); }
  QD_STAMP(stamps, 2);
  // QD_ABL_*: cost-ablation builds of tools/step_variants.py only (never defined in the product)
#if defined(QD_ABL_PHYS2)
  physics_step<T, true, true>(k.ph, e, c.F);
  physics_step<T, true, true>(k.ph, e, c.F);
#elif !defined(QD_ABL_NOPHYS)
  physics_step<T, true, true>(k.ph, e, c.F);  // F = clip(., 0, max) * vs >= 0 (or NaN)
#endif
  if (stamps) { QD_PIN_N(e.pos, 3); QD_PIN_N(e.q, 4); QD_PIN_N(e.th, 4); QD_PIN_N(e.v, 3); QD_PIN_N(e.w, 3); QD_PIN_N(e.s, 4); }
  QD_STAMP(stamps, 3);
  env_post(k, e, r);
  if (stamps) { QD_PIN_N(r.obs, 12); QD_PIN_N(r.state12, 12); }
  QD_STAMP(stamps, 4);
#pragma unroll
  for (int i = 0; i < 4; i++) r.motor[i] = float(c.F[i]);
  r.vscale = float(c.vs);
  if (stamps) { QD_PIN(r.reward); QD_PIN(uint32_t(r.term)); QD_PIN(uint32_t(r.trunc)); QD_PIN_N(r.motor, 4); }
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011) and the reset / action draws
QD_HD void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = uint64_t(0xD2511F53u) * c[0];
    const uint64_t p1 = uint64_t(0xCD9E8D57u) * c[2];
    const uint32_t n0 = uint32_t(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = uint32_t(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = uint32_t(p1); c[2] = n2; c[3] = uint32_t(p0);
  }
}
QD_HD float u01(uint32_t x) { return float(x >> 8) * 0x1p-24f; }
QD_HD float affine32(float lo, float u, float span) {
#pragma clang fp contract(off)
  const float m = u * span;
  return lo + m;
}

// Draws for HoverEnv.reset: 12 init-state values then 3 target values (QuadState.random_reset +
// the target draw, hover_env.py:219-228), Philox-keyed by (seed; global env id, episode, block):
// word j of the draw is word j % 4 of block j / 4.
QD_HD void reset_block(uint64_t seed, uint64_t gid, uint32_t episode, uint32_t blk, uint32_t c[4]) {
  c[0] = uint32_t(gid); c[1] = uint32_t(gid >> 32); c[2] = episode; c[3] = blk;
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
}
// (from the uniforms u = u01(word); the wave-compacted kernels convert where the words are made)
QD_HD void reset_affine_u(const float init_lo[12], const float init_span[12], const float tgt_lo[3],
                          const float tgt_span[3], const float u[16], float init12[12], float tgt[3]) {
#pragma unroll
  for (int i = 0; i < 12; i++) init12[i] = affine32(init_lo[i], u[i], init_span[i]);
#pragma unroll
  for (int i = 0; i < 3; i++) tgt[i] = affine32(tgt_lo[i], u[12 + i], tgt_span[i]);
}
QD_HD void reset_affine(const float init_lo[12], const float init_span[12], const float tgt_lo[3],
                        const float tgt_span[3], const uint32_t r[16], float init12[12], float tgt[3]) {
  float u[16];
#pragma unroll
  for (int i = 0; i < 16; i++) u[i] = u01(r[i]);
  reset_affine_u(init_lo, init_span, tgt_lo, tgt_span, u, init12, tgt);
}
QD_HD void reset_draw(const float init_lo[12], const float init_span[12], const float tgt_lo[3],
                      const float tgt_span[3], uint64_t seed, uint64_t gid, uint32_t episode,
                      float init12[12], float tgt[3]) {
  uint32_t r[16];
#pragma unroll
  for (uint32_t blk = 0; blk < 4; blk++) reset_block(seed, gid, episode, blk, r + 4 * blk);
  reset_affine(init_lo, init_span, tgt_lo, tgt_span, r, init12, tgt);
}

// HoverEnv.reset / TrajectoryFollowEnv.reset given the draws; writes the reset obs.
template <typename T, int KIND>
QD_HD void env_reset_from(const KConsts<T>& k, EnvRegs<T>& e, const float init12[12],
                          const float tgt[3], float obs[12], float s12[12]) {
  T eul[3] = {T(init12[3]), T(init12[4]), T(init12[5])};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    e.pos[i] = T(init12[i]);
    e.v[i] = T(init12[6 + i]);
    e.w[i] = T(init12[9 + i]);
    e.rint[i] = T(0);
    // TrajectoryFollowEnv: target = traj_pos[0] = start position (trajectory_follow_env.py:242-243)
    e.target[i] = KIND == QUAD_ENV_TRAJ ? init12[i] : tgt[i];
  }
  euler_to_quat(eul, e.q);
#pragma unroll
  for (int p = 0; p < 4; p++) { e.th[p] = T(0); e.s[p] = T(0); }
  e.volt = T(k.vnom);
  e.step = 0;
  // QuadState.set_from_mujoco(get_mujoco_state()) returns the drawn attitude: use it directly
#pragma unroll
  for (int i = 0; i < 12; i++) s12[i] = init12[i];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const float x = i < 3 ? sub32(e.target[i], s12[i]) : s12[i];
    obs[i] = norm_obs1(x, k.obs_lo[i], k.obs_span[i], k.obs_rspan[i]);
  }
}

// ---------------------------------------------------------------------------------------------
// brax kinds (train_brax_ppo.py). Step: QuadHoverBraxEnv.step (:131-173) / JaxMJXQuadBraxEnv.step
// (:300-356) for one env; obs21 = [qpos, qvel] (:175-176, :365-366). `term` = the env's done.
template <typename T, int KIND>
QD_HD void brax_step(const KConsts<T>& k, EnvRegs<T>& e, const float act[4], float obs21[21],
                     float& reward, bool& term, bool& trunc, float motor[4]) {
  // (action + 1) * 0.5 * (max - min) + min, clipped (float32 elementwise like JAX, no FMA
  // contraction; jnp.clip keeps NaN). The mixer then runs in float64: four ~13 N motor forces
  // cancel to mN*m torques, where float32 rounding alone would exceed the 1e-5 parity bar.
  float u[4];
  {
#pragma clang fp contract(off)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const float lo = k.act_lo[j], hi = lo + k.act_span[j];
      const float p = (act[j] + 1.0f) * 0.5f * k.act_span[j] + lo;
      u[j] = p < lo ? lo : (p > hi ? hi : p);
    }
  }
  double F[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double s = k.ph.mix[4 * i] * double(u[0]) + k.ph.mix[4 * i + 1] * double(u[1]) +
                     k.ph.mix[4 * i + 2] * double(u[2]) + k.ph.mix[4 * i + 3] * double(u[3]);
    F[i] = s < 0.0 ? 0.0 : (s > k.max_thrust ? k.max_thrust : s);
    motor[i] = float(F[i]);
  }
  physics_step<T, false>(k.ph, e, F);
  e.step += 1;
  const float pos[3] = {float(e.pos[0]), float(e.pos[1]), float(e.pos[2])};
  float tgt[3] = {e.target[0], e.target[1], e.target[2]};
  if (KIND == QUAD_ENV_BRAX_TRAJ) {
    // info["step_count"] lives in rint[0] (a float counter; brax's AutoResetWrapper never resets it)
    const float cnt = float(e.rint[0]) + 1.0f;
    e.rint[0] = T(cnt);
    const float lastf = float(k.max_steps - 1);
    const float idx = cnt < lastf ? cnt : lastf;
    const float t = idx == lastf ? k.bx_tdur : idx * k.bx_tdt;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      float sn, cs;
      q_sincos(k.bx_tw[i] * t, &sn, &cs);
      tgt[i] = k.bx_tc[i] + k.bx_ta[i] * sn;
      e.target[i] = tgt[i];
    }
  }
  obs21[0] = pos[0]; obs21[1] = pos[1]; obs21[2] = pos[2];
#pragma unroll
  for (int i = 0; i < 4; i++) { obs21[3 + i] = float(e.q[i]); obs21[7 + i] = float(e.th[i]); }
#pragma unroll
  for (int i = 0; i < 3; i++) { obs21[11 + i] = float(e.v[i]); obs21[14 + i] = float(e.w[i]); }
#pragma unroll
  for (int i = 0; i < 4; i++) obs21[17 + i] = float(e.s[i]);
  float d2 = 0.f;
#pragma unroll
  for (int i = 0; i < 3; i++) { const float d = pos[i] - tgt[i]; d2 += d * d; }
  const float per = fsqrt(d2);
  const bool oxy = q_abs(pos[0]) > k.term_hi[0] || q_abs(pos[1]) > k.term_hi[1];
  const bool oz = pos[2] < k.term_lo[2] || pos[2] > k.term_hi[2];
  if (KIND == QUAD_ENV_BRAX_TRAJ) {
    bool fin = true;
#pragma unroll
    for (int i = 0; i < 21; i++) fin &= q_abs(obs21[i]) <= 3.4028235e38f;  // isfinite (NaN fails)
    bool ov = false;
#pragma unroll
    for (int i = 0; i < 3; i++) ov |= q_abs(obs21[11 + i]) > k.bx_vlim;
    const bool valid = fin && !oxy && !oz && !ov;
    const float pe = (valid && q_abs(per) <= 3.4028235e38f) ? per : 1e3f;
    float asq = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j++) asq += act[j] * act[j];
    const float rr = q_exp(-k.bx_rpos * pe * pe) - k.bx_ract * asq;
    reward = (valid && q_abs(rr) <= 3.4028235e38f) ? rr : -1.0f;
    term = !valid;
#pragma unroll
    for (int i = 0; i < 21; i++) obs21[i] = q_abs(obs21[i]) <= 3.4028235e38f ? obs21[i] : 0.f;
  } else {
    reward = q_exp(-k.bx_rpos * per * per);
    term = oxy || oz;  // NaN compares false: QuadHoverBraxEnv has no NaN guard
  }
  trunc = e.step >= k.max_steps;  // EpisodeWrapper
}

// brax reset draw: 21 x U(-noise, noise) from Philox(seed; gid, episode, 0x300 + block)
QD_HD void brax_reset_draw(float noise, uint64_t seed, uint64_t gid, uint32_t episode, float u21[21]) {
  uint32_t r[24];
#pragma unroll
  for (uint32_t blk = 0; blk < 6; blk++) {
    uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), episode, 0x300u + blk};
    philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
    r[4 * blk] = c[0]; r[4 * blk + 1] = c[1]; r[4 * blk + 2] = c[2]; r[4 * blk + 3] = c[3];
  }
#pragma unroll
  for (int i = 0; i < 21; i++) u21[i] = affine32(-noise, u01(r[i]), 2.0f * noise);
}

// QuadHoverBraxEnv.reset (:102-129) / JaxMJXQuadBraxEnv.reset (:255-294) from the draw.
// keep_counter: AutoResetWrapper restore (the env's step_count carries on).
template <typename T, int KIND>
QD_HD void brax_reset_from(const KConsts<T>& k, EnvRegs<T>& e, const float u21[21], float obs21[21],
                           bool keep_counter) {
  const float z0 = KIND == QUAD_ENV_BRAX_TRAJ ? 1.0f : 0.0f;
  float q[11] = {0.f, 0.f, z0, 1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 11; i++) q[i] = q[i] + u21[i];
  if (KIND == QUAD_ENV_BRAX_TRAJ) {
    const float n = fsqrt(q[3] * q[3] + q[4] * q[4] + q[5] * q[5] + q[6] * q[6]) + 1e-8f;
#pragma unroll
    for (int i = 3; i < 7; i++) q[i] = q[i] / n;
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    e.pos[i] = T(q[i]);
    e.v[i] = T(u21[11 + i]);
    e.w[i] = T(u21[14 + i]);
    e.target[i] = KIND == QUAD_ENV_BRAX_HOVER ? k.tgt_lo[i] : k.bx_tc[i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    e.q[i] = T(q[3 + i]);
    e.th[i] = T(q[7 + i]);
    e.s[i] = T(u21[17 + i]);
  }
  e.volt = T(0);
  if (!keep_counter) { e.rint[0] = T(0); }
  e.rint[1] = e.rint[2] = T(0);
  e.step = 0;
#pragma unroll
  for (int i = 0; i < 11; i++) obs21[i] = q[i];
#pragma unroll
  for (int i = 0; i < 10; i++) obs21[11 + i] = u21[11 + i];
}

// ---------------------------------------------------------------------------------------------
// TrajectoryFollowEnv info["target"/"target_vel"/"target_acc"] (trajectory_follow_env.py:163-168,
// :175-216, :234-243): waypoints from Philox blocks 4..8 of the episode's reset counter (block 4:
// center, n_wp; blocks 5..8: per-axis offsets, axis a uses values 5a..5a+n_wp-1), first waypoint =
// start position, natural cubic spline in float64 (scipy CubicSpline bc_type="natural"), sampled
// at t = linspace(0, duration, L)[min(step - 1, L - 1)].
template <typename T>
QD_HD void traj_spline_info(const KConsts<T>& k, uint64_t seed, uint64_t gid, uint32_t episode,
                            const float start[3], int32_t step, float out9[9]) {
  uint32_t r[20];
#pragma unroll
  for (uint32_t blk = 0; blk < 5; blk++) {
    uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), episode, 4u + blk};
    philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
    r[4 * blk] = c[0]; r[4 * blk + 1] = c[1]; r[4 * blk + 2] = c[2]; r[4 * blk + 3] = c[3];
  }
  const int nwp = 3 + int((uint64_t(r[3] >> 8) * 3u) >> 24);  // integers(3, 6)
  const int L = k.max_steps;
  const int idx = (step - 1) < (L - 1) ? (step - 1 < 0 ? 0 : step - 1) : L - 1;
  const double Td = double(k.sp_dur);
  const double t = idx == L - 1 ? Td : double(idx) * (Td / double(L > 1 ? L - 1 : 1));
  const double h = Td / double(nwp - 1);
  int seg = int(t / h);
  seg = seg < 0 ? 0 : (seg > nwp - 2 ? nwp - 2 : seg);
  const double a = double(seg + 1) * h - t, b = t - double(seg) * h;  // t_{k+1} - t, t - t_k
#pragma unroll
  for (int ax = 0; ax < 3; ax++) {
    const double center = double(affine32(k.sp_clo[ax], u01(r[ax]), k.sp_cspan[ax]));
    double y[5];
    for (int i = 0; i < 5; i++)
      y[i] = center + double(affine32(-k.sp_amp[ax], u01(r[4 + 5 * ax + i]), 2.0f * k.sp_amp[ax]));
    y[0] = double(start[ax]);
    // natural spline second derivatives: M_0 = M_{n-1} = 0, M_{i-1} + 4 M_i + M_{i+1} = 6 d2y_i / h^2
    double M[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    const double s6 = 6.0 / (h * h);
    if (nwp == 3) {
      M[1] = s6 * (y[2] - 2.0 * y[1] + y[0]) / 4.0;
    } else {
      // Thomas algorithm on the (nwp - 2) interior unknowns
      double cp[3], dp[3];
      const int m = nwp - 2;
      for (int i = 0; i < m; i++) {
        const double d = s6 * (y[i + 2] - 2.0 * y[i + 1] + y[i]);
        const double den = i == 0 ? 4.0 : 4.0 - cp[i - 1];
        cp[i] = 1.0 / den;
        dp[i] = (d - (i == 0 ? 0.0 : dp[i - 1])) / den;
      }
      M[m] = dp[m - 1];
      for (int i = m - 2; i >= 0; i--) M[i + 1] = dp[i] - cp[i] * M[i + 2];
    }
    const double Mk = M[seg], Mk1 = M[seg + 1], yk = y[seg], yk1 = y[seg + 1];
    const double pos = Mk * a * a * a / (6.0 * h) + Mk1 * b * b * b / (6.0 * h) +
                       (yk / h - Mk * h / 6.0) * a + (yk1 / h - Mk1 * h / 6.0) * b;
    const double vel = -Mk * a * a / (2.0 * h) + Mk1 * b * b / (2.0 * h) - (yk / h - Mk * h / 6.0) +
                       (yk1 / h - Mk1 * h / 6.0);
    const double acc = Mk * a / h + Mk1 * b / h;
    out9[ax] = float(pos);
    out9[3 + ax] = float(vel);
    out9[6 + ax] = float(acc);
  }
}

}  // namespace quadenv
