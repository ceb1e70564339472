// quad_model.h -- the drone model (model/drone/drone.xml) reduced to the constants the
// structured step needs, precomputed in double on the host when a handle is created.
//
// Why a reduced model is exact: each prop body is axisymmetric about its hinge axis with its
// COM on that axis (drone.xml:54,59,64,69: inertial pos (0,0,d), quat (.5,.5,-.5,.5) maps the
// principal axis of the 3.75335e-6 moment onto the hinge z, the other two moments are equal).
// Hence every prop's inertia, seen from the base frame, is independent of its hinge angle, the
// gyroscopic term on each hinge vanishes, and the 10x10 mass matrix reduces (Schur complement
// over the four hinge dofs) to a *constant* 3x3 body-frame matrix A = I_com - 4 c_ax z z^T
// whose inverse is precomputed here. The hinge angle survives only in the props' inertia-box
// fluid drag, which is not rotation invariant. make_phys_consts() verifies those structural
// assumptions and refuses the model otherwise (QUAD_EMODEL).
#pragma once

#include <cmath>
#include <cstring>

#include "../../include/quadenv.h"

namespace quadenv {

// The reference defaults for (env_kind, wrapper), arguments already validated (quad_default_cfg in
// quadenv.hip; also the build-time generator of the specialized constant blocks, gen_kconsts.cpp):
// HoverEnv.__init__ (hover_env.py:15-100), TrajectoryFollowEnv.__init__ (trajectory_follow_env.py:
// 22-104), RateControlWrapper.__init__ (rate_wrapper.py:40-64) with pid_gains.json:43-52,
// drone_config.py:9-22, drone.xml:4, and the brax kinds' train_brax_ppo.py defaults.
inline void default_cfg_fill(int32_t env_kind, int32_t wrapper, QuadCfg* c) {
  std::memset(c, 0, sizeof *c);
  c->env_kind = env_kind;
  c->wrapper = wrapper;
  c->auto_reset = 1;
  const double pi = M_PI;
  // HoverEnv._obs_bounds (hover_env.py:36-39) / _state_bounds (:54-57) share the angle/vel rows
  const double ol[12] = {-4, -4, -2, -pi, -pi, -pi, -10, -10, -10, -6 * pi, -6 * pi, -6 * pi};
  // _initial_state_bounds (hover_env.py:42-45; trajectory_follow_env.py:49-52)
  const double il[12] = {-1.5, -1.5, 0.1, -0.3, -0.3, -0.3, -0.5, -0.5, -0.5, -0.5, -0.5, -0.5};
  const double ih[12] = {1.5, 1.5, 1.5, 0.3, 0.3, 0.3, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5};
  for (int i = 0; i < 12; i++) {
    c->obs_low[i] = float(ol[i]);
    c->obs_high[i] = float(-ol[i]);
    c->init_low[i] = float(il[i]);
    c->init_high[i] = float(ih[i]);
    c->term_low[i] = float(ol[i]);
    c->term_high[i] = float(-ol[i]);
  }
  const double xy = env_kind == QUAD_ENV_TRAJ ? 3.0 : 2.0;  // traj :60-63, hover :54-57
  c->term_low[0] = float(-xy); c->term_low[1] = float(-xy); c->term_low[2] = 0.f;
  c->term_high[0] = float(xy); c->term_high[1] = float(xy); c->term_high[2] = float(xy);
  c->max_episode_steps = env_kind == QUAD_ENV_TRAJ ? 2048 : 512;
  c->nominal_voltage = env_kind == QUAD_ENV_TRAJ ? 16.8 : 8.4;
  c->min_voltage = env_kind == QUAD_ENV_TRAJ ? 13.2 : 7.6;
  const float tl[3] = {-1.5f, -1.5f, 0.3f}, th[3] = {1.5f, 1.5f, 1.8f};  // hover_env.py:48-51
  for (int i = 0; i < 3; i++) { c->target_low[i] = tl[i]; c->target_high[i] = th[i]; }
  c->max_motor_thrust = 13.0;  // drone_config.py:9-11,21
  c->arm_length = 0.039799;
  c->yaw_coeff = 0.0201;
  c->max_torque = 0.5;
  const float al[4] = {0.f, -0.5f, -0.5f, -0.5f}, ah[4] = {52.f, 0.5f, 0.5f, 0.5f};  // :60-65
  for (int i = 0; i < 4; i++) { c->act_low[i] = al[i]; c->act_high[i] = ah[i]; }
  c->vdrop_base = 0.01;
  c->vdrop_load = 0.08;
  c->rate_max_rad = 360.0 * (M_PI / 180.0);  // rate_wrapper.py:52, pid_gains.json:43-52
  c->rate_kd[0] = 26; c->rate_kd[1] = 26; c->rate_kd[2] = 18;
  c->rate_ki = 0.025;
  c->rate_imax = 0.01;
  c->inertia[0] = 4.16e-4; c->inertia[1] = 4.23e-4; c->inertia[2] = 5.37e-4;
  c->timestep = 0.01;  // drone.xml:4
  c->gravity[2] = -9.81;
  c->density = 1.225;
  c->viscosity = 1.8e-5;
  {  // TrajectoryFollowEnv spline (trajectory_follow_env.py:25, :55-58, :199-203)
    const float lo[3] = {-1.f, -1.f, 0.4f}, hi[3] = {1.f, 1.f, 1.4f}, amp[3] = {0.6f, 0.6f, 0.4f};
    for (int i = 0; i < 3; i++) {
      c->spline_center_low[i] = lo[i]; c->spline_center_high[i] = hi[i]; c->spline_amp[i] = amp[i];
    }
    c->spline_duration = 30.f;
  }
  if (env_kind >= QUAD_ENV_BRAX_HOVER) {  // train_brax_ppo.py
    const bool traj = env_kind == QUAD_ENV_BRAX_TRAJ;
    c->max_episode_steps = 500;                        // --episode-length (:436)
    for (int i = 0; i < 3; i++) { c->target_low[i] = c->target_high[i] = i == 2 ? 1.f : 0.f; }  // (:55)
    c->term_low[0] = c->term_low[1] = -3.f; c->term_high[0] = c->term_high[1] = 3.f;  // (:48-50)
    c->term_low[2] = 0.02f; c->term_high[2] = 4.f;
    c->reset_noise = 0.01f;                            // (:105-116, :271-272)
    c->reward_pos_coef = traj ? 1.f : 2.f;             // (:146 / :338)
    c->reward_action_coef = traj ? 0.001f : 0.f;       // (:339)
    c->vel_limit = traj ? 20.f : 0.f;                  // (:190)
    const float cen[3] = {0.f, 0.f, 1.f}, amp[3] = {0.5f, 0.5f, 0.2f}, fr[3] = {0.2f, 0.15f, 0.1f};
    for (int i = 0; i < 3; i++) { c->traj_center[i] = cen[i]; c->traj_amp[i] = amp[i]; c->traj_freq[i] = fr[i]; }
    c->traj_duration = 5.f;                            // --traj-duration-seconds (:444)
  }
}

struct ModelData {
  // base_link (drone.xml:34-52): free joint, inertial at origin
  double m0 = 0.195;
  double I0[3] = {4.16e-4, 4.23e-4, 5.37e-4};
  // props (drone.xml:53-72)
  double prop_pos[4][3] = {{0.039799, -0.039799, 0.0336},
                           {-0.039799, -0.039799, 0.032484},
                           {-0.039799, 0.039799, 0.033094},
                           {0.039799, 0.039799, 0.0336}};
  double prop_ipos_z[4] = {-0.001, 0.000116422, -0.000494174, -0.001};
  double prop_iquat[4] = {0.5, 0.5, -0.5, 0.5};
  double mp = 0.00693608;
  double Ip[3] = {3.75335e-06, 1.87898e-06, 1.87898e-06};
  // motors on sites thrust1..4 == prop positions (drone.xml:73-76, 81-84)
  double gear5[4] = {0.0201, -0.0201, 0.0201, -0.0201};
  double ctrl_lo = 0.0, ctrl_hi = 13.0;  // ctrlrange (drone.xml:9), autolimits (:2); ctrl_lo <= 0 is
                                         // assumed by physics_step<.., F_NONNEG = true>
};

// Everything the kernel needs, in double; cast to float for the device.
struct PhysConstsD {
  double mt, inv_mt;           // total mass
  double cbar[3];              // system COM in the base frame
  double IO[9];                // total inertia about the base origin, base frame
  double Ainv[9];              // (I_com - 4 c_ax z z^T)^-1
  double c_ax, inv_c_ax;       // prop axial inertia
  double pc[4][3];             // prop COMs in the base frame
  double sx[4], sy[4], g5[4];  // motor sites and yaw gear
  double b_kql[3], b_kqa[3], b_kvl, b_kva;  // base inertia-box drag (principal == base frame)
  double p_kql[3], p_kqa[3], p_kvl, p_kva;  // prop drag, expressed on prop-frame axes x', y', z
  double gz;                   // gravity z
  double dt;
  double ctrl_lo, ctrl_hi;
  double mix[16];              // np.linalg.inv(A) of the mixer (hover_env.py:94-100)
};

inline void quat2mat_d(const double q[4], double R[9]) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}

inline bool inv3_d(const double A[9], double out[9]) {
  const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8],
               c02 = A[3] * A[7] - A[4] * A[6];
  const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
  if (!(std::fabs(det) > 0)) return false;
  const double id = 1.0 / det;
  out[0] = c00 * id; out[1] = (A[2] * A[7] - A[1] * A[8]) * id; out[2] = (A[1] * A[5] - A[2] * A[4]) * id;
  out[3] = c01 * id; out[4] = (A[0] * A[8] - A[2] * A[6]) * id; out[5] = (A[2] * A[3] - A[0] * A[5]) * id;
  out[6] = c02 * id; out[7] = (A[1] * A[6] - A[0] * A[7]) * id; out[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  return true;
}

// inertia-box equivalent dimensions (mj_inertiaBoxFluidModel)
inline void fluid_box(const double I[3], double m, double box[3]) {
  box[0] = std::sqrt(std::fmax(1e-15, I[1] + I[2] - I[0]) / m * 6.0);
  box[1] = std::sqrt(std::fmax(1e-15, I[0] + I[2] - I[1]) / m * 6.0);
  box[2] = std::sqrt(std::fmax(1e-15, I[0] + I[1] - I[2]) / m * 6.0);
}

inline void fluid_coeffs(const double box[3], double rho, double mu, double kql[3],
                         double kqa[3], double* kvl, double* kva) {
  const double d = (box[0] + box[1] + box[2]) / 3.0;
  *kvl = mu > 0 ? 3.0 * M_PI * d * mu : 0.0;
  *kva = mu > 0 ? M_PI * d * d * d * mu : 0.0;
  const double b4[3] = {std::pow(box[0], 4), std::pow(box[1], 4), std::pow(box[2], 4)};
  for (int j = 0; j < 3; j++) {
    const int k = (j + 1) % 3, l = (j + 2) % 3;
    kql[j] = rho > 0 ? 0.5 * rho * box[k] * box[l] : 0.0;
    kqa[j] = rho > 0 ? rho * box[j] * (b4[k] + b4[l]) / 64.0 : 0.0;
  }
}

// Returns false (and a reason) if the structural assumptions do not hold.
inline bool make_phys_consts(const QuadCfg& cfg, PhysConstsD& c, const char** why) {
  const ModelData md;
  std::memset(&c, 0, sizeof c);
  // prop principal frame in the prop body frame: P = R(iquat); principal axis j -> axis ax[j]
  double P[9];
  quat2mat_d(md.prop_iquat, P);
  int ax[3];
  double Ipf[3] = {0, 0, 0};
  for (int j = 0; j < 3; j++) {
    ax[j] = -1;
    for (int i = 0; i < 3; i++)
      if (std::fabs(std::fabs(P[3 * i + j]) - 1.0) < 1e-12) ax[j] = i;
    if (ax[j] < 0) { *why = "prop inertial frame is not axis-aligned with the hinge frame"; return false; }
    Ipf[ax[j]] = md.Ip[j];
  }
  if (Ipf[0] != Ipf[1]) { *why = "prop inertia is not axisymmetric about the hinge axis"; return false; }
  c.c_ax = Ipf[2];
  c.inv_c_ax = 1.0 / c.c_ax;
  c.mt = md.m0 + 4 * md.mp;
  c.inv_mt = 1.0 / c.mt;
  for (int i = 0; i < 4; i++) {
    c.pc[i][0] = md.prop_pos[i][0];
    c.pc[i][1] = md.prop_pos[i][1];
    c.pc[i][2] = md.prop_pos[i][2] + md.prop_ipos_z[i];
    c.sx[i] = md.prop_pos[i][0];
    c.sy[i] = md.prop_pos[i][1];
    c.g5[i] = md.gear5[i];
    for (int k = 0; k < 3; k++) c.cbar[k] += md.mp * c.pc[i][k];
  }
  for (int k = 0; k < 3; k++) c.cbar[k] /= c.mt;
  // I_O = I0 + sum_i [ Ip_frame + mp (|c_i|^2 I - c_i c_i^T) ]
  double IO[9] = {md.I0[0], 0, 0, 0, md.I0[1], 0, 0, 0, md.I0[2]};
  for (int i = 0; i < 4; i++) {
    const double* r = c.pc[i];
    const double rr = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    for (int a = 0; a < 3; a++) {
      IO[4 * a] += Ipf[a];
      for (int b = 0; b < 3; b++) IO[3 * a + b] += md.mp * ((a == b ? rr : 0.0) - r[a] * r[b]);
    }
  }
  std::memcpy(c.IO, IO, sizeof IO);
  const double* cb = c.cbar;
  const double cc = cb[0] * cb[0] + cb[1] * cb[1] + cb[2] * cb[2];
  double A[9];
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) A[3 * a + b] = IO[3 * a + b] - c.mt * ((a == b ? cc : 0.0) - cb[a] * cb[b]);
  A[8] -= 4 * c.c_ax;
  if (!inv3_d(A, c.Ainv)) { *why = "singular reduced inertia"; return false; }
  // fluid
  double box[3];
  fluid_box(md.I0, md.m0, box);
  fluid_coeffs(box, cfg.density, cfg.viscosity, c.b_kql, c.b_kqa, &c.b_kvl, &c.b_kva);
  double pkql[3], pkqa[3];
  fluid_box(md.Ip, md.mp, box);
  fluid_coeffs(box, cfg.density, cfg.viscosity, pkql, pkqa, &c.p_kvl, &c.p_kva);
  for (int j = 0; j < 3; j++) { c.p_kql[ax[j]] = pkql[j]; c.p_kqa[ax[j]] = pkqa[j]; }
  if (cfg.gravity[0] != 0 || cfg.gravity[1] != 0) { *why = "only vertical gravity is supported"; return false; }
  c.gz = cfg.gravity[2];
  c.dt = cfg.timestep;
  c.ctrl_lo = md.ctrl_lo;
  c.ctrl_hi = md.ctrl_hi;
  // env_step and k_rollout clamp the (non-negative) motor forces with physics_step<.., F_NONNEG>,
  // which applies only the upper ctrlrange bound: that is exact only while ctrl_lo <= 0
  if (!(c.ctrl_lo <= 0.0 && c.ctrl_hi >= c.ctrl_lo)) { *why = "ctrlrange must satisfy lo <= 0 <= hi"; return false; }
  // mixer inverse (Gauss-Jordan, partial pivoting) of A = [[1,1,1,1],[-l,-l,l,l],[-l,l,l,-l],[k,-k,k,-k]]
  const double l = cfg.arm_length, k = cfg.yaw_coeff;
  double M[4][8] = {{1, 1, 1, 1}, {-l, -l, l, l}, {-l, l, l, -l}, {k, -k, k, -k}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) M[i][4 + j] = (i == j);
  for (int col = 0; col < 4; col++) {
    int piv = col;
    for (int r = col + 1; r < 4; r++)
      if (std::fabs(M[r][col]) > std::fabs(M[piv][col])) piv = r;
    for (int j = 0; j < 8; j++) std::swap(M[col][j], M[piv][j]);
    const double d = M[col][col];
    if (!(std::fabs(d) > 0)) { *why = "singular mixer"; return false; }
    for (int j = 0; j < 8; j++) M[col][j] /= d;
    for (int r = 0; r < 4; r++)
      if (r != col) {
        const double f = M[r][col];
        for (int j = 0; j < 8; j++) M[r][j] -= f * M[col][j];
      }
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) c.mix[4 * i + j] = M[i][4 + j];
  return true;
}

}  // namespace quadenv
