/* brax_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU float64 restatement; never linked by the
 * product). The brax-compat env kinds of train_brax_ppo.py, restated from the reference:
 *   QuadHoverBraxEnv   (train_brax_ppo.py:39-176):  action denorm + clip (:133-134), mixer
 *     A_inv with motor clip [0, 13] (:96-98), mjx pipeline step (:140), obs = [q, qd] (:175-176),
 *     reward exp(-2 |pos - (0,0,1)|^2) (:142-148), done |x|,|y| > 3 or z outside [0.02, 4]
 *     (:151-159); reset q = qpos0 + U(+-0.01) (11, quaternion not renormalized), qd = U(+-0.01)
 *     (:102-129).
 *   JaxMJXQuadBraxEnv  (train_brax_ppo.py:179-368): the same control; reset at z = 1 with the
 *     quaternion renormalized by (|q| + 1e-8) (:263-281); target = sinusoid sample
 *     min(step_count, L-1) (:317-319, :358-363); validity = finite & in bounds & |v| <= 20
 *     (:322-327); reward exp(-e^2) - 0.001 |a|^2 or -1 when invalid (:329-335); obs NaN -> 0 (:337).
 * Wrapped as brax ppo.train wraps envs: EpisodeWrapper truncation at episode_length and
 * AutoResetWrapper, which restores the FIRST state of the env (not a fresh draw) and leaves the
 * env's own info (step_count) alone. JAX/brax are absent here: parity vs JAX is unpinned; the
 * reset noise is Philox (not JAX threefry) -- same distribution, different stream.
 */
#include <math.h>
#include <string.h>

#include "quad_oracle.h"

void oracle_brax_default_cfg(int32_t kind, OracleBraxCfg* c) {
  memset(c, 0, sizeof *c);
  c->kind = kind;
  c->episode_length = 500;
  c->target[2] = 1.0f;
  c->pos_limit_xy = 3.0f;
  c->pos_limit_z_low = 0.02f;
  c->pos_limit_z_high = 4.0f;
  c->vel_limit = kind == ORACLE_ENV_BRAX_TRAJ ? 20.0f : 0.0f;
  c->reset_noise = 0.01f;
  c->reward_pos_coef = kind == ORACLE_ENV_BRAX_TRAJ ? 1.0f : 2.0f;
  c->reward_action_coef = kind == ORACLE_ENV_BRAX_TRAJ ? 0.001f : 0.0f;
  c->max_motor_thrust = 13.0;
  c->arm_length = 0.039799;
  c->yaw_coeff = 0.0201;
  const float lo[4] = {0.f, -0.5f, -0.5f, -0.5f}, hi[4] = {52.f, 0.5f, 0.5f, 0.5f};
  for (int i = 0; i < 4; i++) { c->ctrl_min[i] = lo[i]; c->ctrl_max[i] = hi[i]; }
  const float cen[3] = {0.f, 0.f, 1.f}, amp[3] = {0.5f, 0.5f, 0.2f}, fr[3] = {0.2f, 0.15f, 0.1f};
  for (int i = 0; i < 3; i++) { c->traj_center[i] = cen[i]; c->traj_amp[i] = amp[i]; c->traj_freq[i] = fr[i]; }
  c->traj_duration = 5.0f;
  c->opt.timestep = 0.01;
  c->opt.gravity[2] = -9.81;
  c->opt.density = 1.225;
  c->opt.viscosity = 1.8e-5;
}

void oracle_brax_reset_draw(const OracleBraxCfg* c, uint64_t seed, uint64_t gid, uint32_t episode,
                            float u21[21]) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t r[24];
  for (uint32_t b = 0; b < 6; b++) {
    const uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), episode, 0x300u + b};
    oracle_philox4x32_10(ctr, key, r + 4 * b);
  }
  const float lo = -c->reset_noise, span = 2.0f * c->reset_noise;
  for (int i = 0; i < 21; i++) {
    const float u = (float)(r[i] >> 8) * 0x1p-24f;
    const float m = u * span;
    u21[i] = lo + m;
  }
}

static void brax_obs(const OracleBraxEnv* e, float obs[21]) {
  for (int i = 0; i < ORACLE_NQ; i++) obs[i] = (float)e->qpos[i];
  for (int i = 0; i < ORACLE_NV; i++) obs[ORACLE_NQ + i] = (float)e->qvel[i];
}

void oracle_brax_reset(const OracleBraxCfg* c, OracleBraxEnv* e, const float u21[21], float obs[21]) {
  double q0[ORACLE_NQ] = {0, 0, c->kind == ORACLE_ENV_BRAX_TRAJ ? 1.0 : 0.0, 1, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < ORACLE_NQ; i++) e->qpos[i] = (double)(float)(q0[i] + (double)u21[i]);
  for (int i = 0; i < ORACLE_NV; i++) e->qvel[i] = (double)u21[ORACLE_NQ + i];
  if (c->kind == ORACLE_ENV_BRAX_TRAJ) {
    const double n = sqrt(e->qpos[3] * e->qpos[3] + e->qpos[4] * e->qpos[4] + e->qpos[5] * e->qpos[5] +
                          e->qpos[6] * e->qpos[6]);
    for (int i = 3; i < 7; i++) e->qpos[i] /= (n + 1e-8);
  }
  memcpy(e->first_qpos, e->qpos, sizeof e->qpos);
  memcpy(e->first_qvel, e->qvel, sizeof e->qvel);
  e->steps = 0;
  e->env_steps = 0;
  brax_obs(e, obs);
}

static int finite_all(const OracleBraxEnv* e) {
  for (int i = 0; i < ORACLE_NQ; i++) if (!isfinite(e->qpos[i])) return 0;
  for (int i = 0; i < ORACLE_NV; i++) if (!isfinite(e->qvel[i])) return 0;
  return 1;
}

void oracle_brax_step(const OracleBraxCfg* c, OracleBraxEnv* e, const float action[4],
                      int32_t auto_reset, OracleBraxOut* out) {
  /* physical action (:133-134): float32 elementwise as JAX computes it (built without FMA
   * contraction); NaN passes through jnp.clip */
  double u[4];
  for (int i = 0; i < 4; i++) {
    const float span = c->ctrl_max[i] - c->ctrl_min[i];
    const float s1 = action[i] + 1.0f;
    const float s2 = s1 * 0.5f;
    const float s3 = s2 * span;
    float p = s3 + c->ctrl_min[i];
    if (p < c->ctrl_min[i]) p = c->ctrl_min[i];
    else if (p > c->ctrl_max[i]) p = c->ctrl_max[i];
    u[i] = (double)p;
  }
  /* A_inv @ u, clip [0, max_motor_thrust] (:96-98): A = [[1,1,1,1],[-l,-l,l,l],[-l,l,l,-l],[k,-k,k,-k]]
   * (float64 here and in the kernel; JAX's float32 matmul differs by float32 rounding) */
  const double l = c->arm_length, k = c->yaw_coeff;
  const double a = 1.0 / (4.0 * l), b = 1.0 / (4.0 * k);
  const double Ai[4][4] = {{0.25, -a, -a, b}, {0.25, -a, a, -b}, {0.25, a, a, b}, {0.25, a, -a, -b}};
  double F[4];
  for (int i = 0; i < 4; i++) {
    double s = 0;
    for (int j = 0; j < 4; j++) s += Ai[i][j] * u[j];
    F[i] = s < 0.0 ? 0.0 : (s > c->max_motor_thrust ? c->max_motor_thrust : s);
    out->motor_commands[i] = F[i];
  }
  oracle_mjx_step(&c->opt, e->qpos, e->qvel, F);
  e->steps += 1;
  const double* pos = e->qpos;
  double tgt[3] = {c->target[0], c->target[1], c->target[2]};
  int done;
  double reward;
  if (c->kind == ORACLE_ENV_BRAX_TRAJ) {
    e->env_steps += 1;
    const int L = c->episode_length;
    const int idx = e->env_steps < L - 1 ? e->env_steps : L - 1;
    const double t = idx == L - 1 ? (double)c->traj_duration : idx * ((double)c->traj_duration / (L - 1));
    for (int i = 0; i < 3; i++)
      tgt[i] = c->traj_center[i] + c->traj_amp[i] * sin(2.0 * M_PI * c->traj_freq[i] * t);
    const int fin = finite_all(e);
    const int oxy = fabs(pos[0]) > c->pos_limit_xy || fabs(pos[1]) > c->pos_limit_xy;
    const int oz = pos[2] < c->pos_limit_z_low || pos[2] > c->pos_limit_z_high;
    int ov = 0;
    for (int i = 0; i < 3; i++) ov |= fabs(e->qvel[i]) > c->vel_limit;
    const int valid = fin && !oxy && !oz && !ov;
    double d2 = 0;
    for (int i = 0; i < 3; i++) d2 += (pos[i] - tgt[i]) * (pos[i] - tgt[i]);
    const double per = sqrt(d2);
    const double pe = valid && isfinite(per) ? per : 1e3;
    double asq = 0;
    for (int i = 0; i < 4; i++) asq += (double)action[i] * action[i];
    const double rr = exp(-c->reward_pos_coef * pe * pe) - c->reward_action_coef * asq;
    reward = valid && isfinite(rr) ? rr : -1.0;
    done = !valid;
  } else {
    double d2 = 0;
    for (int i = 0; i < 3; i++) d2 += (pos[i] - tgt[i]) * (pos[i] - tgt[i]);
    const double pe = sqrt(d2);
    reward = exp(-c->reward_pos_coef * pe * pe);
    done = fabs(pos[0]) > c->pos_limit_xy || fabs(pos[1]) > c->pos_limit_xy ||
           pos[2] < c->pos_limit_z_low || pos[2] > c->pos_limit_z_high;  /* NaN: not done */
  }
  for (int i = 0; i < 3; i++) out->target[i] = (float)tgt[i];
  brax_obs(e, out->obs);
  if (c->kind == ORACLE_ENV_BRAX_TRAJ)
    for (int i = 0; i < 21; i++) if (!isfinite(out->obs[i])) out->obs[i] = 0.f;
  memcpy(out->terminal_obs, out->obs, sizeof out->obs);
  out->reward = reward;
  out->terminated = done;
  out->truncated = e->steps >= c->episode_length;
  if (auto_reset && (out->terminated || out->truncated)) {
    memcpy(e->qpos, e->first_qpos, sizeof e->qpos);
    memcpy(e->qvel, e->first_qvel, sizeof e->qvel);
    e->steps = 0;  /* env_steps continues (AutoResetWrapper restores pipeline_state/obs only) */
    brax_obs(e, out->obs);
  }
}

size_t oracle_sizeof_brax_cfg(void) { return sizeof(OracleBraxCfg); }
size_t oracle_sizeof_brax_env(void) { return sizeof(OracleBraxEnv); }
size_t oracle_sizeof_brax_out(void) { return sizeof(OracleBraxOut); }
