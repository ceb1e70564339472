/* Sanitizer driver (TEST INFRASTRUCTURE ONLY): every entry point of the CPU oracle
 * (oracle/quad_oracle.c, oracle/brax_oracle.c) under AddressSanitizer + UndefinedBehaviorSanitizer,
 * built by tools/san/Makefile with -fno-sanitize-recover=all, so any finding aborts the run.
 * Covers: the four wrapper kinds on hover and trajectory envs with auto-resets, saturated and
 * non-finite actions, NaN / Inf / huge states (MuJoCo's bad-state resets), mj_forward, the Euler
 * conversions at the gimbal poles, the Philox draws, and both brax kinds. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/quad_oracle.h"

static unsigned long long rng = 88172645463325252ull;
static double urand(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (double)(rng >> 11) / 9007199254740992.0; }

static void random_action(float a[4], int t) {
  for (int k = 0; k < 4; k++) a[k] = (float)(2.0 * urand() - 1.0);
  if (t % 97 == 5) a[t % 4] = 1e30f;                 /* far outside the action box */
  if (t % 131 == 7) a[(t + 1) % 4] = NAN;            /* non-finite action */
  if (t % 173 == 9) a[(t + 2) % 4] = -INFINITY;
}

static double run_env(int kind, int wrap, int steps) {
  OracleCfg cfg;
  oracle_default_cfg(kind, wrap, &cfg);
  OracleEnv env;
  memset(&env, 0, sizeof env);
  float i12[12], t3[3], obs[12], a[4], o7[7];
  uint32_t ep = 0;
  oracle_reset_draw(&cfg, 7, 3, ep++, i12, t3);
  oracle_env_reset(&cfg, &env, i12, t3, obs);
  OracleStepOut out;
  double sum = 0;
  for (int t = 0; t < steps; t++) {
    random_action(a, t);
    if (t % 211 == 17) env.qpos[t % ORACLE_NQ] = NAN;  /* bad state: MuJoCo resets, env terminates */
    if (t % 223 == 19) env.qvel[t % ORACLE_NV] = 1e12;
    oracle_env_step(&cfg, &env, a, &out);
    oracle_relpos_obs(&env, out.obs, o7);
    sum += isfinite(out.reward) ? out.reward : 0.0;
    if (out.terminated || out.truncated) {
      oracle_reset_draw(&cfg, 7, 3, ep++, i12, t3);
      oracle_env_reset(&cfg, &env, i12, t3, obs);
    }
  }
  OracleEnv envs[16];
  OracleStepOut outs[16];
  float acts[64];
  for (int i = 0; i < 16; i++) {
    oracle_reset_draw(&cfg, 11, (uint64_t)i, 0, i12, t3);
    oracle_env_reset(&cfg, &envs[i], i12, t3, obs);
  }
  for (int i = 0; i < 64; i++) acts[i] = (float)(2.0 * urand() - 1.0);
  oracle_env_step_batch(&cfg, envs, 16, acts, outs);
  return sum + oracle_bench_rollout(&cfg, 8, 64, 5);
}

static void run_brax(int kind, int steps) {
  OracleBraxCfg cfg;
  oracle_brax_default_cfg(kind, &cfg);
  OracleBraxEnv env;
  memset(&env, 0, sizeof env);
  float u21[21], obs[21], a[4];
  oracle_brax_reset_draw(&cfg, 9, 1, 0, u21);
  oracle_brax_reset(&cfg, &env, u21, obs);
  OracleBraxOut out;
  for (int t = 0; t < steps; t++) {
    random_action(a, t);
    if (t % 211 == 17) env.qvel[t % ORACLE_NV] = NAN;
    oracle_brax_step(&cfg, &env, a, t % 2, &out);
  }
}

int main(void) {
  double s = 0;
  for (int kind = ORACLE_ENV_HOVER; kind <= ORACLE_ENV_TRAJ; kind++)
    for (int wrap = ORACLE_WRAP_NONE; wrap <= ORACLE_WRAP_CTBR_RELPOS; wrap++) s += run_env(kind, wrap, 3000);
  run_brax(ORACLE_ENV_BRAX_HOVER, 1500);
  run_brax(ORACLE_ENV_BRAX_TRAJ, 1500);
  /* physics entry points on their own */
  OracleOpt opt = {0.01, {0, 0, -9.81}, 1.225, 1.8e-5};
  double qpos[ORACLE_NQ] = {0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0}, qvel[ORACLE_NV] = {0}, ctrl[4] = {3, 3, 3, 3};
  double M[100], bias[10], pas[10], act[10], qacc[10];
  oracle_mj_forward(&opt, qpos, qvel, ctrl, M, bias, pas, act, qacc);
  oracle_mj_forward(&opt, qpos, qvel, ctrl, NULL, NULL, NULL, NULL, qacc);
  for (int t = 0; t < 500; t++) {
    ctrl[t % 4] = t % 50 == 3 ? 1e9 : 13.0 * urand();
    oracle_mj_step(&opt, qpos, qvel, ctrl);
    oracle_mjx_step(&opt, qpos, qvel, ctrl);
  }
  qpos[0] = INFINITY;
  oracle_mj_step(&opt, qpos, qvel, ctrl);
  /* Euler conversions at and around the poles */
  const double poles[][3] = {{0, M_PI / 2, 0}, {0, -M_PI / 2, 0}, {M_PI, 0, -M_PI}, {0.3, 1.5707963267948966, 0.2}};
  for (int i = 0; i < 4; i++) {
    double q[4], e[3];
    oracle_euler_to_quat(poles[i], q);
    oracle_quat_to_euler(q, e);
  }
  double qz[4] = {0, 0, 0, 0}, e[3];
  oracle_quat_to_euler(qz, e);
  uint32_t ctr[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, key[2] = {0xffffffffu, 0xffffffffu}, o[4];
  oracle_philox4x32_10(ctr, key, o);
  float ra[4];
  oracle_random_action(~0ull, ~0ull, 0xffffffffu, ra);
  printf("san_oracle OK %.6e\n", s);
  return 0;
}
