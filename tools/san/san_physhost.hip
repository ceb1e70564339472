// Sanitizer driver (TEST INFRASTRUCTURE ONLY): the product's quad_physics.h / quad_model.h
// templates instantiated on the host (tests/native/phys_host.hip, T = double and T = float) under
// AddressSanitizer + UndefinedBehaviorSanitizer on the host side of the hipcc compile
// (tools/san/Makefile: -Xarch_host -fsanitize=...). Drives the step (plain and CTBR, hover and
// trajectory constants), the physics step, the Philox reset draw and the f32 math helpers over
// random, saturated and non-finite inputs.
#include "../../tests/native/phys_host.hip"

#include <cmath>
#include <cstdio>

namespace {
unsigned long long rs = 0x9E3779B97F4A7C15ull;
double urand() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return double(rs >> 11) / 9007199254740992.0; }

template <int F64>
void drive(int kind, int wrap) {
  QuadCfg cfg;
  default_cfg_fill(kind, wrap, &cfg);
  double qpos[11] = {0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0}, qvel[10] = {0}, volt = 16.8, rint[3] = {0, 0, 0};
  float tgt[3] = {0.1f, -0.2f, 1.0f}, act[4], obs[12], s12[12], rew, motor[4], vs;
  int32_t step = 0, term = 0, trunc = 0;
  for (int t = 0; t < 2000; t++) {
    for (int k = 0; k < 4; k++) act[k] = float(2.0 * urand() - 1.0);
    if (t % 97 == 5) act[t % 4] = 1e30f;
    if (t % 131 == 7) act[(t + 1) % 4] = NAN;
    if (t % 211 == 17) qvel[t % 10] = NAN;
    const int rc = F64 ? host_env_step_f64(&cfg, qpos, qvel, &volt, tgt, &step, rint, act, obs, s12, &rew, &term,
                                           &trunc, motor, &vs)
                       : host_env_step_f32(&cfg, qpos, qvel, &volt, tgt, &step, rint, act, obs, s12, &rew, &term,
                                           &trunc, motor, &vs);
    if (rc != 0) { std::printf("step rc %d\n", rc); std::abort(); }
    if (term || trunc || !std::isfinite(qpos[0] + qvel[0])) {
      float i12[12], t3[3];
      host_reset_draw(&cfg, 5, 1, uint32_t(t), i12, t3);
      for (int i = 0; i < 11; i++) qpos[i] = 0;
      qpos[2] = 1; qpos[3] = 1;
      for (int i = 0; i < 10; i++) qvel[i] = 0;
      step = 0; volt = 16.8;
    }
  }
  double ctrl[4] = {3, 3, 3, 3};
  for (int t = 0; t < 200; t++) {
    ctrl[t % 4] = t % 50 == 3 ? 1e9 : 13.0 * urand();
    host_physics_step_f64(&cfg, qpos, qvel, ctrl);
  }
}
}  // namespace

int main() {
  for (int kind = QUAD_ENV_HOVER; kind <= QUAD_ENV_TRAJ; kind++)
    for (int wrap = QUAD_WRAP_NONE; wrap <= QUAD_WRAP_CTBR; wrap++) { drive<1>(kind, wrap); drive<0>(kind, wrap); }
  float x[9] = {0.f, -0.f, 1e-30f, 3.14159274f, -3.14159274f, 1e30f, NAN, INFINITY, -INFINITY}, s[9], c[9], r[9];
  host_fsincos(x, s, c, 9);
  host_fatan2(x, x + 1, r, 8);
  host_div_const(x, 3.0f, r, 9);
  float i12[12], t3[3];
  QuadCfg cfg;
  default_cfg_fill(QUAD_ENV_HOVER, QUAD_WRAP_NONE, &cfg);
  host_reset_draw(&cfg, ~0ull, ~0ull, 0xffffffffu, i12, t3);
  std::printf("san_physhost OK\n");
  return 0;
}
