// quadenv.hip -- gfx950 kernels + the extern "C" ABI declared in include/quadenv.h.
//
// Data layout in HBM (one allocation per handle, field-major SoA, stride N):
//   soa[f * N + i], f = 0..10 qpos, 11..20 qvel, 21 voltage, 22..24 target, 25..27 CTBR integral
//   step[N] int32, episode[N] uint32
// One thread owns one env for a whole step; every per-field access of a wave is a coalesced
// 256-B line. The [N,12] row-major observation rows (48 B per env, what the policy GEMM wants)
// are transposed through LDS so that each wave-store instruction writes 1 KiB contiguously.
//
// Kernels
//   k_step<KIND, CTBR>   fused: (CTBR) -> mixer -> voltage -> mj_step -> obs -> reward ->
//                        termination/truncation -> SB3 auto-reset -> obs (LDS transpose)
//   k_reset<KIND>        HoverEnv.reset for all / masked envs
//   k_observe            HoverEnv._get_obs of the current state
//   k_random_actions     action_space.sample() stand-in (Philox), config 2
//   k_gae                SB3 GAE(lambda) reverse scan, one thread per env
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/quadenv.h"
#include "quad_model.h"
#include "quad_physics.h"

using namespace quadenv;

namespace {

constexpr int NF = 28;
constexpr int F_QPOS = 0, F_QVEL = 11, F_VOLT = 21, F_TGT = 22, F_RINT = 25;
constexpr int BLOCK = 256;

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(QUAD_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e__ = (expr);                           \
    if (e__ != hipSuccess) return hip_fail(e__, #expr); \
  } while (0)

struct KParams {
  KConsts<float> k;
  float* soa;
  int32_t* step;
  uint32_t* ep;
  int32_t n;
  int32_t auto_reset;
  uint64_t seed;
  uint64_t gid_base;
};

__device__ __forceinline__ void load_env(const KParams& p, int i, EnvRegs<float>& e, bool ctbr) {
  const int n = p.n;
  const float* s = p.soa;
#pragma unroll
  for (int j = 0; j < 3; j++) e.pos[j] = s[(F_QPOS + j) * n + i];
#pragma unroll
  for (int j = 0; j < 4; j++) e.q[j] = s[(F_QPOS + 3 + j) * n + i];
#pragma unroll
  for (int j = 0; j < 4; j++) e.th[j] = s[(F_QPOS + 7 + j) * n + i];
#pragma unroll
  for (int j = 0; j < 3; j++) e.v[j] = s[(F_QVEL + j) * n + i];
#pragma unroll
  for (int j = 0; j < 3; j++) e.w[j] = s[(F_QVEL + 3 + j) * n + i];
#pragma unroll
  for (int j = 0; j < 4; j++) e.s[j] = s[(F_QVEL + 6 + j) * n + i];
  e.volt = s[F_VOLT * n + i];
#pragma unroll
  for (int j = 0; j < 3; j++) e.target[j] = s[(F_TGT + j) * n + i];
  if (ctbr) {
#pragma unroll
    for (int j = 0; j < 3; j++) e.rint[j] = s[(F_RINT + j) * n + i];
  } else {
    e.rint[0] = e.rint[1] = e.rint[2] = 0.f;
  }
  e.step = p.step[i];
}

__device__ __forceinline__ void store_env(const KParams& p, int i, const EnvRegs<float>& e,
                                          bool ctbr) {
  const int n = p.n;
  float* s = p.soa;
#pragma unroll
  for (int j = 0; j < 3; j++) s[(F_QPOS + j) * n + i] = e.pos[j];
#pragma unroll
  for (int j = 0; j < 4; j++) s[(F_QPOS + 3 + j) * n + i] = e.q[j];
#pragma unroll
  for (int j = 0; j < 4; j++) s[(F_QPOS + 7 + j) * n + i] = e.th[j];
#pragma unroll
  for (int j = 0; j < 3; j++) s[(F_QVEL + j) * n + i] = e.v[j];
#pragma unroll
  for (int j = 0; j < 3; j++) s[(F_QVEL + 3 + j) * n + i] = e.w[j];
#pragma unroll
  for (int j = 0; j < 4; j++) s[(F_QVEL + 6 + j) * n + i] = e.s[j];
  s[F_VOLT * n + i] = e.volt;
#pragma unroll
  for (int j = 0; j < 3; j++) s[(F_TGT + j) * n + i] = e.target[j];
  if (ctbr) {
#pragma unroll
    for (int j = 0; j < 3; j++) s[(F_RINT + j) * n + i] = e.rint[j];
  }
  p.step[i] = e.step;
}

template <int KIND>
__device__ __forceinline__ void reset_env(const KParams& p, int i, EnvRegs<float>& e,
                                          float obs[12]) {
  const uint32_t ep = p.ep[i];
  float init12[12], tgt[3], s12[12];
  reset_draw(p.k.init_lo, p.k.init_span, p.k.tgt_lo, p.k.tgt_span, p.seed, p.gid_base + uint64_t(i),
             ep, init12, tgt);
  env_reset_from<float, KIND>(p.k, e, init12, tgt, obs, s12);
  p.ep[i] = ep + 1;
}

// Stage the block's [256,12] obs rows through LDS; write them as contiguous float4.
__device__ __forceinline__ void store_obs_rows(float4* lds, const float obs[12], float* out,
                                               int block_first, int n) {
  const int t = threadIdx.x;
  lds[3 * t + 0] = make_float4(obs[0], obs[1], obs[2], obs[3]);
  lds[3 * t + 1] = make_float4(obs[4], obs[5], obs[6], obs[7]);
  lds[3 * t + 2] = make_float4(obs[8], obs[9], obs[10], obs[11]);
  __syncthreads();
  const int rows = min(BLOCK, n - block_first);
  const int nf4 = rows * 3;
  float4* dst = reinterpret_cast<float4*>(out + size_t(block_first) * 12);
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int idx = j * BLOCK + t;
    if (idx < nf4) dst[idx] = lds[idx];
  }
}

template <int KIND, bool CTBR>
__global__ __launch_bounds__(BLOCK) void k_step(KParams p, const float4* __restrict__ act,
                                                QuadStepOut out) {
  __shared__ float4 lds[BLOCK * 3];
  const int block_first = blockIdx.x * BLOCK;
  const int i = block_first + threadIdx.x;
  float obs[12];
  if (i < p.n) {
    EnvRegs<float> e;
    load_env(p, i, e, CTBR);
    const float4 a4 = act[i];
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
    StepRes r;
    env_step<float, CTBR>(p.k, e, a, r);
    out.reward[i] = r.reward;
    out.terminated[i] = r.term;
    out.truncated[i] = r.trunc;
    if (out.motor_commands)
      reinterpret_cast<float4*>(out.motor_commands)[i] =
          make_float4(r.motor[0], r.motor[1], r.motor[2], r.motor[3]);
    if (out.voltage_scale) out.voltage_scale[i] = r.vscale;
    if (out.state12) {
#pragma unroll
      for (int j = 0; j < 12; j++) out.state12[size_t(i) * 12 + j] = r.state12[j];
    }
#pragma unroll
    for (int j = 0; j < 12; j++) obs[j] = r.obs[j];
    if ((r.term || r.trunc) && p.auto_reset) {
      if (out.terminal_obs) {
#pragma unroll
        for (int j = 0; j < 12; j++) out.terminal_obs[size_t(i) * 12 + j] = r.obs[j];
      }
      reset_env<KIND>(p, i, e, obs);
    }
    store_env(p, i, e, CTBR);
  }
  store_obs_rows(lds, obs, out.obs, block_first, p.n);
}

template <int KIND>
__global__ __launch_bounds__(BLOCK) void k_reset(KParams p, const uint8_t* __restrict__ mask,
                                                 float* __restrict__ obs_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  if (mask && !mask[i]) return;
  EnvRegs<float> e;
  float obs[12];
  reset_env<KIND>(p, i, e, obs);
  store_env(p, i, e, true);
  if (obs_out) {
#pragma unroll
    for (int j = 0; j < 12; j++) obs_out[size_t(i) * 12 + j] = obs[j];
  }
}

__global__ __launch_bounds__(BLOCK) void k_observe(KParams p, float* __restrict__ obs_out,
                                                   float* __restrict__ s12_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  EnvRegs<float> e;
  load_env(p, i, e, false);
  float obs[12], s12[12];
  observe(p.k, e, obs, s12);
#pragma unroll
  for (int j = 0; j < 12; j++) obs_out[size_t(i) * 12 + j] = obs[j];
  if (s12_out) {
#pragma unroll
    for (int j = 0; j < 12; j++) s12_out[size_t(i) * 12 + j] = s12[j];
  }
}

__global__ __launch_bounds__(BLOCK) void k_random_actions(int32_t n, uint64_t seed, uint64_t gid_base,
                                                          uint32_t step, float4* __restrict__ act) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const uint64_t gid = gid_base + uint64_t(i);
  uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), step, 0x100u};
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
  act[i] = make_float4(float(c[0] >> 8) * 0x1p-23f - 1.0f, float(c[1] >> 8) * 0x1p-23f - 1.0f,
                       float(c[2] >> 8) * 0x1p-23f - 1.0f, float(c[3] >> 8) * 0x1p-23f - 1.0f);
}

// SB3 RolloutBuffer.compute_returns_and_advantage, time-major [T, N]
__global__ __launch_bounds__(BLOCK) void k_gae(const float* __restrict__ rew, const float* __restrict__ val,
                                               const float* __restrict__ starts,
                                               const float* __restrict__ last_val,
                                               const float* __restrict__ dones, int32_t T, int32_t n,
                                               float gamma, float lam, float* __restrict__ adv,
                                               float* __restrict__ ret) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  float last = 0.f;
  float next_v = last_val[i];
  float next_nt = 1.0f - dones[i];
  for (int t = T - 1; t >= 0; t--) {
    const size_t o = size_t(t) * n + i;
    const float v = val[o];
    const float delta = rew[o] + gamma * next_v * next_nt - v;
    last = delta + gamma * lam * next_nt * last;
    adv[o] = last;
    ret[o] = last + v;
    next_v = v;
    next_nt = 1.0f - starts[o];
  }
}

}  // namespace

struct QuadHandle {
  QuadCfg cfg;
  PhysConstsD pd;
  KParams kp;
  int device;
  int n;
  float* soa = nullptr;
  int32_t* step = nullptr;
  uint32_t* ep = nullptr;
};

namespace {

int grid_of(int n) { return (n + BLOCK - 1) / BLOCK; }

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

int quad_abi_version(void) { return QUADENV_ABI_VERSION; }

const char* quad_last_error(void) { return g_err.c_str(); }

int quad_default_cfg(int32_t env_kind, int32_t wrapper, QuadCfg* c) {
  if (!c) return fail(QUAD_EINVAL, "cfg is NULL");
  if (env_kind != QUAD_ENV_HOVER && env_kind != QUAD_ENV_TRAJ)
    return fail(QUAD_EINVAL, "unknown env_kind");
  if (wrapper != QUAD_WRAP_NONE && wrapper != QUAD_WRAP_CTBR) return fail(QUAD_EINVAL, "unknown wrapper");
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
  return QUAD_OK;
}

int quad_create(const QuadCfg* cfg, int32_t device, uint64_t seed, uint64_t env_id_base,
                int32_t n_envs, QuadHandle** out) {
  if (!cfg || !out) return fail(QUAD_EINVAL, "cfg/out is NULL");
  *out = nullptr;
  if (n_envs <= 0) return fail(QUAD_EINVAL, "n_envs must be > 0");
  if (int64_t(n_envs) * NF > int64_t(INT32_MAX)) return fail(QUAD_EINVAL, "n_envs too large");
  if (cfg->env_kind != QUAD_ENV_HOVER && cfg->env_kind != QUAD_ENV_TRAJ)
    return fail(QUAD_EINVAL, "unknown env_kind");
  if (cfg->wrapper != QUAD_WRAP_NONE && cfg->wrapper != QUAD_WRAP_CTBR)
    return fail(QUAD_EINVAL, "unknown wrapper");
  if (cfg->max_episode_steps <= 0) return fail(QUAD_EINVAL, "max_episode_steps must be > 0");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(QUAD_EINVAL, "device out of range");
  QuadHandle* h = new (std::nothrow) QuadHandle();
  if (!h) return fail(QUAD_ENOMEM, "host allocation failed");
  h->cfg = *cfg;
  const char* why = "";
  if (!make_phys_consts(*cfg, h->pd, &why)) {
    delete h;
    return fail(QUAD_EMODEL, why);
  }
  make_kconsts<float>(*cfg, h->pd, h->kp.k);
  h->device = device;
  h->n = n_envs;
  DeviceGuard g(device);
  hipError_t e = hipMalloc(&h->soa, sizeof(float) * size_t(NF) * n_envs);
  if (e == hipSuccess) e = hipMalloc(&h->step, sizeof(int32_t) * size_t(n_envs));
  if (e == hipSuccess) e = hipMalloc(&h->ep, sizeof(uint32_t) * size_t(n_envs));
  if (e == hipSuccess) e = hipMemset(h->soa, 0, sizeof(float) * size_t(NF) * n_envs);
  if (e == hipSuccess) e = hipMemset(h->step, 0, sizeof(int32_t) * size_t(n_envs));
  if (e == hipSuccess) e = hipMemset(h->ep, 0, sizeof(uint32_t) * size_t(n_envs));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    quad_destroy(h);
    return hip_fail(e, "quad_create allocation");
  }
  h->kp.soa = h->soa;
  h->kp.step = h->step;
  h->kp.ep = h->ep;
  h->kp.n = n_envs;
  h->kp.auto_reset = cfg->auto_reset;
  h->kp.seed = seed;
  h->kp.gid_base = env_id_base;
  *out = h;
  return QUAD_OK;
}

void quad_destroy(QuadHandle* h) {
  if (!h) return;
  DeviceGuard g(h->device);
  if (h->soa) (void)hipFree(h->soa);
  if (h->step) (void)hipFree(h->step);
  if (h->ep) (void)hipFree(h->ep);
  delete h;
}

int32_t quad_num_envs(const QuadHandle* h) { return h ? h->n : 0; }

int quad_seed(QuadHandle* h, uint64_t seed, void* stream) {
  if (!h) return fail(QUAD_EINVAL, "handle is NULL");
  DeviceGuard g(h->device);
  h->kp.seed = seed;
  HIP_TRY(hipMemsetAsync(h->ep, 0, sizeof(uint32_t) * size_t(h->n), static_cast<hipStream_t>(stream)));
  return QUAD_OK;
}

int quad_reset(QuadHandle* h, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail(QUAD_EINVAL, "handle is NULL");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (h->cfg.env_kind == QUAD_ENV_TRAJ)
    hipLaunchKernelGGL(k_reset<QUAD_ENV_TRAJ>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else
    hipLaunchKernelGGL(k_reset<QUAD_ENV_HOVER>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_step(QuadHandle* h, const float* actions, const QuadStepOut* out, void* stream) {
  if (!h || !actions || !out) return fail(QUAD_EINVAL, "handle/actions/out is NULL");
  if (!out->obs || !out->reward || !out->terminated || !out->truncated)
    return fail(QUAD_EINVAL, "obs, reward, terminated and truncated are required");
  if ((reinterpret_cast<uintptr_t>(actions) | reinterpret_cast<uintptr_t>(out->obs)) & 15u)
    return fail(QUAD_EINVAL, "actions and obs must be 16-byte aligned");
  if (out->motor_commands && (reinterpret_cast<uintptr_t>(out->motor_commands) & 15u))
    return fail(QUAD_EINVAL, "motor_commands must be 16-byte aligned");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(grid_of(h->n)), blk(BLOCK);
  const float4* a = reinterpret_cast<const float4*>(actions);
  const bool traj = h->cfg.env_kind == QUAD_ENV_TRAJ, ctbr = h->cfg.wrapper == QUAD_WRAP_CTBR;
  if (traj && ctbr)
    hipLaunchKernelGGL((k_step<QUAD_ENV_TRAJ, true>), grid, blk, 0, s, h->kp, a, *out);
  else if (traj)
    hipLaunchKernelGGL((k_step<QUAD_ENV_TRAJ, false>), grid, blk, 0, s, h->kp, a, *out);
  else if (ctbr)
    hipLaunchKernelGGL((k_step<QUAD_ENV_HOVER, true>), grid, blk, 0, s, h->kp, a, *out);
  else
    hipLaunchKernelGGL((k_step<QUAD_ENV_HOVER, false>), grid, blk, 0, s, h->kp, a, *out);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_observe(QuadHandle* h, float* obs, float* state12, void* stream) {
  if (!h || !obs) return fail(QUAD_EINVAL, "handle/obs is NULL");
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(k_observe, dim3(grid_of(h->n)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                     h->kp, obs, state12);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_random_actions(QuadHandle* h, uint32_t step_index, float* actions, void* stream) {
  if (!h || !actions) return fail(QUAD_EINVAL, "handle/actions is NULL");
  if (reinterpret_cast<uintptr_t>(actions) & 15u) return fail(QUAD_EINVAL, "actions must be 16-byte aligned");
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(k_random_actions, dim3(grid_of(h->n)), dim3(BLOCK), 0,
                     static_cast<hipStream_t>(stream), h->n, h->kp.seed, h->kp.gid_base, step_index,
                     reinterpret_cast<float4*>(actions));
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

static int copy_state(QuadHandle* h, const QuadStateSoA* u, int on_host, void* stream, bool to_handle) {
  if (!h || !u) return fail(QUAD_EINVAL, "handle/state is NULL");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t n = size_t(h->n);
  const hipMemcpyKind kind = on_host ? (to_handle ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost)
                                     : hipMemcpyDeviceToDevice;
  struct Piece { void* user; void* mine; size_t bytes; };
  const Piece pieces[7] = {
      {u->qpos, h->soa + F_QPOS * n, 11 * n * sizeof(float)},
      {u->qvel, h->soa + F_QVEL * n, 10 * n * sizeof(float)},
      {u->voltage, h->soa + F_VOLT * n, n * sizeof(float)},
      {u->target, h->soa + F_TGT * n, 3 * n * sizeof(float)},
      {u->rate_int, h->soa + F_RINT * n, 3 * n * sizeof(float)},
      {u->step_count, h->step, n * sizeof(int32_t)},
      {u->episode, h->ep, n * sizeof(uint32_t)},
  };
  for (const Piece& p : pieces) {
    if (!p.user) continue;
    if (to_handle)
      HIP_TRY(hipMemcpyAsync(p.mine, p.user, p.bytes, kind, s));
    else
      HIP_TRY(hipMemcpyAsync(p.user, p.mine, p.bytes, kind, s));
  }
  if (on_host) HIP_TRY(hipStreamSynchronize(s));
  return QUAD_OK;
}

int quad_get_state(QuadHandle* h, const QuadStateSoA* dst, int32_t on_host, void* stream) {
  return copy_state(h, dst, on_host, stream, false);
}

int quad_set_state(QuadHandle* h, const QuadStateSoA* src, int32_t on_host, void* stream) {
  return copy_state(h, src, on_host, stream, true);
}

int quad_gae(const float* rewards, const float* values, const float* episode_starts,
             const float* last_values, const float* dones, int32_t T, int32_t N, float gamma,
             float gae_lambda, float* advantages, float* returns, void* stream) {
  if (!rewards || !values || !episode_starts || !last_values || !dones || !advantages || !returns)
    return fail(QUAD_EINVAL, "NULL argument");
  if (T <= 0 || N <= 0) return fail(QUAD_EINVAL, "T and N must be > 0");
  hipLaunchKernelGGL(k_gae, dim3(grid_of(N)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream), rewards,
                     values, episode_starts, last_values, dones, T, N, gamma, gae_lambda, advantages,
                     returns);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

}  // extern "C"
