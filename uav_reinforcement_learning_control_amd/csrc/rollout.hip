// rollout.hip -- the fused PPO rollout: policy (MFMA) + env step + SB3 bookkeeping for many steps
// in ONE launch (quad_rollout, include/quadenv.h).
//
// Reference loop (SB3 OnPolicyAlgorithm.collect_rollouts as train.py:50-68 configures it, with
// HoverEnv.step / TrajectoryFollowEnv.step (+ RateControlWrapper) as the env and DummyVecEnv's
// auto-reset): obs -> policy -> a ~ N(mean, std) -> clip -> env.step -> (TimeLimit bootstrap,
// Monitor statistics, rollout-buffer rows) -> next obs.
//
// Why one launch: every piece of that loop is per env -- no env ever reads another env's data --
// so a 256-env block can run ALL the steps of its envs without a grid-wide barrier. The block
// stages the packed actor + critic (152 KB) into LDS once, keeps each env's state (one env per
// thread, as the step kernels) and its observation in registers across steps, and per step only
// WRITES its buffer rows to HBM (80 B per env-step). The two-launch form (k_policy_act with the
// fused epilogue + k_step_h) re-stages the weights, reloads and restores the env state and round-
// trips the observation and action through HBM on every step, and pays two launches per step.
//
// Wave w of a block owns envs 64w .. 64w + 63, which are exactly the two 32-env MFMA tiles the
// policy evaluates together (net_forward<., 2>): tile j = envs 64w + 32j + (lane & 31). The X^T
// fragment lane l needs (component 2s + (l >> 5) of env l & 31 of the tile) is one lane-half
// exchange away from the thread that owns the env, and the head outputs land on both lane halves,
// so lane l takes tile (l >> 5)'s output -- its own env's. The arithmetic is the same as the
// two-launch path's, operation for operation, so the buffers are bit-identical to it
// (tests/test_gpu_rollout.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "../../include/quadenv.h"
#include "env_tiles.h"
#include "kconsts_default.h"
#include "policy_net.h"
#include "quad_physics.h"
#include "rollout.h"

namespace quadenv {

namespace {

constexpr int RBLOCK = 256;  // envs per block; one block per CU (the LDS holds the nets)
constexpr int ROLLOUT_NT_DEFAULT = 2;

// X^T fragments of the wave's tile(s) from the per-thread observation rows (see top): lane half h
// takes features 8h .. 8h + 7 (zero past feature 11) of its env in each tile.
template <int NT>
__device__ __forceinline__ void fragments(const float ob[12], float (&xb)[NT][8]) {
  const bool h = (threadIdx.x & 32) != 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float lo = ob[k], hi = k < 4 ? ob[8 + k] : 0.f;  // this env's features k and 8 + k
    if constexpr (NT == 2) {  // lane l's env is tile (l >> 5)'s env l & 31
      // the other lane half's value (v_permlane32_swap: first result = lanes 0-31's, second = 32-63's)
      const float x = h ? lo : hi;
      const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
      const float got = __uint_as_float(h ? p[0] : p[1]);
      xb[0][k] = h ? got : lo;
      xb[NT - 1][k] = h ? hi : got;
    } else {  // both lane halves carry env l & 31
      xb[0][k] = h ? hi : lo;
    }
  }
}

// The reset draws of the wave's resetting envs, compacted across the wave (the round-1..5 one-wave
// step kernel did the same through LDS): one Philox pass of (env, block) items for up to 16 resetting
// envs. The words travel by lane shuffles instead of LDS (the nets fill it). Identical words.
// `publish`: this lane lists its env (one lane per env); `apply`: this lane takes the words of the
// env listed under key `key` (KEY_MASK = 31 when lanes l and l + 32 carry the same env).
template <int KEY_MASK>
__device__ __forceinline__ void reset_words_shfl(const KParams& p, uint32_t (&renv)[64], uint32_t (&rep)[64],
                                                 uint32_t i, uint32_t ep, bool publish, bool apply,
                                                 float u16[16]) {
  const uint64_t m = __ballot(publish);
  if (m == 0) return;
  const int lane = __lane_id();
  const int nres = __popcll(m);
  const int rank = __popcll(m & ((1ull << (lane & KEY_MASK)) - 1ull));
  if (publish) { renv[rank] = i; rep[rank] = ep; }
  __builtin_amdgcn_wave_barrier();
  const int passes = (nres * 4 + 63) >> 6;
  for (int t = 0; t < passes; t++) {
    const int item = t * 64 + lane, rr = item >> 2;
    uint32_t c[4] = {0u, 0u, 0u, 0u};
    if (rr < nres) reset_block(p.seed, p.gid_base + uint64_t(renv[rr]), rep[rr], uint32_t(item & 3), c);
    float cu[4];  // the uniforms u01(word), converted here: 4 per lane instead of 16 per resetting lane
#pragma unroll
    for (int k = 0; k < 4; k++) cu[k] = u01(c[k]);
    const bool mine = apply && (rank >> 4) == t;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int src = (rank * 4 + b) & 63;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const float v = __shfl(cu[k], src);
        if (mine) u16[4 * b + k] = v;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void store_row(float* __restrict__ base, size_t row, const float v[12]) {
  float4* b4 = reinterpret_cast<float4*>(base + row * 12);
  b4[0] = make_float4(v[0], v[1], v[2], v[3]);
  b4[1] = make_float4(v[4], v[5], v[6], v[7]);
  b4[2] = make_float4(v[8], v[9], v[10], v[11]);
}

// The actor's W2 pieces come from LDS (policy_net.h stage_pieces / LP_SPLIT), the critic's from L2
// (round 4; both from L2 was round 3's form, same bits).

// the Gaussian action of this lane's env (SB3 policy.forward: a = mean + std z), its log-prob as
// PPO.train recomputes it, and the clipped action the env receives
template <int NT>
__device__ __forceinline__ void sample_action(const RollArgs& a, const KParams& p, int i, uint32_t t, bool h,
                                              const float (&mean)[NT][ACT], const float (&sd)[ACT],
                                              const float (&lstd)[ACT], float (&act)[ACT], float (&ac)[ACT],
                                              float& lp) {
  float z[ACT] = {0.f, 0.f, 0.f, 0.f};
  if (!a.deterministic) gauss4(a.seed, p.gid_base + uint64_t(i), t, z);
  lp = 0.f;
#pragma unroll
  for (int k = 0; k < ACT; k++) {
    const float mk = (NT == 2 && h) ? mean[NT - 1][k] : mean[0][k];
    act[k] = mk + sd[k] * z[k];
    const float zz = (act[k] - mk) / sd[k];  // as PPO.train recomputes it (policy.log_prob)
    lp += -0.5f * zz * zz - lstd[k] - 0.91893853320467274f;  // 0.5 log(2 pi)
    ac[k] = fminf(fmaxf(act[k], -1.f), 1.f);
  }
}

// NT = 2: 4 waves (one per SIMD), wave w owns envs 64w .. 64w + 63 = its two MFMA tiles.
// NT = 1: 8 waves (two per SIMD), wave w owns the 32 envs 32w .. 32w + 31 = one tile; lanes l and
// l + 32 both carry env l & 31 (the same state, the same action, bit for bit), so the tile's X^T
// fragment needs no exchange, and one wave's env step (VALU) can run under the other wave's MFMA.
template <int KIND, bool CTBR, int NT>
__device__ __forceinline__ void rollout_body(const KConsts<float>& K, KParams p, const float* __restrict__ packed,
                                             RollArgs a) {
  constexpr int BLK = 512 / NT, WAVES = BLK / 64;
  extern __shared__ float lds[];
  __shared__ uint32_t renv[WAVES][64], rep[WAVES][64];
  const int w = threadIdx.x >> 6;
  const bool h = (threadIdx.x & 32) != 0;
  const int i_raw = blockIdx.x * RBLOCK + (NT == 2 ? int(threadIdx.x) : w * 32 + int(threadIdx.x & 31));
  const bool ok = i_raw < p.n;
  const bool owner = ok && (NT == 2 || !h);  // the lane that stores this env's outputs
  // lanes past the last env shadow it (in-range loads, MFMA columns of their own) and store nothing
  const int i = ok ? i_raw : p.n - 1;
  const size_t n = size_t(p.n);

  // ---- per-env state into registers (issued before the weight staging so both are in flight)
  EnvRegs<float> e;
  load_env(p, i, e, CTBR);
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  uint32_t ep = S.ldu(F_EP, vo);
  float ob[12];
  {
    const float4* r4 = reinterpret_cast<const float4*>(a.last_obs + size_t(i) * 12);
    const float4 x0 = r4[0], x1 = r4[1], x2 = r4[2];
    ob[0] = x0.x; ob[1] = x0.y; ob[2] = x0.z; ob[3] = x0.w;
    ob[4] = x1.x; ob[5] = x1.y; ob[6] = x1.z; ob[7] = x1.w;
    ob[8] = x2.x; ob[9] = x2.y; ob[10] = x2.z; ob[11] = x2.w;
  }
  float ls = a.last_start[i], ret = a.ep_ret[i], len = a.ep_len[i];
  stage_lds<BLK>(lds, packed);
  stage_pieces<BLK>(lds, packed);  // the actor's W2 pieces, once per launch
  const float* log_std = packed + LDS_F;
  float lstd[ACT], sd[ACT];
#pragma unroll
  for (int k = 0; k < ACT; k++) { lstd[k] = log_std[k]; sd[k] = expf(lstd[k]); }
  double st[3] = {0.0, 0.0, 0.0};

  for (int s = 0; s < a.steps; s++) {
    const uint32_t t = a.t0 + uint32_t(s);
    const size_t row = size_t(t % a.rows) * n + size_t(i);
    // ---- policy: both nets on the wave's two tiles, then this lane's env
    float xb[NT][8], mean[NT][ACT], val[NT][1];
    fragments<NT>(ob, xb);
    // QD_ROLL_*: cost-ablation builds of tools/rollout_variants.py only (never defined in the product)
#if defined(QD_ROLL_NOMLP)
#pragma unroll
    for (int j = 0; j < NT; j++) {
      val[j][0] = xb[j][0];
#pragma unroll
      for (int k = 0; k < ACT; k++) mean[j][k] = xb[j][k];
    }
#else
#if defined(QD_ROLL_NOCRITIC)
    net_forward<ACT, NT>(lds, packed, xb, mean);
#pragma unroll
    for (int j = 0; j < NT; j++) val[j][0] = mean[j][0];
#else
    net_forward2<NT, true>(lds, packed, xb, mean, val);
#endif
#endif
    float act[ACT], ac[ACT], lp = 0.f;
    sample_action<NT>(a, p, i, t, h, mean, sd, lstd, act, ac, lp);
    if (owner) {
#if !defined(QD_ROLL_NOOBSCOPY)  // cost ablation (tools/rollout_variants.sh only): the strided obs rows
      store_row(a.obs_copy, row, ob);
#endif
      reinterpret_cast<float4*>(a.actions)[row] = make_float4(act[0], act[1], act[2], act[3]);
      a.log_prob[row] = lp;
      a.value[row] = (NT == 2 && h) ? val[NT - 1][0] : val[0][0];
      a.starts[row] = ls;
    }
    // ---- env step (HoverEnv.step / TrajectoryFollowEnv.step, RateControlWrapper.action)
    StepRes r;
#if defined(QD_ROLL_NOENV)
#pragma unroll
    for (int j = 0; j < 12; j++) r.obs[j] = fminf(fmaxf(ob[j] + 1e-3f * ac[j & 3], -1.f), 1.f);
    r.reward = ac[0]; r.term = false; r.trunc = false;
#else
    env_step<float, CTBR>(K, e, ac, r);
#endif
    const bool done = r.term || r.trunc;
    // ---- TimeLimit bootstrap: r += gamma V(terminal_obs) (critic only if the wave holds one)
    const bool timeout = ok && r.trunc && !r.term;
    float tv = 0.f;
    if (__any(timeout)) {
      float xt[NT][8], vt[NT][1];
      fragments<NT>(r.obs, xt);
      net_forward<1, NT>(lds + ACTOR_F, packed, xt, vt);
      tv = (NT == 2 && h) ? vt[NT - 1][0] : vt[0][0];
    }
    // ---- reward row, Monitor statistics, episode_starts of the next step
    const float rret = ret + r.reward, rlen = len + 1.f;
    if (owner) {
      a.rewards[row] = timeout ? r.reward + a.gamma * tv : r.reward;
      if (done) { st[0] += double(rret); st[1] += double(rlen); st[2] += 1.0; }  // owner lanes only
    }
    ret = done ? 0.f : rret;
    len = done ? 0.f : rlen;
    ls = done ? 1.f : 0.f;
#pragma unroll
    for (int j = 0; j < 12; j++) ob[j] = r.obs[j];
    // ---- SB3 auto-reset: the next step starts from the reset observation
    const bool rs = ok && done;
    float u16[16];
    reset_words_shfl<NT == 2 ? 63 : 31>(p, renv[w], rep[w], uint32_t(i), ep, owner && done, rs, u16);
    if (rs) {
      float init12[12], tgt[3], s12[12];
      reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
      env_reset_from<float, KIND>(K, e, init12, tgt, ob, s12);
      ep += 1u;
    }
  }

  // ---- carry the rollout to the next call
  if (owner) {
    store_env(p, i, e, CTBR);
    S.stu(F_EP, vo, ep);
    store_row(a.last_obs, size_t(i), ob);
    a.last_start[i] = ls;
    a.ep_ret[i] = ret;
    a.ep_len[i] = len;
  }
  // Monitor statistics: block sum into this block's slot (uncontended double atomics)
  __shared__ double red[3][WAVES];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    double v = st[j];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if ((threadIdx.x & 63) == 0) red[j][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int k = 0; k < WAVES; k++) s += red[threadIdx.x][k];
    if (s != 0.0) atomicAdd(&a.stats[(blockIdx.x % QUAD_POLICY_STAT_SLOTS) * 3 + threadIdx.x], s);
  }
}

// SPEC: the handle's constant block is the reference default (kconsts_default.h): immediates
template <int KIND, bool CTBR, int NT, bool SPEC>
__global__ __launch_bounds__(512 / NT) void k_rollout(const KConsts<float>* __restrict__ kc, KParams p,
                                                            const float* __restrict__ packed, RollArgs a) {
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    rollout_body<KIND, CTBR, NT>(K, p, packed, a);
  } else {
    rollout_body<KIND, CTBR, NT>(*kc, p, packed, a);
  }
}

template <int KIND, bool CTBR, int NT, bool SPEC>
hipError_t launch(const KConsts<float>* kc, const KParams& kp, const float* packed, const RollArgs& a,
                  hipStream_t s) {
  static bool opted[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  const int bytes = LDS_F * int(sizeof(float));
  if (!opted[dev]) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rollout<KIND, CTBR, NT, SPEC>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    opted[dev] = true;
  }
  hipLaunchKernelGGL((k_rollout<KIND, CTBR, NT, SPEC>), dim3((kp.n + RBLOCK - 1) / RBLOCK), dim3(512 / NT), bytes,
                     s, kc, kp, packed, a);
  return hipGetLastError();
}

}  // namespace

template <int NT, bool SPEC>
hipError_t launch_nt(const KConsts<float>* kc, const KParams& kp, int env_kind, bool ctbr, const float* packed,
                     const RollArgs& a, hipStream_t s) {
  if (env_kind == QUAD_ENV_TRAJ)
    return ctbr ? launch<QUAD_ENV_TRAJ, true, NT, SPEC>(kc, kp, packed, a, s)
                : launch<QUAD_ENV_TRAJ, false, NT, SPEC>(kc, kp, packed, a, s);
  return ctbr ? launch<QUAD_ENV_HOVER, true, NT, SPEC>(kc, kp, packed, a, s)
              : launch<QUAD_ENV_HOVER, false, NT, SPEC>(kc, kp, packed, a, s);
}

hipError_t launch_rollout(const KConsts<float>* kc, const KParams& kp, int env_kind, bool ctbr, bool spec,
                          const float* packed, const RollArgs& a, hipStream_t s) {
  const char* v = std::getenv("QUADENV_ROLLOUT_NT");  // A/B override: 1 or 2 tiles per wave
  const int nt = v && std::atoi(v) == 1 ? 1 : (v && std::atoi(v) == 2 ? 2 : ROLLOUT_NT_DEFAULT);
  if (nt == 1) return spec ? launch_nt<1, true>(kc, kp, env_kind, ctbr, packed, a, s)
                           : launch_nt<1, false>(kc, kp, env_kind, ctbr, packed, a, s);
  return spec ? launch_nt<2, true>(kc, kp, env_kind, ctbr, packed, a, s)
              : launch_nt<2, false>(kc, kp, env_kind, ctbr, packed, a, s);
}

}  // namespace quadenv
