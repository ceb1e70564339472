// policy.hip -- the PPO rollout policy (SB3 ActorCritic as configured by train.py:50-68:
// separate actor / critic MLPs 12 -> 128 -> 128, ReLU, action head 4, value head 1, fp32) as
// MFMA kernels for gfx950, plus the per-step rollout epilogue.
//
// Layout trick: every hidden layer is computed TRANSPOSED, H^T = W . X^T, with
// v_mfma_f32_32x32x2_f32 (A = weights, B = activations). A 32x32 accumulator tile then holds
// neurons in its registers and envs on its lanes (col = lane & 31, row = (r & 3) + 8 (r >> 2) +
// 4 (lane >> 5)), which is exactly the B-operand layout of the next layer if k-step r of that layer
// consumes the input neurons held in register r -- so the whole MLP stays in registers. The
// weights are packed once per rollout (k_policy_pack) into that permuted fragment order and staged
// in LDS (148 KB for actor + critic). Output heads (4 and 1 wide) run on the VALU with one
// lane-half exchange. f32-input MFMA is exact f32 (an ordered fma chain), the VALU-rate
// peak, and one wave per SIMD already saturates the matrix pipe.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/quadenv.h"
#include "quad_physics.h"

using namespace quadenv;

namespace quadenv {
int set_error(int code, const char* msg);  // quadenv.hip
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int H = 128, OBS = 12, ACT = 4;
constexpr int TILE = 32;          // envs per MFMA tile (one wave holds one tile at a time)
constexpr int PBLOCK = 256;       // 4 waves

// packed net image (floats), identical layout for actor and critic:
//   W1: [4 n][6 s][64 lane]            A fragments of layer 1 (K = 12 -> 6 k-steps of 2)
//   W2: [4 m][4 n][4 q][64 lane][4 r]   A fragments of layer 2, k-step r + 4q of input tile n
//   B1, B2: [4 tile][16 reg][2 half]    biases in accumulator order
//   W3: [4 out][4 tile][16 reg][2 half] head weights in accumulator order (critic: 1 out)
//   B3: [4]
constexpr int W1_F = 4 * 6 * 64, W2_F = 4 * 4 * 4 * 64 * 4, B_F = 4 * 16 * 2;
constexpr int NET_W1 = 0, NET_W2 = NET_W1 + W1_F, NET_B1 = NET_W2 + W2_F, NET_B2 = NET_B1 + B_F;
constexpr int NET_W3 = NET_B2 + B_F;
constexpr int ACTOR_F = NET_W3 + ACT * B_F + 4;
constexpr int CRITIC_F = NET_W3 + 1 * B_F + 4;
constexpr int PACKED_F = ACTOR_F + CRITIC_F + 4;  // + log_std[4]
constexpr int LDS_F = ACTOR_F + CRITIC_F;         // 37,224 floats = 148.9 KB

__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---- pack: one thread per packed float
struct NetPtrs {
  const float *w0, *b0, *w1, *b1, *w2, *b2;  // [128,12] [128] [128,128] [128] [out,128] [out]
};

__device__ float pack_one(const NetPtrs& p, int nout, int idx) {
  if (idx < NET_W2) {  // W1[n][s][lane]: A[i = lane&31][k = lane>>5] of tile n, k-step s
    const int lane = idx % 64, s = (idx / 64) % 6, n = idx / 384;
    return p.w0[(32 * n + (lane & 31)) * OBS + 2 * s + (lane >> 5)];
  }
  if (idx < NET_B1) {  // W2[m][n][q][lane][r]
    int t = idx - NET_W2;
    const int r = t % 4; t /= 4;
    const int lane = t % 64; t /= 64;
    const int q = t % 4; t /= 4;
    const int n = t % 4, m = t / 4;
    const int kreg = 4 * q + r;  // register of the input tile consumed at this k-step
    const int in = 32 * n + acc_row(kreg, lane >> 5);
    return p.w1[(32 * m + (lane & 31)) * H + in];
  }
  if (idx < NET_W3) {  // B1 / B2 [tile][reg][half]
    const bool second = idx >= NET_B2;
    const int t = idx - (second ? NET_B2 : NET_B1);
    const int h = t % 2, r = (t / 2) % 16, tile = t / 32;
    return (second ? p.b1 : p.b0)[32 * tile + acc_row(r, h)];
  }
  int t = idx - NET_W3;
  if (t < nout * B_F) {  // W3[out][tile][reg][half]
    const int h = t % 2, r = (t / 2) % 16, tile = (t / 32) % 4, o = t / 128;
    return p.w2[o * H + 32 * tile + acc_row(r, h)];
  }
  t -= nout * B_F;
  return t < nout ? p.b2[t] : 0.f;
}

__global__ void k_policy_pack(NetPtrs actor, NetPtrs critic, const float* __restrict__ log_std,
                              float* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= PACKED_F) return;
  float v;
  if (idx < ACTOR_F) v = pack_one(actor, ACT, idx);
  else if (idx < ACTOR_F + CRITIC_F) v = pack_one(critic, 1, idx - ACTOR_F);
  else v = log_std[idx - ACTOR_F - CRITIC_F];
  out[idx] = v;
}

// ---- the MLP trunk of one net for one 32-env tile: returns head outputs (per env, combined over
// the two lane halves), NOUT of them. X^T fragments: xb[s] = obs[env = lane&31][2 s + (lane>>5)].
template <int NOUT>
__device__ __forceinline__ void net_forward(const float* __restrict__ L, const float xb[6], float out[NOUT]) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  f32x16 h1[4];
#pragma unroll
  for (int n = 0; n < 4; n++) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = L[NET_B1 + (n * 16 + r) * 2 + h];
#pragma unroll
    for (int s = 0; s < 6; s++)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(L[NET_W1 + (n * 6 + s) * 64 + lane], xb[s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = fmaxf(acc[r], 0.f);  // ReLU
    h1[n] = acc;
  }
  float part[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; o++) part[o] = 0.f;
#pragma unroll 1
  for (int m = 0; m < 4; m++) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = L[NET_B2 + (m * 16 + r) * 2 + h];
#pragma unroll
    for (int n = 0; n < 4; n++) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const float4 a4 = *reinterpret_cast<const float4*>(&L[NET_W2 + (((m * 4 + n) * 4 + q) * 64 + lane) * 4]);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, h1[n][4 * q + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, h1[n][4 * q + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, h1[n][4 * q + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, h1[n][4 * q + 3], acc, 0, 0, 0);
      }
    }
    // ReLU, then this 32-neuron slice's contribution to the head (VALU)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const float a = fmaxf(acc[r], 0.f);
#pragma unroll
      for (int o = 0; o < NOUT; o++) part[o] = fmaf(L[NET_W3 + ((o * 4 + m) * 16 + r) * 2 + h], a, part[o]);
    }
  }
  // lanes l and l ^ 32 hold the two halves of the same env's neurons
#pragma unroll
  for (int o = 0; o < NOUT; o++) {
    const float other = __shfl_xor(part[o], 32);
    out[o] = (part[o] + other) + L[NET_W3 + NOUT * B_F + o];
  }
}

__device__ __forceinline__ void stage_lds(float* lds, const float* __restrict__ packed) {
  const float4* src = reinterpret_cast<const float4*>(packed);
  float4* dst = reinterpret_cast<float4*>(lds);
  for (int k = threadIdx.x; k < LDS_F / 4; k += PBLOCK) dst[k] = src[k];
  __syncthreads();
}

__device__ __forceinline__ void load_xb(const float* __restrict__ obs, int env, bool ok, float xb[6]) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int s = 0; s < 6; s++) xb[s] = ok ? obs[size_t(env) * OBS + 2 * s + h] : 0.f;
}

// Box-Muller on Philox(seed; env, step, 0x200) -> 4 standard normals
__device__ __forceinline__ void gauss4(uint64_t seed, uint64_t env, uint32_t step, float z[4]) {
  uint32_t c[4] = {uint32_t(env), uint32_t(env >> 32), step, 0x200u};
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const float u1 = (float(c[2 * k] >> 8) + 1.0f) * 0x1p-24f;  // (0, 1]
    const float u2 = float(c[2 * k + 1] >> 8) * 0x1p-24f;
    const float r = sqrtf(-2.0f * logf(u1));
    float s, co;
    sincosf(6.283185307179586f * u2, &s, &co);
    z[2 * k] = r * co;
    z[2 * k + 1] = r * s;
  }
}

struct ActArgs {
  const float* obs;        // [N,12]
  float* act_env;          // [N,4] clipped
  float* act;              // [N,4] unclipped sample (buffer row) or NULL
  float* logp;             // [N] or NULL
  float* value;            // [N] or NULL
  float* obs_copy;         // [N,12] or NULL
  const float* last_start; // [N] or NULL
  float* starts;           // [T,N] or NULL
  const uint32_t* t_index; // device step counter (row t % rows of the buffers) or NULL
  int32_t rows;
  uint64_t seed;
  uint64_t env_base;
  int32_t n;
  int32_t deterministic;
};

__global__ __launch_bounds__(PBLOCK) void k_policy_act(const float* __restrict__ packed, ActArgs a) {
  extern __shared__ float lds[];
  stage_lds(lds, packed);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int tiles = (a.n + TILE - 1) / TILE;
  const uint32_t t = a.t_index ? *a.t_index : 0u;
  const size_t row0 = size_t(t % uint32_t(a.rows)) * a.n;
  for (int tile = blockIdx.x * 4 + wave; tile < tiles; tile += gridDim.x * 4) {
    const int env = tile * TILE + (lane & 31);
    const bool ok = env < a.n;
    float xb[6];
    load_xb(a.obs, env, ok, xb);
    float mean[ACT], val[1];
    net_forward<ACT>(lds, xb, mean);
    net_forward<1>(lds + ACTOR_F, xb, val);
    if (!ok) continue;
    if (a.obs_copy) {
#pragma unroll
      for (int s = 0; s < 6; s++) a.obs_copy[(row0 + env) * OBS + 2 * s + h] = xb[s];
    }
    if (h) continue;  // one lane per env from here
    if (a.starts) a.starts[row0 + env] = a.last_start ? a.last_start[env] : 0.f;
    const float* log_std = packed + ACTOR_F + CRITIC_F;
    float z[ACT] = {0.f, 0.f, 0.f, 0.f};
    if (!a.deterministic) gauss4(a.seed, a.env_base + uint64_t(env), t, z);
    float act[ACT], lp = 0.f;
#pragma unroll
    for (int j = 0; j < ACT; j++) {
      const float sd = expf(log_std[j]);
      act[j] = mean[j] + sd * z[j];
      const float zz = (act[j] - mean[j]) / sd;  // as PPO.train recomputes it (policy.log_prob)
      lp += -0.5f * zz * zz - log_std[j] - 0.91893853320467274f;  // 0.5 log(2 pi)
    }
    reinterpret_cast<float4*>(a.act_env)[env] =
        make_float4(fminf(fmaxf(act[0], -1.f), 1.f), fminf(fmaxf(act[1], -1.f), 1.f),
                    fminf(fmaxf(act[2], -1.f), 1.f), fminf(fmaxf(act[3], -1.f), 1.f));
    if (a.act) reinterpret_cast<float4*>(a.act + row0 * ACT)[env] = make_float4(act[0], act[1], act[2], act[3]);
    if (a.logp) a.logp[row0 + env] = lp;
    if (a.value) a.value[row0 + env] = val[0];
  }
}

// Rollout epilogue for step t (after quad_step): TimeLimit bootstrap r += gamma V(terminal_obs)
// where truncated & !terminated (critic run only on tiles that need it), reward buffer row,
// episode_start for t + 1, Monitor episode statistics, t += 1.
struct PostArgs {
  const float* reward;
  const uint8_t* terminated;
  const uint8_t* truncated;
  const float* terminal_obs;
  float* buf_rew;        // [T,N]
  float* last_start;     // [N] episode_starts for the next step
  float* ep_ret;         // [N]
  float* ep_len;         // [N]
  double* stats;         // [3]: sum of finished returns, lengths, count
  const uint32_t* t_index;
  int32_t rows;
  float gamma;
  int32_t n;
};

__global__ __launch_bounds__(PBLOCK) void k_rollout_post(const float* __restrict__ packed, PostArgs a) {
  extern __shared__ float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tiles = (a.n + TILE - 1) / TILE;
  // does any tile of this block need the critic? (stage the weights only then)
  bool need = false;
  for (int tile = blockIdx.x * 4; tile < blockIdx.x * 4 + 4 && tile < tiles; tile++) {
    const int env = tile * TILE + (lane & 31);
    if (env < a.n) need |= a.truncated[env] && !a.terminated[env];
  }
  need = __syncthreads_or(need);
  if (need) stage_lds(lds, packed);
  const size_t row0 = size_t(*a.t_index % uint32_t(a.rows)) * a.n;
  const int tile = blockIdx.x * 4 + wave;
  float dret = 0.f, dlen = 0.f, dcnt = 0.f;
  if (tile < tiles) {
    const int env = tile * TILE + (lane & 31);
    const bool ok = env < a.n;
    const bool timeout = ok && a.truncated[env] && !a.terminated[env];
    float tv = 0.f;
    if (__any(timeout)) {
      float xb[6], v[1];
      load_xb(a.terminal_obs, env, ok, xb);
      net_forward<1>(lds + ACTOR_F, xb, v);
      tv = v[0];
    }
    if (ok && (lane >> 5) == 0) {
      const float r = a.reward[env];
      a.buf_rew[row0 + env] = timeout ? r + a.gamma * tv : r;
      const bool done = a.terminated[env] || a.truncated[env];
      const float ret = a.ep_ret[env] + r, len = a.ep_len[env] + 1.f;
      if (done) { dret = ret; dlen = len; dcnt = 1.f; }
      a.ep_ret[env] = done ? 0.f : ret;
      a.ep_len[env] = done ? 0.f : len;
      a.last_start[env] = done ? 1.f : 0.f;
    }
  }
  // block reduction of the episode statistics -> one atomic per block
  __shared__ float red[3][PBLOCK / 64];
  for (int off = 32; off > 0; off >>= 1) {
    dret += __shfl_down(dret, off);
    dlen += __shfl_down(dlen, off);
    dcnt += __shfl_down(dcnt, off);
  }
  if (lane == 0) { red[0][wave] = dret; red[1][wave] = dlen; red[2][wave] = dcnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int w = 0; w < PBLOCK / 64; w++) { s0 += red[0][w]; s1 += red[1][w]; s2 += red[2][w]; }
    if (s2 > 0.f) {
      atomicAdd(&a.stats[0], double(s0));
      atomicAdd(&a.stats[1], double(s1));
      atomicAdd(&a.stats[2], double(s2));
    }
  }
}

__global__ void k_t_advance(uint32_t* t) { *t += 1u; }

int pfail(int code, const char* m) { return set_error(code, m); }

// the kernels take 149 KB of dynamic LDS (gfx950 has 160 KB per CU): opt in once per device
int lds_opt_in() {
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return pfail(QUAD_EHIP, "hipGetDevice failed");
  if (done[dev]) return QUAD_OK;
  const int bytes = LDS_F * int(sizeof(float));
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_policy_act),
                          hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess ||
      hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rollout_post),
                          hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    return pfail(QUAD_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  done[dev] = true;
  return QUAD_OK;
}

int grid_for(int n) {
  const int tiles = (n + TILE - 1) / TILE;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  }
  const int want = (tiles + 3) / 4;
  return want < cus ? want : cus;  // one 149-KB-LDS block per CU, grid-stride over tiles
}

}  // namespace

extern "C" {

int32_t quad_policy_packed_floats(void) { return PACKED_F; }

int quad_policy_pack(const QuadPolicyParams* p, float* packed, void* stream) {
  if (!p || !packed) return pfail(QUAD_EINVAL, "params/packed is NULL");
  if (int rc = lds_opt_in()) return rc;
  if (reinterpret_cast<uintptr_t>(packed) & 15u) return pfail(QUAD_EINVAL, "packed must be 16-byte aligned");
  NetPtrs actor{p->pi_w0, p->pi_b0, p->pi_w1, p->pi_b1, p->act_w, p->act_b};
  NetPtrs critic{p->vf_w0, p->vf_b0, p->vf_w1, p->vf_b1, p->val_w, p->val_b};
  hipLaunchKernelGGL(k_policy_pack, dim3((PACKED_F + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), actor, critic, p->log_std, packed);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_policy_pack launch failed");
}

int quad_policy_act(const float* packed, const QuadPolicyAct* s, int32_t n, void* stream) {
  if (!packed || !s || !s->obs || !s->actions_env) return pfail(QUAD_EINVAL, "NULL argument");
  if (n <= 0) return pfail(QUAD_EINVAL, "n must be > 0");
  if ((reinterpret_cast<uintptr_t>(s->actions_env) | reinterpret_cast<uintptr_t>(s->actions)) & 15u)
    return pfail(QUAD_EINVAL, "action buffers must be 16-byte aligned");
  if (s->rows < 1) return pfail(QUAD_EINVAL, "rows must be >= 1");
  if (int rc = lds_opt_in()) return rc;
  ActArgs a{s->obs, s->actions_env, s->actions, s->log_prob, s->value, s->obs_copy,
            s->last_start, s->episode_starts, s->t_index, s->rows,
            s->seed, s->env_id_base, n, s->deterministic};
  hipLaunchKernelGGL(k_policy_act, dim3(grid_for(n)), dim3(PBLOCK), LDS_F * sizeof(float),
                     static_cast<hipStream_t>(stream), packed, a);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_policy_act launch failed");
}

int quad_rollout_post(const float* packed, const QuadRolloutPost* s, int32_t n, void* stream) {
  if (!packed || !s || !s->reward || !s->terminated || !s->truncated || !s->terminal_obs ||
      !s->buf_rew || !s->last_start || !s->ep_ret || !s->ep_len || !s->stats || !s->t_index)
    return pfail(QUAD_EINVAL, "NULL argument");
  if (n <= 0) return pfail(QUAD_EINVAL, "n must be > 0");
  if (s->rows < 1) return pfail(QUAD_EINVAL, "rows must be >= 1");
  if (int rc = lds_opt_in()) return rc;
  PostArgs a{s->reward, s->terminated, s->truncated, s->terminal_obs, s->buf_rew, s->last_start,
             s->ep_ret, s->ep_len, s->stats, s->t_index, s->rows, s->gamma, n};
  const int tiles = (n + TILE - 1) / TILE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_rollout_post, dim3((tiles + 3) / 4), dim3(PBLOCK), LDS_F * sizeof(float), st, packed, a);
  hipLaunchKernelGGL(k_t_advance, dim3(1), dim3(1), 0, st, s->t_index);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_rollout_post launch failed");
}

}  // extern "C"
