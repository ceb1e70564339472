// policy.hip -- the PPO rollout policy (SB3 ActorCritic as configured by train.py:50-68:
// separate actor / critic MLPs 12 -> 128 -> 128, ReLU, action head 4, value head 1, fp32) as
// MFMA kernels for gfx950, with the per-step rollout epilogue fused in.
//
// Layout trick: every hidden layer is computed TRANSPOSED, H^T = W . X^T, with
// bf16 MFMA over three-piece splits (A = weights, B = activations; policy_net.h). A 32x32 accumulator tile then holds
// neurons in its registers and envs on its lanes (col = lane & 31, row = (r & 3) + 8 (r >> 2) +
// 4 (lane >> 5)), which is exactly the B-operand layout of the next layer if k-step r of that layer
// consumes the input neurons held in register r -- so the whole MLP stays in registers. The
// weights are packed once per rollout (k_policy_pack) into that permuted fragment order and staged
// in LDS (152 KB for actor + critic; one 4-wave block per CU, grid-stride over 32-env tiles).
// Output heads (4 and 1 wide) run on the VALU with one lane-half exchange. f32-input MFMA is exact
// f32 (an ordered fma chain) at the VALU-rate peak; one wave per SIMD saturates the matrix pipe.
//
// Rollout step t = one k_policy_act launch + one quad_step launch. k_policy_act first finishes
// step t-1 (reward row with the TimeLimit bootstrap, episode_starts, Monitor statistics) when the
// cursor says it is pending, then evaluates the policy for step t; its last block to finish
// advances the cursor. quad_rollout_post finishes the final step of a rollout.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/quadenv.h"
#include "quad_physics.h"
#include "policy_net.h"

using namespace quadenv;

namespace quadenv {
int set_error(int code, const char* msg);  // quadenv.hip
}


namespace {

enum { CUR_T = 0, CUR_PENDING = 1, CUR_ARRIVED = 2 };


// ---- pack: one thread per packed float
struct NetPtrs {
  const float *w0, *b0, *w1, *b1, *w2, *b2;  // [128,12] [128] [128,128] [128] [out,128] [out]
};

__device__ float pack_one(const NetPtrs& p, int nout, int idx) {
  if (idx < NET_W2) {  // A[neuron 32n + lane&31][feature 8 (lane>>5) + j] of block n
    const int j = idx % 8, lane = (idx / 8) % 64, n = idx / 512;
    const int f = 8 * (lane >> 5) + j;
    return f < OBS ? p.w0[(32 * n + (lane & 31)) * OBS + f] : 0.f;
  }
  if (idx < NET_B1) {
    int t = idx - NET_W2;
    const int j = t % 8; t /= 8;
    const int lane = t % 64; t /= 64;
    const int half = t % 2; t /= 2;
    const int n = t % 4, m = t / 4;
    const int in = 32 * n + acc_row(8 * half + j, lane >> 5);  // input neuron held in register 8 half + j
    return p.w1[(32 * m + (lane & 31)) * H + in];
  }
  if (idx < NET_W3) {
    const bool second = idx >= NET_B2;
    const int t = idx - (second ? NET_B2 : NET_B1);
    const int r = t % 16, h = (t / 16) % 2, tile = t / 32;
    return (second ? p.b1 : p.b0)[32 * tile + acc_row(r, h)];
  }
  int t = idx - NET_W3;
  if (t < nout * 128) {
    if (nout == ACT) {
      const int o = t % 4, h = (t / 4) % 2, r = (t / 8) % 16, m = t / 128;
      return p.w2[o * H + 32 * m + acc_row(r, h)];
    }
    const int r4 = t % 4, h = (t / 4) % 2, rq = (t / 8) % 4, m = t / 32;
    return p.w2[32 * m + acc_row(4 * rq + r4, h)];
  }
  t -= nout * 128;
  return t < nout ? p.b2[t] : 0.f;
}

__global__ void k_policy_pack(NetPtrs actor, NetPtrs critic, const float* __restrict__ log_std,
                              float* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= PACKED_F + 2 * 32 * 64 + 2 * 4 * 64) return;
  if (idx >= PACKED_F + 2 * 32 * 64) {  // one (net, layer-1 block n, lane) unit of the W1 pieces
    const int u = idx - PACKED_F - 2 * 32 * 64, net = u / 256, n = (u / 64) % 4, lane = u % 64;
    const int f = NET_W1 + n * 512 + lane * 8;
    float v8[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v8[j] = net ? pack_one(critic, 1, f + j) : pack_one(actor, ACT, f + j);
    const P3 x = split8(v8);
    bf16x8* pieces = reinterpret_cast<bf16x8*>(out + PACKED_F + PIECES_F);
#pragma unroll
    for (int p = 0; p < 3; p++) pieces[((net * 4 + n) * 3 + p) * 64 + lane] = x.p[p];
    return;
  }
  if (idx >= PACKED_F) {  // one (net, k-step g, lane) unit of the pre-split W2 pieces (policy_net.h)
    const int u = idx - PACKED_F, net = u / 2048, g = (u / 64) % 32, lane = u % 64;
    const int f = NET_W2 + (((g & 3) * 4 + (g >> 3)) * 2 + ((g >> 2) & 1)) * 512 + lane * 8;  // w2_frag's
    float v8[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v8[j] = net ? pack_one(critic, 1, f + j) : pack_one(actor, ACT, f + j);
    const P3 x = split8(v8);
    bf16x8* pieces = reinterpret_cast<bf16x8*>(out + PACKED_F);
#pragma unroll
    for (int p = 0; p < 3; p++) pieces[((net * 32 + g) * 3 + p) * 64 + lane] = x.p[p];
    return;
  }
  float v;
  if (idx < ACTOR_F) v = pack_one(actor, ACT, idx);
  else if (idx < LDS_F) v = pack_one(critic, 1, idx - ACTOR_F);
  else v = log_std[idx - LDS_F];
  out[idx] = v;
}

// the input fragment of one env: features 8 (lane>>5) .. + 7 (zero past feature 11)
__device__ __forceinline__ void load_xb(const float* __restrict__ x, int env, bool ok, float xb[8]) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int k = 0; k < 8; k++) xb[k] = ok && (h == 0 || k < 4) ? x[size_t(env) * OBS + 8 * h + k] : 0.f;
}


struct EpiArgs {  // QuadRolloutPost, flattened
  const float* reward;
  const uint8_t* terminated;
  const uint8_t* truncated;
  const float* terminal_obs;
  float* buf_rew;
  float* last_start;
  float* ep_ret;
  float* ep_len;
  double* stats;
  int32_t rows;
  float gamma;
};

// Everything a tile reads from HBM, loaded in one go (issued a tile ahead, see k_policy_act).
struct TileIn {
  float xb[8];           // X^T fragments of the obs rows
  float rew, ret, len;   // epilogue inputs (step t-1)
  uint32_t flags;        // bit0 terminated, bit1 truncated
};

__device__ __forceinline__ void load_tile(TileIn& in, const float* __restrict__ obs, const EpiArgs& e,
                                          bool pend, int env, bool ok) {
  load_xb(obs, env, ok, in.xb);
  in.rew = in.ret = in.len = 0.f;
  in.flags = 0u;
  if (pend && ok) {
    in.flags = uint32_t(e.terminated[env] != 0) | (uint32_t(e.truncated[env] != 0) << 1);
    in.rew = e.reward[env];
    in.ret = e.ep_ret[env];
    in.len = e.ep_len[env];
  }
}

// finish step t-1 for one tile: TimeLimit bootstrap r += gamma V(terminal_obs) where truncated and
// not terminated (critic only when the tile holds such an env), reward row, last_start, episode
// statistics (accumulated in st[3] of the h == 0 lanes). Returns the env's new last_start.
__device__ __forceinline__ float epilogue_tile(const float* __restrict__ Lc, const float* packed, const EpiArgs& e,
                                               const TileIn& in, int env, bool ok, size_t row, float st[3]) {
  const int h = (threadIdx.x & 63) >> 5;
  const bool term = in.flags & 1u, trunc = in.flags & 2u;
  const bool timeout = ok && trunc && !term;
  float tv = 0.f;
  if (__any(timeout)) {
    float xb[1][8], v[1][1];
    load_xb(e.terminal_obs, env, ok, xb[0]);
    net_forward<1, 1>(Lc, packed, xb, v);
    tv = v[0][0];
  }
  const bool done = term || trunc;
  if (ok && h == 0) {
    e.buf_rew[row + env] = timeout ? in.rew + e.gamma * tv : in.rew;
    const float ret = in.ret + in.rew, len = in.len + 1.f;
    if (done) { st[0] += ret; st[1] += len; st[2] += 1.f; }
    e.ep_ret[env] = done ? 0.f : ret;
    e.ep_len[env] = done ? 0.f : len;
    e.last_start[env] = done ? 1.f : 0.f;
  }
  return done ? 1.f : 0.f;
}

// block-reduce the episode statistics into this block's slot (uncontended atomics)
template <int BLK>
__device__ void flush_stats(double* stats, float st[3]) {
  __shared__ float red[3][BLK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    float v = st[j];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if (lane == 0) red[j][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float s = 0.f;
    for (int w = 0; w < BLK / 64; w++) s += red[threadIdx.x][w];
    if (s != 0.f) atomicAdd(&stats[(blockIdx.x % QUAD_POLICY_STAT_SLOTS) * 3 + threadIdx.x], double(s));
  }
}

// Last block to arrive applies `t_next` / `pending_next` to the cursor. Only READS of the cursor
// need ordering (every block has consumed t and pending before it arrives); the data the kernel
// wrote is published by the kernel boundary, so no release fence (an agent-scope release would
// write back every XCD's L2 in every block).
__device__ void cursor_arrive(uint32_t* cursor, uint32_t t_next, uint32_t pending_next, bool set_t) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(&cursor[CUR_ARRIVED], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      cursor[CUR_ARRIVED] = 0u;
      if (set_t) cursor[CUR_T] = t_next;
      cursor[CUR_PENDING] = pending_next;
    }
  }
}

struct ActArgs {
  const float* obs;         // [N,12]
  float* act_env;           // [N,4] clipped
  float* act;               // [T,N,4] unclipped sample or NULL
  float* logp;              // [T,N] or NULL
  float* value;             // [T,N] or NULL
  float* obs_copy;          // [T,N,12] or NULL
  const float* last_start;  // [N] or NULL
  float* starts;            // [T,N] or NULL
  uint32_t* cursor;         // {t, pending, arrivals} or NULL
  int32_t rows;
  int32_t deterministic;
  uint64_t seed;
  uint64_t env_base;
  int32_t n;
  int32_t fused;            // epilogue of step t-1 + cursor advance
};

// NT_ACT tiles per wave iteration (sharing weight fragments), BLK threads per block (one block per
// CU; BLK = 512 puts two waves on each SIMD, which caps a wave at 256 registers)
template <int NT_ACT, int BLK>
__global__ __launch_bounds__(BLK) void k_policy_act(const float* __restrict__ packed, ActArgs a, EpiArgs e) {
  extern __shared__ float lds[];
  constexpr int WAVES = BLK / 64;
  stage_lds<BLK>(lds, packed);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int tiles = (a.n + TILE - 1) / TILE;
  const uint32_t t = a.cursor ? a.cursor[CUR_T] : 0u;
  const bool pend = a.fused && a.cursor[CUR_PENDING] != 0u;
  const uint32_t rows = uint32_t(a.rows);
  const size_t row0 = size_t(t % rows) * a.n;
  const size_t rowp = size_t((t + rows - 1u) % rows) * a.n;
  const float* log_std = packed + LDS_F;
  float st[3] = {0.f, 0.f, 0.f};
  const int groups = (tiles + NT_ACT - 1) / NT_ACT;
  const int stride = gridDim.x * WAVES;
  int g = blockIdx.x * WAVES + wave;
  TileIn cur[NT_ACT];
#pragma unroll
  for (int j = 0; j < NT_ACT; j++) {
    const int env = (g * NT_ACT + j) * TILE + (lane & 31);
    load_tile(cur[j], a.obs, e, pend, env, g < groups && env < a.n);
  }
  for (; g < groups; g += stride) {
    // issue the next group's loads now; they land while this group runs on the matrix cores
    TileIn nxt[NT_ACT];
#pragma unroll
    for (int j = 0; j < NT_ACT; j++) {
      const int env = ((g + stride) * NT_ACT + j) * TILE + (lane & 31);
      load_tile(nxt[j], a.obs, e, pend, env, g + stride < groups && env < a.n);
    }
    int envs[NT_ACT];
    bool oks[NT_ACT];
    float ls[NT_ACT], xb[NT_ACT][8];
#pragma unroll
    for (int j = 0; j < NT_ACT; j++) {
      envs[j] = (g * NT_ACT + j) * TILE + (lane & 31);
      oks[j] = envs[j] < a.n;
      ls[j] = 0.f;
      if (pend) ls[j] = epilogue_tile(lds + ACTOR_F, packed, e, cur[j], envs[j], oks[j], rowp, st);
      else if (a.last_start && oks[j]) ls[j] = a.last_start[envs[j]];
#pragma unroll
      for (int k = 0; k < 8; k++) xb[j][k] = cur[j].xb[k];
    }
    float mean[NT_ACT][ACT], val[NT_ACT][1];
    net_forward2<NT_ACT>(lds, packed, xb, mean, val);
#pragma unroll
    for (int j = 0; j < NT_ACT; j++) {
      const int env = envs[j];
      cur[j] = nxt[j];
      if (!oks[j]) continue;
      if (a.obs_copy) {
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (h == 0 || k < 4) a.obs_copy[(row0 + env) * OBS + 8 * h + k] = xb[j][k];
      }
      if (h) continue;  // one lane per env from here
      if (a.starts) a.starts[row0 + env] = ls[j];
      float z[ACT] = {0.f, 0.f, 0.f, 0.f};
      if (!a.deterministic) gauss4(a.seed, a.env_base + uint64_t(env), t, z);
      float act[ACT], lp = 0.f;
#pragma unroll
      for (int k = 0; k < ACT; k++) {
        const float sd = expf(log_std[k]);
        act[k] = mean[j][k] + sd * z[k];
        const float zz = (act[k] - mean[j][k]) / sd;  // as PPO.train recomputes it (policy.log_prob)
        lp += -0.5f * zz * zz - log_std[k] - 0.91893853320467274f;  // 0.5 log(2 pi)
      }
      reinterpret_cast<float4*>(a.act_env)[env] =
          make_float4(fminf(fmaxf(act[0], -1.f), 1.f), fminf(fmaxf(act[1], -1.f), 1.f),
                      fminf(fmaxf(act[2], -1.f), 1.f), fminf(fmaxf(act[3], -1.f), 1.f));
      if (a.act) reinterpret_cast<float4*>(a.act + row0 * ACT)[env] = make_float4(act[0], act[1], act[2], act[3]);
      if (a.logp) a.logp[row0 + env] = lp;
      if (a.value) a.value[row0 + env] = val[j][0];
    }
  }
  if (a.fused) {
    if (pend) flush_stats<BLK>(e.stats, st);
    cursor_arrive(a.cursor, t + 1u, 1u, true);
  }
}

__global__ __launch_bounds__(PBLOCK) void k_rollout_post(const float* __restrict__ packed, EpiArgs e,
                                                         uint32_t* cursor, int32_t n) {
  extern __shared__ float lds[];
  if (cursor[CUR_PENDING] == 0u) return;  // grid-uniform: nothing to finish
  stage_lds<PBLOCK>(lds, packed);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tiles = (n + TILE - 1) / TILE;
  const uint32_t t = cursor[CUR_T], rows = uint32_t(e.rows);
  const size_t rowp = size_t((t + rows - 1u) % rows) * n;
  float st[3] = {0.f, 0.f, 0.f};
  for (int tile = blockIdx.x * 4 + wave; tile < tiles; tile += gridDim.x * 4) {
    const int env = tile * TILE + (lane & 31);
    TileIn in;
    load_tile(in, e.terminal_obs, e, true, env, env < n);  // xb unused here
    epilogue_tile(lds + ACTOR_F, packed, e, in, env, env < n, rowp, st);
  }
  flush_stats<PBLOCK>(e.stats, st);
  cursor_arrive(cursor, 0u, 0u, false);
}

int pfail(int code, const char* m) { return set_error(code, m); }

// the kernels take 152 KB of dynamic LDS (gfx950 has 160 KB per CU): opt in once per device
int lds_opt_in() {
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return pfail(QUAD_EHIP, "hipGetDevice failed");
  if (done[dev]) return QUAD_OK;
  const int bytes = LDS_F * int(sizeof(float));
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_policy_act<2, 256>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess ||

      hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rollout_post),
                          hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    return pfail(QUAD_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  done[dev] = true;
  return QUAD_OK;
}

int grid_for(int n, int nt, int waves) {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev]) {
    hipDeviceProp_t prop;
    cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const int groups = ((n + TILE - 1) / TILE + nt - 1) / nt;
  const int want = (groups + waves - 1) / waves;
  return want < cus[dev] ? want : cus[dev];  // one LDS-filling block per CU, grid-stride over tiles
}

EpiArgs epi_args(const QuadRolloutPost* p) {
  return EpiArgs{p->reward, p->terminated, p->truncated, p->terminal_obs, p->buf_rew, p->last_start,
                 p->ep_ret, p->ep_len, p->stats, p->rows, p->gamma};
}

int check_epi(const QuadRolloutPost* p) {
  if (!p->reward || !p->terminated || !p->truncated || !p->terminal_obs || !p->buf_rew ||
      !p->last_start || !p->ep_ret || !p->ep_len || !p->stats)
    return pfail(QUAD_EINVAL, "rollout epilogue: NULL buffer");
  if (p->rows < 1) return pfail(QUAD_EINVAL, "rollout epilogue: rows must be >= 1");
  return QUAD_OK;
}

}  // namespace

extern "C" {

int32_t quad_policy_packed_floats(void) { return PACKED_ALL_F; }

int quad_policy_pack(const QuadPolicyParams* p, float* packed, void* stream) {
  if (!p || !packed) return pfail(QUAD_EINVAL, "params/packed is NULL");
  if (!p->pi_w0 || !p->pi_b0 || !p->pi_w1 || !p->pi_b1 || !p->act_w || !p->act_b || !p->vf_w0 ||
      !p->vf_b0 || !p->vf_w1 || !p->vf_b1 || !p->val_w || !p->val_b || !p->log_std)
    return pfail(QUAD_EINVAL, "a policy parameter pointer is NULL");
  if (reinterpret_cast<uintptr_t>(packed) & 15u) return pfail(QUAD_EINVAL, "packed must be 16-byte aligned");
  if (int rc = lds_opt_in()) return rc;
  NetPtrs actor{p->pi_w0, p->pi_b0, p->pi_w1, p->pi_b1, p->act_w, p->act_b};
  NetPtrs critic{p->vf_w0, p->vf_b0, p->vf_w1, p->vf_b1, p->val_w, p->val_b};
  hipLaunchKernelGGL(k_policy_pack, dim3((PACKED_F + 2 * 32 * 64 + 2 * 4 * 64 + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), actor, critic, p->log_std, packed);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_policy_pack launch failed");
}

int quad_policy_act(const float* packed, const QuadPolicyAct* s, int32_t n, void* stream) {
  if (!packed || !s || !s->obs || !s->actions_env) return pfail(QUAD_EINVAL, "NULL argument");
  if (n <= 0) return pfail(QUAD_EINVAL, "n must be > 0");
  if (s->rows < 1) return pfail(QUAD_EINVAL, "rows must be >= 1");
  if ((reinterpret_cast<uintptr_t>(packed) | reinterpret_cast<uintptr_t>(s->actions_env) |
       reinterpret_cast<uintptr_t>(s->actions)) & 15u)
    return pfail(QUAD_EINVAL, "packed and action buffers must be 16-byte aligned");
  EpiArgs e{};
  if (s->epilogue) {
    if (!s->cursor) return pfail(QUAD_EINVAL, "a fused epilogue needs the cursor");
    if (int rc = check_epi(s->epilogue)) return rc;
    if (s->epilogue->rows != s->rows) return pfail(QUAD_EINVAL, "epilogue rows != rows");
    e = epi_args(s->epilogue);
  }
  if (int rc = lds_opt_in()) return rc;
  ActArgs a{s->obs, s->actions_env, s->actions, s->log_prob, s->value, s->obs_copy, s->last_start,
            s->episode_starts, s->cursor, s->rows, s->deterministic, s->seed, s->env_id_base, n,
            s->epilogue ? 1 : 0};
  // 2 tiles per wave, 4 waves per CU: measured best (8-wave blocks cap a wave at 256 registers and
  // spill)
  hipLaunchKernelGGL((k_policy_act<2, 256>), dim3(grid_for(n, 2, 4)), dim3(256), LDS_F * sizeof(float),
                     static_cast<hipStream_t>(stream), packed, a, e);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_policy_act launch failed");
}

int quad_rollout_post(const float* packed, const QuadRolloutPost* p, uint32_t* cursor, int32_t n,
                      void* stream) {
  if (!packed || !p || !cursor) return pfail(QUAD_EINVAL, "NULL argument");
  if (n <= 0) return pfail(QUAD_EINVAL, "n must be > 0");
  if (reinterpret_cast<uintptr_t>(packed) & 15u) return pfail(QUAD_EINVAL, "packed must be 16-byte aligned");
  if (int rc = check_epi(p)) return rc;
  if (int rc = lds_opt_in()) return rc;
  hipLaunchKernelGGL(k_rollout_post, dim3(grid_for(n, 1, 4)), dim3(PBLOCK), LDS_F * sizeof(float),
                     static_cast<hipStream_t>(stream), packed, epi_args(p), cursor, n);
  return hipGetLastError() == hipSuccess ? QUAD_OK : pfail(QUAD_EHIP, "k_rollout_post launch failed");
}

}  // extern "C"
