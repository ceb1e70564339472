// learner.h -- definitions shared by the two forms of the PPO minibatch-gradient kernel (device
// and host): learner.hip (f32-input MFMA, k_ppo_grad) and learner_x3.hip (bf16x3 split MFMA,
// k_ppo_grad_x3). Both write the same per-block partial image, summed by k_ppo_reduce.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "policy_net.h"

namespace quadenv {

namespace lrn {

constexpr int LB = 256;       // threads per block: 4 waves, one per SIMD
constexpr int RND = 64;       // rows per round (two 32-row MFMA tiles)
constexpr int ADV_BLOCKS = 256;
constexpr int MAX_NB = 128;   // blocks per net on average (the device has 256 CUs)

// per-net partial image (floats): W1 [128][12], b1, W2 [128][128], b2, W3 [NOUT][128], b3,
// log_std [4] (actor), then 4 statistic slots
constexpr int P_W1 = 0, P_B1 = P_W1 + H * OBS, P_W2 = P_B1 + H, P_B2 = P_W2 + H * H, P_W3 = P_B2 + H;
constexpr int P_B3A = P_W3 + ACT * H, P_LS = P_B3A + ACT, P_STATS = P_LS + ACT;  // 18,696
constexpr int P_B3C = P_W3 + H;
constexpr int PSTRIDE = P_STATS + 8;   // 18,704 (16-byte multiple)
static_assert(P_STATS == 18696 && P_B3C + 1 == 18305, "SB3 parameter counts (actor 18,696, critic 18,305)");

struct NetW {
  const float *w0, *b0, *w1, *b1, *w2, *b2;
};

struct GArgs {
  NetW actor, critic;
  const float* log_std;
  const float *obs, *act, *logp_old, *adv, *ret;
  const int64_t* idx;
  const double* adv_part;  // [ADV_BLOCKS][2] or NULL (no normalization)
  float* part;             // [nb + nbc][PSTRIDE]: actor blocks, then critic blocks
  int32_t batch, nb, per_block;     // actor: nb blocks of per_block rows
  int32_t nbc, per_block_c;         // critic: nbc blocks of per_block_c rows
  float clip, inv_batch, vf_coef;
  float* dump;  // diagnostics only (k_ppo_grad*_dump): [2 nets][batch][256] hidden pre-activations
  const void* wimg;  // bf16x3 form: the W2 fragments of every wave as bf16 pieces (k_split_w2, WIMG_BYTES)
};

struct Layout {
  int nb, per_block, nbc, per_block_c;
  int64_t part_bytes, adv_bytes, wimg_bytes;
};

// the bf16x3 form's pre-split W2 image (learner_x3.hip k_split_w2): 2 nets x 4 waves x 2 uses x
// 8 k-steps x 3 pieces x 64 lanes x 16 bytes, after the partial image in the workspace
constexpr int64_t WIMG_BYTES = int64_t(2) * 4 * 2 * 8 * 3 * 64 * 16;

// Block split of a minibatch of `batch` rows: the two nets share the 2 * MAX_NB block slots in
// proportion `actor_share` / 1000 (a critic round costs less than an actor round: no log-prob /
// ratio work). The partial image is sized for every split (nb + nbc <= slots).
inline Layout layout_of(int32_t batch, int actor_share) {
  Layout l{};
  const int rounds = (batch + RND - 1) / RND;
  const int slots = rounds < MAX_NB ? 2 * rounds : 2 * MAX_NB;
  int na = int((int64_t(slots) * actor_share + 500) / 1000);
  na = na < 1 ? 1 : (na > slots - 1 ? slots - 1 : na);
  l.nb = na < rounds ? na : rounds;
  l.nbc = slots - na < rounds ? slots - na : rounds;
  l.per_block = ((rounds + l.nb - 1) / l.nb) * RND;
  l.per_block_c = ((rounds + l.nbc - 1) / l.nbc) * RND;
  l.part_bytes = int64_t(slots) * PSTRIDE * int64_t(sizeof(float));
  l.adv_bytes = int64_t(ADV_BLOCKS) * 2 * int64_t(sizeof(double));
  l.wimg_bytes = WIMG_BYTES;
  return l;
}

// The bf16x3 form (learner_x3.hip): every block runs both nets over the same rows (the actor's
// rounds, then the critic's), X3_BLOCKS blocks = one per CU, so every CU carries the same work. A
// split of the CUs between the nets (the f32 form's actor share) left the slower net's blocks ~5 %
// longer than the average at any share (round granularity).
constexpr int X3_BLOCKS = 256;
inline Layout layout_both(int32_t batch) {
  Layout l{};
  const int rounds = (batch + RND - 1) / RND;
  const int nb = rounds < X3_BLOCKS ? rounds : X3_BLOCKS;
  l.nb = l.nbc = nb;
  l.per_block = l.per_block_c = ((rounds + nb - 1) / nb) * RND;
  l.part_bytes = int64_t(2) * nb * PSTRIDE * int64_t(sizeof(float));
  l.adv_bytes = int64_t(ADV_BLOCKS) * 2 * int64_t(sizeof(double));
  l.wimg_bytes = WIMG_BYTES;
  return l;
}
// k_x3_prep (the W2 split, + the advantage statistics when adv_stats != NULL) + k_ppo_grad_x3
int launch_ppo_grad_x3(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv);
int launch_ppo_grad_x3_dump(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv);

// Block `blk` of the minibatch advantage statistics (sum and sum of squares in float64; fixed
// order: per-thread strided over i = blk * 256 + tid + k * ADV_BLOCKS * 256, then a tree) into
// part[2 blk], part[2 blk + 1]. The index loads and the gathers go out 8 at a time (the sums keep the
// same order): one at a time, each thread waited out 8 dependent HBM round trips (12.4 us per
// 524,288-row minibatch under rocprof). Needs 256 threads and `red` [2][256] in LDS.
__device__ __forceinline__ void adv_stats_block(const float* __restrict__ adv, const int64_t* __restrict__ idx,
                                                int batch, double* __restrict__ part, int blk, double (*red)[256]) {
  const int tid = threadIdx.x;
  double s = 0.0, s2 = 0.0;
  constexpr int STRIDE = ADV_BLOCKS * 256, U = 8;
  for (int i0 = blk * 256 + tid; i0 < batch; i0 += U * STRIDE) {
    int64_t j[U];
#pragma unroll
    for (int u = 0; u < U; u++) j[u] = i0 + u * STRIDE < batch ? idx[i0 + u * STRIDE] : int64_t(-1);
    float v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = j[u] >= 0 ? adv[j[u]] : 0.f;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (j[u] < 0) continue;
      const double d = v[u];
      s += d;
      s2 += d * d;
    }
  }
  red[0][tid] = s;
  red[1][tid] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) { red[0][tid] += red[0][tid + o]; red[1][tid] += red[1][tid + o]; }
    __syncthreads();
  }
  if (tid == 0) { part[2 * blk] = red[0][0]; part[2 * blk + 1] = red[1][0]; }
}

// Diagnostics (quad_ppo_hidden): the kernels' own hidden pre-activations of minibatch row `pos`
// (before the ReLU; layer 0 = h1, 1 = h2) -- the dump instantiation of the same body, so the same
// arithmetic as the gradient launch
__device__ __forceinline__ void dump_pre(float* dump, int net, int batch, int pos, int layer, int neuron, float v) {
  dump[(size_t(net) * size_t(batch) + size_t(pos)) * 256 + size_t(128 * layer + neuron)] = v;
}

}  // namespace lrn
}  // namespace quadenv
