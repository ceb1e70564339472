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

// the bf16x3 form (learner_x3.hip): its actor share and launcher
int x3_actor_share();
int launch_ppo_grad_x3(const GArgs& g, hipStream_t s);  // k_split_w2 + k_ppo_grad_x3
int launch_ppo_grad_x3_dump(const GArgs& g, hipStream_t s);

// Diagnostics (quad_ppo_hidden): the kernels' own hidden pre-activations of minibatch row `pos`
// (before the ReLU; layer 0 = h1, 1 = h2) -- the dump instantiation of the same body, so the same
// arithmetic as the gradient launch
__device__ __forceinline__ void dump_pre(float* dump, int net, int batch, int pos, int layer, int neuron, float v) {
  dump[(size_t(net) * size_t(batch) + size_t(pos)) * 256 + size_t(128 * layer + neuron)] = v;
}

}  // namespace lrn
}  // namespace quadenv
