// learner.hip -- the PPO minibatch gradient (row P) of the 12-128-128 actor / critic on MFMA.
//
// SB3 PPO.train (stable_baselines3/ppo/ppo.py, third-party; driven by the reference's train.py:50-68)
// takes 2,560 Adam steps per update at the reference schedule; at 65,536 envs each minibatch is
// 524,288 rows and its forward + backward is ~200 GFLOP of tall-skinny products that the BLAS
// path (ppo/ppo.py + policy._SplitKLinear) runs at ~30 TF/s. This file computes the whole minibatch
// gradient of both nets in one launch (plus a stats pre-pass and a partial-sum reduction).
//
// Work split. One 256-thread block per CU works on ONE net (blocks [0, nb) the actor, [nb, nb + nbc)
// the critic) over a contiguous slice of the minibatch, in rounds of 64 rows (two 32-row tiles).
// Wave w owns neurons 32w..32w+31 of BOTH hidden layers, so its rows of W2 and its columns of W2
// stay in registers for the whole launch (128 VGPRs of MFMA A/B fragments) and each wave
// accumulates its own 32-row slab of dW2 / dW1 / db in registers across all rounds. The waves
// exchange activations through [row][neuron] LDS images (stride 130 floats: conflict-free for the
// column reads and 8-byte aligned for the paired reads). Per round (v_mfma_f32_32x32x2_f32 only,
// exact f32 fma chains; "E" = a 32x32 accumulator with neurons in registers and rows on lanes,
// "R" = rows in registers and neurons on lanes):
//   L1   h1^T = W1 x^T           E, 12 MFMAs          -> H1 image (relu)
//   L2   h2^T = W2 h1^T          E, 128 MFMAs         (A = W2 rows in registers, B = H1 image)
//   head partial sums over the wave's 32 neurons -> LDS; every wave then forms mean / value,
//        the loss terms and dL/dmean (dL/dV) of its rows (same order in every wave)
//   dh2 = relu'(h2) . (W3^T dmean) E, VALU          -> DH2 image, relu(h2) -> H2 image
//   dW2  = dh2^T h1  (K = rows)  128 MFMAs          (A = DH2 column block w, B = H1 image)
//   dW3  = dmean^T h2            32 16x16x4 MFMAs   (A = dL/dmean image, B = H2 image)
//   dh1  = relu'(h1) . dh2 W2    R, 128 MFMAs        (A = DH2 rows, B = W2 columns in registers)
//   dW1  = dh1^T x               32 MFMAs            (dh1 accumulator used directly as A^T)
// Block partials go to the workspace in the parameter layout; k_ppo_reduce sums them in block
// order (deterministic) into the parameter-shaped gradients.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../../include/quadenv.h"
#include "learner.h"
#include "policy_net.h"

namespace quadenv {

int set_error(int code, const char* msg);  // quadenv.hip

namespace {

using namespace lrn;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SH = 130;       // row stride (floats) of the [row][neuron] images
constexpr int SO = 13;        // row stride of the observation image (odd: conflict-free columns)
// measured: 500 -> 1.30 ms, 525 -> 1.26, 540 -> 1.22-1.25, 550 -> 1.23, 580 -> 1.32
constexpr int ACTOR_SHARE = 540;  // per mille of the block slots that run the actor

// LDS image (floats)
constexpr int L_H1 = 0, L_DH2 = L_H1 + RND * SH, L_H2 = L_DH2 + RND * SH;
constexpr int L_OBS = L_H2 + RND * SH;          // 2 buffers (round parity)
constexpr int L_SC = L_OBS + 2 * RND * SO;      // 2 buffers of [64][8] row scalars: action 4, old logp, adv, return
constexpr int L_DM = L_SC + 2 * RND * 8;        // [64][4] dL/dmean (dL/dV in column 0)
constexpr int L_PART = L_DM + RND * 4;          // [4 waves][64][4] head partial sums
constexpr int L_W3T = L_PART + 4 * RND * 4;     // [128][4] head weights, neuron-major
constexpr int L_B1 = L_W3T + H * 4, L_B2 = L_B1 + H;
constexpr int L_TOTAL = L_B2 + H;               // 29,704 floats = 116 KB
static_assert(L_H1 % 2 == 0 && L_DH2 % 2 == 0 && SH % 2 == 0, "paired reads need 8-byte alignment");
static_assert(L_W3T % 4 == 0 && L_SC % 4 == 0, "float4 LDS reads");

// pair-step k order: MFMA step s of lane half h reads neuron 4(s/2) + 2h + (s&1), so two
// consecutive steps of a lane read two adjacent floats (one ds_read_b64)
__device__ __forceinline__ int kperm(int s, int h) { return 4 * (s >> 1) + 2 * h + (s & 1); }

__device__ __forceinline__ float2 ld2(const float* L, int off) { return *reinterpret_cast<const float2*>(L + off); }

template <int NOUT, bool DUMP = false>
__device__ __forceinline__ void body(const GArgs& g, float* __restrict__ L, int blk) {
  const NetW& W = NOUT == ACT ? g.actor : g.critic;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int n_own = 32 * w + l32;  // this lane's neuron in the lane-indexed forms

  // ---- advantage statistics of the minibatch (actor): fixed-order tree over the pre-pass partials
  __shared__ double red[2][LB];
  float adv_mu = 0.f, adv_den = 1.f;
  if (NOUT == ACT && g.adv_part) {
    red[0][tid] = g.adv_part[2 * tid];
    red[1][tid] = g.adv_part[2 * tid + 1];
    __syncthreads();
    for (int o = LB / 2; o > 0; o >>= 1) {
      if (tid < o) { red[0][tid] += red[0][tid + o]; red[1][tid] += red[1][tid + o]; }
      __syncthreads();
    }
    const double n = double(g.batch), s = red[0][0], s2 = red[1][0];
    const double var = fmax((s2 - s * s / n) / (n - 1.0), 0.0);
    adv_mu = float(s / n);
    adv_den = float(sqrt(var)) + 1e-8f;
  }
  const float adv_rden = 1.f / adv_den;

  // ---- stage the small weights in LDS, the wave's W1 / W2 fragments in registers
  for (int i = tid; i < H; i += LB) {
    L[L_B1 + i] = W.b0[i];
    L[L_B2 + i] = W.b1[i];
#pragma unroll
    for (int k = 0; k < 4; k++) L[L_W3T + 4 * i + k] = k < NOUT ? W.w2[k * H + i] : 0.f;
  }
  float b3[NOUT];
#pragma unroll
  for (int k = 0; k < NOUT; k++) b3[k] = W.b2[k];
  float w1f[6];
#pragma unroll
  for (int s = 0; s < 6; s++) w1f[s] = W.w0[n_own * OBS + 2 * s + h];
  float w2r[64], w2c[64];  // W2[n_own][kperm(s)] (A of L2), W2[kperm(s)][n_own] (B of dh1)
#pragma unroll
  for (int s = 0; s < 64; s++) {
    w2r[s] = W.w1[n_own * H + kperm(s, h)];
    w2c[s] = W.w1[kperm(s, h) * H + n_own];
  }
  float ls[ACT], sd[ACT], isd[ACT];  // isd: the row loop multiplies (a full-precision division is ~10 VALU)
  if constexpr (NOUT == ACT) {
#pragma unroll
    for (int k = 0; k < ACT; k++) { ls[k] = g.log_std[k]; sd[k] = expf(ls[k]); isd[k] = 1.f / sd[k]; }
  }

  // accumulators (whole launch)
  f32x16 dW2[4], dW1;
  f32x4 dW3[2];
#pragma unroll
  for (int r = 0; r < 16; r++) {
    dW1[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j++) dW2[j][r] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) { dW3[0][r] = 0.f; dW3[1][r] = 0.f; }
  float db1 = 0.f, db2 = 0.f;
  float db3[NOUT], dls[ACT], st[3] = {0.f, 0.f, 0.f};  // st: pg sum, vf sum, clipped count
#pragma unroll
  for (int k = 0; k < NOUT; k++) db3[k] = 0.f;
#pragma unroll
  for (int k = 0; k < ACT; k++) dls[k] = 0.f;
  const bool acc_lane = w == 0 && h == 0;  // one lane per row accumulates the per-row sums

  const int per_block = NOUT == ACT ? g.per_block : g.per_block_c;
  const int s0 = blk * per_block;
  const int s1 = min(g.batch, s0 + per_block);
  const int rounds = s1 > s0 ? (s1 - s0 + RND - 1) / RND : 0;
  // Row staging, one round ahead: threads 0..191 gather the observation rows (float4 each),
  // threads 192..255 the row scalars; the minibatch indices are loaded two rounds ahead, so no
  // gather waits on its index load. Rows past the slice stage zeros (and are masked as invalid).
  const int srow = tid < 3 * RND ? tid / 3 : tid - 3 * RND;
  auto index_of = [&](int rd) -> int64_t {
    const int i = s0 + rd * RND + srow;
    return (rd < rounds && i < s1) ? g.idx[i] : int64_t(-1);
  };
  float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
  float pfs[3] = {0.f, 0.f, 0.f};
  auto gather = [&](int64_t row) {
    pf = make_float4(0.f, 0.f, 0.f, 0.f);
    pfs[0] = pfs[1] = pfs[2] = 0.f;
    if (row < 0) return;
    if (tid < 3 * RND) {
      pf = reinterpret_cast<const float4*>(g.obs)[size_t(row) * 3 + tid % 3];
    } else if (NOUT == ACT) {
      pf = reinterpret_cast<const float4*>(g.act)[row];
      pfs[0] = g.logp_old[row];
      pfs[1] = g.adv[row];
    } else {
      pfs[2] = g.ret[row];
    }
  };
  gather(index_of(0));
  int64_t next_row = index_of(1);
  __syncthreads();

  for (int rd = 0; rd < rounds; rd++) {
    const int base = s0 + rd * RND;
    float* OBSI = L + L_OBS + (rd & 1) * RND * SO;
    float* SCI = L + L_SC + (rd & 1) * RND * 8;
    if (tid < 3 * RND) {
      float* o = OBSI + srow * SO + 4 * (tid % 3);
      o[0] = pf.x; o[1] = pf.y; o[2] = pf.z; o[3] = pf.w;
    } else {
      *reinterpret_cast<float4*>(SCI + srow * 8) = pf;
      SCI[srow * 8 + 4] = pfs[0]; SCI[srow * 8 + 5] = pfs[1]; SCI[srow * 8 + 6] = pfs[2];
    }
    gather(next_row);           // round rd + 1, in flight during this round
    next_row = index_of(rd + 2);
    bool valid[2];
#pragma unroll
    for (int t = 0; t < 2; t++) valid[t] = base + 32 * t + l32 < s1;
    __syncthreads();  // B1: observation image complete; the previous round's readers are done

    // ---- L1 (E form): h1^T block w of both tiles -> H1 image
#pragma unroll
    for (int t = 0; t < 2; t++) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = L[L_B1 + 32 * w + acc_row(r, h)];
#pragma unroll
      for (int s = 0; s < 6; s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[s], OBSI[(32 * t + l32) * SO + 2 * s + h], acc, 0, 0, 0);
      if constexpr (DUMP) {
        if (valid[t])
          for (int r = 0; r < 16; r++) dump_pre(g.dump, NOUT == ACT ? 0 : 1, g.batch, base + 32 * t + l32, 0, 32 * w + acc_row(r, h), acc[r]);
      }
      float* row = L + L_H1 + (32 * t + l32) * SH + 32 * w;
#pragma unroll
      for (int r = 0; r < 16; r += 2)  // rows acc_row(r), acc_row(r)+1 are adjacent neurons
        *reinterpret_cast<float2*>(row + acc_row(r, h)) = make_float2(relu(acc[r]), relu(acc[r + 1]));
    }
    __syncthreads();  // B2: H1 image complete

    // ---- L2 (E form): h2^T block w, A = W2 rows (registers), B = H1 image (paired reads)
    f32x16 h2[2];
#pragma unroll
    for (int r = 0; r < 16; r++) h2[0][r] = L[L_B2 + 32 * w + acc_row(r, h)];
    h2[1] = h2[0];
#if !defined(QD_LRN_NOL2)  // QD_LRN_*: cost-ablation builds of tools/learner_variants.sh only
#pragma unroll
    for (int m = 0; m < 32; m++) {
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const float2 b = ld2(L, L_H1 + (32 * t + l32) * SH + 4 * m + 2 * h);
        h2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w2r[2 * m], b.x, h2[t], 0, 0, 0);
        h2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w2r[2 * m + 1], b.y, h2[t], 0, 0, 0);
      }
    }
#endif
    if constexpr (DUMP) {
      for (int t = 0; t < 2; t++)
        if (valid[t])
          for (int r = 0; r < 16; r++) dump_pre(g.dump, NOUT == ACT ? 0 : 1, g.batch, base + 32 * t + l32, 1, 32 * w + acc_row(r, h), h2[t][r]);
    }
    // head partial sums over the wave's 32 neurons (the two lane halves hold 16 each)
    float part[2][NOUT];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
      for (int k = 0; k < NOUT; k++) part[t][k] = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        h2[t][r] = relu(h2[t][r]);
        const float4 w3 = *reinterpret_cast<const float4*>(L + L_W3T + 4 * (32 * w + acc_row(r, h)));
        const float wk[4] = {w3.x, w3.y, w3.z, w3.w};
#pragma unroll
        for (int k = 0; k < NOUT; k++) part[t][k] = fmaf(wk[k], h2[t][r], part[t][k]);
      }
#pragma unroll
      for (int k = 0; k < NOUT; k++) {
        const float o = __shfl_xor(part[t][k], 32);
        if (h == 0) L[L_PART + (w * RND + 32 * t + l32) * 4 + k] = part[t][k] + o;
      }
    }
    __syncthreads();  // B3: head partials complete

    // ---- per-row loss terms and dL/d(head output) (every wave, identical arithmetic)
    float d[2][NOUT];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int e = 32 * t + l32;
      float out[NOUT];
#pragma unroll
      for (int k = 0; k < NOUT; k++)
        out[k] = (((L[L_PART + e * 4 + k] + L[L_PART + (RND + e) * 4 + k]) + L[L_PART + (2 * RND + e) * 4 + k]) +
                  L[L_PART + (3 * RND + e) * 4 + k]) + b3[k];
      const float4 a4 = *reinterpret_cast<const float4*>(SCI + e * 8);
      const float a4k[4] = {a4.x, a4.y, a4.z, a4.w};
      if constexpr (NOUT == ACT) {
        float z[ACT], lp = 0.f;
#pragma unroll
        for (int k = 0; k < ACT; k++) {
          z[k] = (a4k[k] - out[k]) * isd[k];
          lp += -0.5f * z[k] * z[k] - ls[k] - 0.91893853320467274f;
        }
        // ratio = exp(logp - old) on the hardware exp2 (~1 ulp; the correctly rounded expf is ~10 VALU)
        const float r = __builtin_amdgcn_exp2f((lp - SCI[e * 8 + 4]) * 1.44269504088896341f);
        const float A = g.adv_part ? (SCI[e * 8 + 5] - adv_mu) * adv_rden : SCI[e * 8 + 5];
        const float cr = fminf(fmaxf(r, 1.f - g.clip), 1.f + g.clip);
        const float sa = A * r, sb = A * cr;
        const float w1 = sa < sb ? 1.f : (sa == sb ? 0.5f : 0.f);
        const float inr = (r >= 1.f - g.clip && r <= 1.f + g.clip) ? 1.f : 0.f;
        const float dlp = valid[t] ? -g.inv_batch * A * (w1 + (1.f - w1) * inr) * r : 0.f;
#pragma unroll
        for (int k = 0; k < ACT; k++) d[t][k] = dlp * z[k] * isd[k];
        if (acc_lane && valid[t]) {
          st[0] += -fminf(sa, sb);
          st[2] += fabsf(r - 1.f) > g.clip ? 1.f : 0.f;
#pragma unroll
          for (int k = 0; k < ACT; k++) dls[k] += dlp * (z[k] * z[k] - 1.f);
        }
      } else {
        const float diff = out[0] - SCI[e * 8 + 6];
        d[t][0] = valid[t] ? 2.f * g.vf_coef * g.inv_batch * diff : 0.f;
        if (acc_lane && valid[t]) st[1] += diff * diff;
      }
      if (acc_lane) {
#pragma unroll
        for (int k = 0; k < NOUT; k++) {
          db3[k] += d[t][k];
          L[L_DM + e * 4 + k] = d[t][k];
        }
      }
    }
    // ---- dh2 (E form) -> DH2 image; relu(h2) -> H2 image
#pragma unroll
    for (int t = 0; t < 2; t++) {
      float* rowd = L + L_DH2 + (32 * t + l32) * SH + 32 * w;
      float* rowh = L + L_H2 + (32 * t + l32) * SH + 32 * w;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const float4 w3 = *reinterpret_cast<const float4*>(L + L_W3T + 4 * (32 * w + acc_row(r + u, h)));
          const float wk[4] = {w3.x, w3.y, w3.z, w3.w};
          float gsum = 0.f;
#pragma unroll
          for (int k = 0; k < NOUT; k++) gsum = fmaf(wk[k], d[t][k], gsum);
          v[u] = h2[t][r + u] > 0.f ? gsum : 0.f;
        }
        *reinterpret_cast<float2*>(rowd + acc_row(r, h)) = make_float2(v[0], v[1]);
        *reinterpret_cast<float2*>(rowh + acc_row(r, h)) = make_float2(h2[t][r], h2[t][r + 1]);
      }
    }
    __syncthreads();  // B4: DH2, H2 and dL/dmean images complete

#if !defined(QD_LRN_NODW)
    // ---- dW2 slab (rows 32w..): K = the round's 64 rows; db2 from the same A fragments
#pragma unroll 8  // (measured: full 1.226 ms, 8 1.204, 4 1.208, 2 1.234)
    for (int s = 0; s < 32; s++) {
      const int e = 2 * s + h;
      const float a = L[L_DH2 + e * SH + n_own];
      db2 += a;
#pragma unroll
      for (int j = 0; j < 4; j++)
        dW2[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, L[L_H1 + e * SH + 32 * j + l32], dW2[j], 0, 0, 0);
    }
    // ---- dW3 columns 32w.. (16x16x4: A = dL/dmean^T (rows = outputs), B = relu(h2) rows)
#pragma unroll
    for (int s = 0; s < 16; s++) {
      const int e = 4 * s + (lane >> 4), k = lane & 15;
      const float a = k < NOUT ? L[L_DM + e * 4 + k] : 0.f;
#pragma unroll
      for (int b = 0; b < 2; b++)
        dW3[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, L[L_H2 + e * SH + 32 * w + 16 * b + k], dW3[b], 0, 0, 0);
    }
#endif
#if !defined(QD_LRN_NODH1)
    // ---- dh1 (R form) = relu'(h1) . (dh2 W2[:, block w]); then db1 and the dW1 slab
#pragma unroll
    for (int t = 0; t < 2; t++) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
      for (int m = 0; m < 32; m++) {
        const float2 a = ld2(L, L_DH2 + (32 * t + l32) * SH + 4 * m + 2 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w2c[2 * m], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w2c[2 * m + 1], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; r++) {  // register r: row 32t + acc_row(r, h), neuron n_own
        const int e = 32 * t + acc_row(r, h);
        acc[r] = L[L_H1 + e * SH + n_own] > 0.f ? acc[r] : 0.f;
        db1 += acc[r];
      }
      // dW1[n][f] += sum_rows dh1[row][n] x[row][f]: register r is the A^T fragment of k-step r
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int e = 32 * t + acc_row(r, h);
        const float b = l32 < OBS ? OBSI[e * SO + l32] : 0.f;
        dW1 = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[r], b, dW1, 0, 0, 0);
      }
    }
#endif
  }

  // ---- block partials in the parameter layout
  float* P = g.part + size_t(blk + (NOUT == ACT ? 0 : g.nb)) * PSTRIDE;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int n = 32 * w + acc_row(r, h);
    if (l32 < OBS) P[P_W1 + n * OBS + l32] = dW1[r];
#pragma unroll
    for (int j = 0; j < 4; j++) P[P_W2 + n * H + 32 * j + l32] = dW2[j][r];
  }
  {
    const float o1 = __shfl_xor(db1, 32), o2 = __shfl_xor(db2, 32);
    if (h == 0) { P[P_B1 + n_own] = db1 + o1; P[P_B2 + n_own] = db2 + o2; }
  }
  if (lane < 16) {
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int r = 0; r < NOUT; r++) P[P_W3 + r * H + 32 * w + 16 * b + lane] = dW3[b][r];
  }
  if (w == 0) {  // lanes 0..31 hold the per-row sums (lanes 32..63 hold zeros)
    float v[NOUT + ACT + 3];
    int nv = 0;
#pragma unroll
    for (int k = 0; k < NOUT; k++) v[nv++] = db3[k];
#pragma unroll
    for (int k = 0; k < ACT; k++) v[nv++] = dls[k];
#pragma unroll
    for (int k = 0; k < 3; k++) v[nv++] = st[k];
#pragma unroll
    for (int q = 0; q < NOUT + ACT + 3; q++) {
      float x = v[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
      v[q] = x;
    }
    if (lane == 0) {
      const int b3off = NOUT == ACT ? P_B3A : P_B3C;
#pragma unroll
      for (int k = 0; k < NOUT; k++) P[b3off + k] = v[k];
      if (NOUT == ACT) {
#pragma unroll
        for (int k = 0; k < ACT; k++) P[P_LS + k] = v[NOUT + k];
      }
#pragma unroll
      for (int k = 0; k < 3; k++) P[P_STATS + k] = v[NOUT + ACT + k];
    }
  }
}

__global__ __launch_bounds__(LB, 1) void k_ppo_grad(GArgs g) {
  extern __shared__ float lds[];
  if (int(blockIdx.x) < g.nb) body<ACT>(g, lds, blockIdx.x);
  else body<1>(g, lds, blockIdx.x - g.nb);
}

__global__ __launch_bounds__(LB, 1) void k_ppo_grad_dump(GArgs g) {
  extern __shared__ float lds_d[];
  if (int(blockIdx.x) < g.nb) body<ACT, true>(g, lds_d, blockIdx.x);
  else body<1, true>(g, lds_d, blockIdx.x - g.nb);
}

// minibatch sums of adv and adv^2 in float64 (adv_stats_block, learner.h)
__global__ __launch_bounds__(256) void k_adv_stats(const float* __restrict__ adv, const int64_t* __restrict__ idx,
                                                   int batch, double* __restrict__ part) {
  __shared__ double red[2][256];
  adv_stats_block(adv, idx, batch, part, blockIdx.x, red);
}

// every minibatch of an epoch: block (b, m) is block b of minibatch m's statistics
__global__ __launch_bounds__(256) void k_adv_stats_epoch(const float* __restrict__ adv, const int64_t* __restrict__ perm,
                                                         int batch, double* __restrict__ sums) {
  __shared__ double red[2][256];
  const size_t m = blockIdx.y;
  adv_stats_block(adv, perm + m * size_t(batch), batch, sums + m * QUAD_ADV_SUM_DOUBLES, blockIdx.x, red);
}
static_assert(QUAD_ADV_SUM_DOUBLES == 2 * ADV_BLOCKS, "ABI constant");

struct RArgs {
  QuadPolicyGrads gr;
  const float* part;
  const float* log_std;
  float* stats;
  int32_t nb, nbc;
  float inv_batch, ent_coef;
};

// (net, parameter) sums of the nb block partials, in float64 (the partials of a bias or head
// gradient are sums over disjoint row sets that largely cancel): 64 parameters per block, each
// summed by 4 threads over consecutive quarters of the blocks (block order within a quarter), the
// quarters then added in order. One thread per parameter left 147 blocks to stream the 38 MB
// partial image of the bf16x3 form (13.3 us)
constexpr int RQ = 4;
__global__ __launch_bounds__(256) void k_ppo_reduce(RArgs a) {
  __shared__ double qs[RQ][64];
  const int pl = threadIdx.x & 63, qt = threadIdx.x >> 6;
  const int q = blockIdx.x * 64 + pl;
  const bool live = q < 2 * PSTRIDE;
  const int net = live ? q / PSTRIDE : 0, p = live ? q % PSTRIDE : 0;
  const float* src = a.part + size_t(net) * a.nb * PSTRIDE + p;
  const int nb = net ? a.nbc : a.nb;
  const int per = (nb + RQ - 1) / RQ, b0 = qt * per, b1 = min(nb, b0 + per);
  double sd = 0.0;
  int b = b0;
  if (live) {
    for (; b + 8 <= b1; b += 8) {  // 8 loads in flight per thread; summed in block order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) v[u] = src[size_t(b + u) * PSTRIDE];
#pragma unroll
      for (int u = 0; u < 8; u++) sd += double(v[u]);
    }
    for (; b < b1; b++) sd += double(src[size_t(b) * PSTRIDE]);
  }
  qs[qt][pl] = sd;
  __syncthreads();
  if (qt != 0 || !live) return;
  const float s = float(((qs[0][pl] + qs[1][pl]) + qs[2][pl]) + qs[3][pl]);
  const QuadPolicyGrads& g = a.gr;
  if (p < P_B1) { (net ? g.vf_w0 : g.pi_w0)[p - P_W1] = s; return; }
  if (p < P_W2) { (net ? g.vf_b0 : g.pi_b0)[p - P_B1] = s; return; }
  if (p < P_B2) { (net ? g.vf_w1 : g.pi_w1)[p - P_W2] = s; return; }
  if (p < P_W3) { (net ? g.vf_b1 : g.pi_b1)[p - P_B2] = s; return; }
  if (net == 0) {
    if (p < P_B3A) { g.act_w[p - P_W3] = s; return; }
    if (p < P_LS) { g.act_b[p - P_B3A] = s; return; }
    if (p < P_STATS) { g.log_std[p - P_LS] = s - a.ent_coef; return; }  // + d(-ent_coef * entropy)
  } else {
    if (p < P_B3C) { g.val_w[p - P_W3] = s; return; }
    if (p == P_B3C) { g.val_b[0] = s; return; }
  }
  if (!a.stats) return;
  // statistics: pg (actor slot 0), vf (critic slot 1), clipped count (actor slot 2)
  if (net == 0 && p == P_STATS) a.stats[0] = s * a.inv_batch;
  if (net == 1 && p == P_STATS + 1) a.stats[1] = s * a.inv_batch;
  if (net == 0 && p == P_STATS + 2) a.stats[3] = s * a.inv_batch;
  if (net == 0 && p == P_STATS + 3) {
    float e = 0.f;
    for (int k = 0; k < ACT; k++) e += 0.5f + 0.91893853320467274f + a.log_std[k];
    a.stats[2] = e;
  }
}

// ---- the epoch permutation of PPO.train (SB3: indices = np.random.permutation(buffer_size)).
// A keyed bijection of [0, 2^(2k)) -- a 4-round balanced Feistel network whose round function is a
// 32-bit integer hash of (half, key, round) -- walked until it lands in [0, n) (cycle walking:
// a permutation of the 2^(2k) >= n codes restricted to [0, n) is a permutation of [0, n); with
// 2^(2k) < 4n the expected walk is < 4 steps). One thread per output index, no sort: the
// torch.randperm it replaces sorts 67 M random keys per epoch (5.3 ms at config 3).
__host__ __device__ __forceinline__ uint32_t perm_hash(uint32_t x, uint32_t k) {
  x ^= k;
  x *= 0x7feb352du; x ^= x >> 15;
  x *= 0x846ca68bu; x ^= x >> 16;
  x *= 0x7feb352du; x ^= x >> 15;
  return x;
}

__host__ __device__ __forceinline__ uint64_t perm_feistel(uint64_t x, int half_bits, uint64_t seed) {
  const uint32_t mask = half_bits >= 32 ? 0xffffffffu : ((1u << half_bits) - 1u);
  uint32_t L = uint32_t(x >> half_bits) & mask, R = uint32_t(x) & mask;
#pragma unroll
  for (uint32_t r = 0; r < 4; r++) {
    const uint32_t k = uint32_t(seed >> (r & 1 ? 32 : 0)) + 0x9e3779b9u * (r + 1u);
    const uint32_t nl = R, nr = (L ^ perm_hash(R, k)) & mask;
    L = nl; R = nr;
  }
  return (uint64_t(L) << half_bits) | R;
}

__global__ __launch_bounds__(256) void k_permutation(int64_t n, int half_bits, uint64_t seed, int64_t* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    uint64_t x = uint64_t(i);
    do { x = perm_feistel(x, half_bits, seed); } while (x >= uint64_t(n));
    out[i] = int64_t(x);
  }
}

int lfail(int code, const char* m) { return set_error(code, m); }

// ---- fused clip_grad_norm_ + Adam (quad_clip_adam)
constexpr int ADAM_BLOCK = 256;

struct AdamArgs {
  QuadAdam a;
  int32_t offs[QUAD_ADAM_MAX_TENSORS + 1];  // prefix sums of numel
  float* part;                              // [nblocks] sums of squares
  int32_t nblocks;
};

__device__ __forceinline__ int tensor_of(const AdamArgs& g, int i) {
  int t = 0;
#pragma unroll
  for (int k = 1; k < QUAD_ADAM_MAX_TENSORS; k++) t += (k < g.a.count && i >= g.offs[k]) ? 1 : 0;
  return t;
}

// per-block sums of squared gradients (fixed-order tree); block 0 advances the step counters
__global__ __launch_bounds__(ADAM_BLOCK) void k_grad_sumsq(AdamArgs g) {
  __shared__ float red[ADAM_BLOCK];
  const int i = blockIdx.x * ADAM_BLOCK + threadIdx.x;
  float v = 0.f;
  if (i < g.offs[g.a.count]) {
    const int t = tensor_of(g, i);
    const float x = g.a.grads[t][i - g.offs[t]];
    v = x * x;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = ADAM_BLOCK / 2; o > 0; o >>= 1) {
    if (int(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) g.part[blockIdx.x] = red[0];
  if (blockIdx.x == 0 && int(threadIdx.x) < g.a.count) g.a.step[threadIdx.x][0] += 1.f;
}

// every block reduces the partials in the same order (same norm everywhere), then clips + updates
__global__ __launch_bounds__(ADAM_BLOCK) void k_adam(AdamArgs g) {
  __shared__ float red[ADAM_BLOCK];
  float v = 0.f;
  for (int b = threadIdx.x; b < g.nblocks; b += ADAM_BLOCK) v += g.part[b];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = ADAM_BLOCK / 2; o > 0; o >>= 1) {
    if (int(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const int i = blockIdx.x * ADAM_BLOCK + threadIdx.x;
  if (i >= g.offs[g.a.count]) return;
  const int t = tensor_of(g, i), j = i - g.offs[t];
  float gr = g.a.grads[t][j];
  if (g.a.max_grad_norm > 0.f) {
    const float coef = fminf(g.a.max_grad_norm / (sqrtf(red[0]) + 1e-6f), 1.f);
    gr *= coef;
    g.a.grads[t][j] = gr;
  }
  const double step = g.a.step[t][0];
  const double b1 = g.a.beta1, b2 = g.a.beta2, gd = gr;
  const float m = float(b1 * double(g.a.exp_avg[t][j]) + (1.0 - b1) * gd);
  const float vv = float(b2 * double(g.a.exp_avg_sq[t][j]) + (1.0 - b2) * gd * gd);
  g.a.exp_avg[t][j] = m;
  g.a.exp_avg_sq[t][j] = vv;
  const double bc1 = 1.0 - pow(b1, step), bc2 = 1.0 - pow(b2, step);
  const double denom = sqrt(double(vv)) / sqrt(bc2) + g.a.eps;
  g.a.params[t][j] = float(double(g.a.params[t][j]) - (g.a.lr / bc1) * double(m) / denom);
}

int adam_layout(const QuadAdam* a, AdamArgs& g) {
  if (!a || a->count < 1 || a->count > QUAD_ADAM_MAX_TENSORS) return lfail(QUAD_EINVAL, "count out of range");
  g.a = *a;
  g.offs[0] = 0;
  for (int t = 0; t < a->count; t++) {
    if (!a->params[t] || !a->grads[t] || !a->exp_avg[t] || !a->exp_avg_sq[t] || !a->step[t])
      return lfail(QUAD_EINVAL, "a tensor pointer is NULL");
    if (a->numel[t] < 1) return lfail(QUAD_EINVAL, "numel must be >= 1");
    if (int64_t(g.offs[t]) + a->numel[t] > (int64_t(1) << 30)) return lfail(QUAD_EINVAL, "too many elements");
    g.offs[t + 1] = g.offs[t] + a->numel[t];
  }
  for (int t = a->count; t < QUAD_ADAM_MAX_TENSORS; t++) g.offs[t + 1] = g.offs[a->count];
  g.nblocks = (g.offs[a->count] + ADAM_BLOCK - 1) / ADAM_BLOCK;
  return QUAD_OK;
}
}  // namespace
}  // namespace quadenv

using namespace quadenv;
using namespace quadenv::lrn;

extern "C" {

int64_t quad_ppo_workspace_bytes(int32_t batch) {
  if (batch < 1) return 0;
  const Layout l = layout_of(batch, ACTOR_SHARE);  // the partial image is sized for every split
  const Layout lb = layout_both(batch);             // the bf16x3 form's
  return l.adv_bytes + (lb.part_bytes > l.part_bytes ? lb.part_bytes : l.part_bytes) + l.wimg_bytes;
}

// 1: the bf16x3 form (k_ppo_grad_x3, default), 0: the f32-input MFMA form (k_ppo_grad);
// QUADENV_LEARNER=f32 selects the latter (read per call, so a process can A/B both)
int quad_ppo_grad_form(void) {
  const char* v = std::getenv("QUADENV_LEARNER");
  return (v && std::strcmp(v, "f32") == 0) ? 0 : 1;
}

}  // extern "C"

namespace {
// quad_ppo_grad, or (dump != NULL: quad_ppo_hidden) the dump instantiation of the same gradient
// kernel, which also records every minibatch row's hidden pre-activations
int ppo_grad_impl(const QuadPolicyParams* p, const QuadPPOBatch* b, const QuadPolicyGrads* gr, void* workspace,
                  int64_t workspace_bytes, void* stream, float* dump) {
  if (!p || !b || !gr || !workspace) return lfail(QUAD_EINVAL, "NULL argument");
  if (!p->pi_w0 || !p->pi_b0 || !p->pi_w1 || !p->pi_b1 || !p->act_w || !p->act_b || !p->vf_w0 || !p->vf_b0 ||
      !p->vf_w1 || !p->vf_b1 || !p->val_w || !p->val_b || !p->log_std)
    return lfail(QUAD_EINVAL, "a policy parameter pointer is NULL");
  if (!gr->pi_w0 || !gr->pi_b0 || !gr->pi_w1 || !gr->pi_b1 || !gr->act_w || !gr->act_b || !gr->vf_w0 ||
      !gr->vf_b0 || !gr->vf_w1 || !gr->vf_b1 || !gr->val_w || !gr->val_b || !gr->log_std)
    return lfail(QUAD_EINVAL, "a gradient pointer is NULL");
  if (!b->obs || !b->actions || !b->log_prob || !b->advantages || !b->returns || !b->index)
    return lfail(QUAD_EINVAL, "a minibatch buffer is NULL");
  if (b->batch < 1) return lfail(QUAD_EINVAL, "batch must be >= 1");
  if ((reinterpret_cast<uintptr_t>(b->obs) | reinterpret_cast<uintptr_t>(b->actions)) & 15u)
    return lfail(QUAD_EINVAL, "obs and actions must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(workspace) & 15u) return lfail(QUAD_EINVAL, "workspace must be 16-byte aligned");
  if (!(b->clip_range > 0.f)) return lfail(QUAD_EINVAL, "clip_range must be > 0");
  const bool x3 = quad_ppo_grad_form() == 1;
  const Layout l = x3 ? layout_both(b->batch) : layout_of(b->batch, ACTOR_SHARE);
  if (dump && int64_t(b->batch) * 2 * 256 * 4 > (int64_t(1) << 40)) return lfail(QUAD_EINVAL, "batch too large to dump");
  if (workspace_bytes < l.adv_bytes + l.part_bytes + (x3 ? l.wimg_bytes : 0))
    return lfail(QUAD_EINVAL, "workspace too small");
  static bool opted[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return lfail(QUAD_EHIP, "hipGetDevice failed");
  const int lds_bytes = L_TOTAL * int(sizeof(float));
  if (!x3 && !opted[dev]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad), hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_bytes) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_dump), hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_bytes) != hipSuccess)
      return lfail(QUAD_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    opted[dev] = true;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  double* adv_part = static_cast<double*>(workspace);
  float* part = reinterpret_cast<float*>(static_cast<char*>(workspace) + l.adv_bytes);
  const bool norm = b->normalize_advantage && b->batch > 1;
  const bool given = b->normalize_advantage == QUAD_ADV_GIVEN;  // (3: quad_ppo_adv_stats_epoch's slice)
  if (norm && given && !b->adv_sums) return lfail(QUAD_EINVAL, "QUAD_ADV_GIVEN needs adv_sums");
  // (2: quad_ppo_adv_stats ran into the workspace; 3: the sums are given)
  const bool need_stats = norm && b->normalize_advantage != QUAD_ADV_PRECOMPUTED && !given;
  if (norm && given) adv_part = const_cast<double*>(b->adv_sums);
  if (need_stats && !x3) {  // the bf16x3 form computes them in its prep launch
    hipLaunchKernelGGL(k_adv_stats, dim3(ADV_BLOCKS), dim3(256), 0, s, b->advantages, b->index, b->batch, adv_part);
    if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_adv_stats launch failed");
  }
  GArgs g{};
  g.actor = NetW{p->pi_w0, p->pi_b0, p->pi_w1, p->pi_b1, p->act_w, p->act_b};
  g.critic = NetW{p->vf_w0, p->vf_b0, p->vf_w1, p->vf_b1, p->val_w, p->val_b};
  g.log_std = p->log_std;
  g.obs = b->obs; g.act = b->actions; g.logp_old = b->log_prob; g.adv = b->advantages; g.ret = b->returns;
  g.idx = b->index;
  g.adv_part = norm ? adv_part : nullptr;
  g.part = part;
  g.batch = b->batch; g.nb = l.nb; g.per_block = l.per_block; g.nbc = l.nbc; g.per_block_c = l.per_block_c;
  g.clip = b->clip_range; g.inv_batch = 1.0f / float(b->batch); g.vf_coef = b->vf_coef;
  g.dump = dump;
  g.wimg = static_cast<char*>(workspace) + l.adv_bytes + l.part_bytes;
  if (x3) {
    double* st = need_stats ? adv_part : nullptr;
    if (int rc = dump ? launch_ppo_grad_x3_dump(g, s, st, b->advantages) : launch_ppo_grad_x3(g, s, st, b->advantages))
      return rc;
  } else if (dump) {
    hipLaunchKernelGGL(k_ppo_grad_dump, dim3(l.nb + l.nbc), dim3(LB), lds_bytes, s, g);
    if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_ppo_grad_dump launch failed");
  } else {
    hipLaunchKernelGGL(k_ppo_grad, dim3(l.nb + l.nbc), dim3(LB), lds_bytes, s, g);
    if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_ppo_grad launch failed");
  }
  RArgs r{};
  r.gr = *gr; r.part = part; r.log_std = p->log_std; r.stats = b->stats; r.nb = l.nb; r.nbc = l.nbc;
  r.inv_batch = 1.0f / float(b->batch); r.ent_coef = b->ent_coef;
  hipLaunchKernelGGL(k_ppo_reduce, dim3((2 * PSTRIDE + 63) / 64), dim3(256), 0, s, r);
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_ppo_reduce launch failed");
  return QUAD_OK;
}
}  // namespace

extern "C" {

int quad_ppo_grad(const QuadPolicyParams* p, const QuadPPOBatch* b, const QuadPolicyGrads* gr, void* workspace,
                  int64_t workspace_bytes, void* stream) {
  return ppo_grad_impl(p, b, gr, workspace, workspace_bytes, stream, nullptr);
}

int quad_ppo_adv_stats(const QuadPPOBatch* b, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!b || !workspace || !b->advantages || !b->index) return lfail(QUAD_EINVAL, "NULL argument");
  if (b->batch < 1) return lfail(QUAD_EINVAL, "batch must be >= 1");
  const Layout l = layout_of(b->batch, ACTOR_SHARE);
  if (workspace_bytes < l.adv_bytes + l.part_bytes) return lfail(QUAD_EINVAL, "workspace too small");
  if (b->batch > 1)
    hipLaunchKernelGGL(k_adv_stats, dim3(ADV_BLOCKS), dim3(256), 0, static_cast<hipStream_t>(stream), b->advantages,
                       b->index, b->batch, static_cast<double*>(workspace));
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_adv_stats launch failed");
  return QUAD_OK;
}

int quad_ppo_adv_stats_epoch(const float* advantages, const int64_t* perm, int32_t batch, int32_t n_minibatches,
                             double* sums, void* stream) {
  if (!advantages || !perm || !sums) return lfail(QUAD_EINVAL, "NULL argument");
  if (batch < 1 || n_minibatches < 1 || n_minibatches > 65535) return lfail(QUAD_EINVAL, "need batch >= 1, 1 <= n_minibatches <= 65535");
  hipLaunchKernelGGL(k_adv_stats_epoch, dim3(ADV_BLOCKS, n_minibatches), dim3(256), 0, static_cast<hipStream_t>(stream),
                     advantages, perm, batch, sums);
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_adv_stats_epoch launch failed");
  return QUAD_OK;
}

int quad_ppo_hidden(const QuadPolicyParams* p, const QuadPPOBatch* b, const QuadPolicyGrads* gr, float* hidden,
                    void* workspace, int64_t workspace_bytes, void* stream) {
  if (!hidden) return lfail(QUAD_EINVAL, "hidden is NULL");
  return ppo_grad_impl(p, b, gr, workspace, workspace_bytes, stream, hidden);
}

int quad_permutation(int64_t n, uint64_t seed, int64_t* out, void* stream) {
  if (n < 1 || n > (int64_t(1) << 40) || !out) return lfail(QUAD_EINVAL, "need 1 <= n <= 2^40 and an output");
  int bits = 2;
  while ((int64_t(1) << bits) < n) bits += 2;  // even: a balanced Feistel on 2^bits codes, 2^bits < 4n
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_permutation, dim3(unsigned(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, bits / 2, seed, out);
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_permutation launch failed");
  return QUAD_OK;
}

int64_t quad_adam_workspace_bytes(const QuadAdam* a) {
  AdamArgs g{};
  if (adam_layout(a, g) != QUAD_OK) return 0;
  return int64_t(g.nblocks) * int64_t(sizeof(float));
}

int quad_clip_adam(const QuadAdam* a, void* workspace, int64_t workspace_bytes, void* stream) {
  AdamArgs g{};
  if (int rc = adam_layout(a, g)) return rc;
  if (!workspace || workspace_bytes < int64_t(g.nblocks) * int64_t(sizeof(float)))
    return lfail(QUAD_EINVAL, "workspace too small");
  if (!(a->eps > 0.0) || !(a->lr >= 0.0) || !(a->beta1 >= 0.0 && a->beta1 < 1.0) || !(a->beta2 >= 0.0 && a->beta2 < 1.0))
    return lfail(QUAD_EINVAL, "need lr >= 0, eps > 0, 0 <= betas < 1");
  g.part = static_cast<float*>(workspace);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_grad_sumsq, dim3(g.nblocks), dim3(ADAM_BLOCK), 0, s, g);
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_grad_sumsq launch failed");
  hipLaunchKernelGGL(k_adam, dim3(g.nblocks), dim3(ADAM_BLOCK), 0, s, g);
  if (hipGetLastError() != hipSuccess) return lfail(QUAD_EHIP, "k_adam launch failed");
  return QUAD_OK;
}

}  // extern "C"
