// policy_net.h -- the rollout policy's MLP on MFMA (device only), shared by the policy kernel
// (policy.hip) and the fused rollout kernel (rollout.hip). See policy.hip for the layout trick.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "quad_physics.h"

namespace quadenv {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int H = 128, OBS = 12, ACT = 4;
constexpr int TILE = 32;     // envs per MFMA tile (one wave holds one tile at a time)
constexpr int PBLOCK = 256;  // 4 waves (k_rollout_post; k_policy_act takes BLK)

// packed net image (floats); NOUT = 4 (actor) or 1 (critic):
//   W1: [4 n][64 lane][8]              layer-1 A fragments, k-steps s = 0..5 (6, 7 zero)
//   W2: [4 m][4 n][4 q][64 lane][4 r]   layer-2 A fragments, k-step 4q + r of input tile n
//   B1, B2: [4 tile][2 half][16 reg]    biases in accumulator order
//   W3 actor:  [4 m][16 reg][2 half][4 out]   head weights in accumulator order
//   W3 critic: [4 m][4 rq][2 half][4 r]       (reg = 4 rq + r)
//   B3: [4]
constexpr int W1_F = 4 * 64 * 8, W2_F = 4 * 4 * 4 * 64 * 4, B_F = 4 * 2 * 16;
constexpr int NET_W1 = 0, NET_W2 = NET_W1 + W1_F, NET_B1 = NET_W2 + W2_F, NET_B2 = NET_B1 + B_F;
constexpr int NET_W3 = NET_B2 + B_F;
constexpr int ACTOR_F = NET_W3 + ACT * 128 + 4;
constexpr int CRITIC_F = NET_W3 + 128 + 4;
constexpr int LDS_F = ACTOR_F + CRITIC_F;  // 38,024 floats = 152 KB
constexpr int PACKED_F = LDS_F + 4;        // + log_std[4]
static_assert(ACTOR_F % 4 == 0 && LDS_F % 4 == 0, "float4 staging");

__host__ __device__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ReLU as one integer max on the bits: a float with the sign bit set is a negative int32 (-0 -> +0,
// negatives -> +0), a non-negative float keeps its bits. A float max with 0 compiles to two
// v_max_f32 on gfx950 (first a canonicalizing max of x with itself: accumulator values are not known
// to be canonical); the results are the same for every non-NaN x.
__device__ __forceinline__ float relu(float x) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

__device__ __forceinline__ float4 ld4(const float* L, int off) {
  return *reinterpret_cast<const float4*>(L + off);
}

__device__ __forceinline__ void bias_init(f32x16& acc, const float* L, int off) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const float4 b = ld4(L, off + 4 * j);
    acc[4 * j] = b.x; acc[4 * j + 1] = b.y; acc[4 * j + 2] = b.z; acc[4 * j + 3] = b.w;
  }
}

// 1/16 of one 32-neuron block's head: ReLU of accumulator register(s) `i` (actor: register i; critic:
// registers 4(i/4).. handled at i % 4 == 0) times the packed head weights, into part[][].
template <int NOUT, int NT>
__device__ __forceinline__ void head_part(const float* __restrict__ L, const f32x16 (&x)[NT], int m, int i,
                                          int h, float (&part)[NT][NOUT]) {
  if constexpr (NOUT == ACT) {
    const float4 w = ld4(L, NET_W3 + ((m * 16 + i) * 2 + h) * 4);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const float v = relu(x[j][i]);
      part[j][0] = fmaf(w.x, v, part[j][0]);
      part[j][1] = fmaf(w.y, v, part[j][1]);
      part[j][2] = fmaf(w.z, v, part[j][2]);
      part[j][3] = fmaf(w.w, v, part[j][3]);
    }
  } else {
    if (i % 4 != 0) return;
    const float4 w = ld4(L, NET_W3 + ((m * 4 + i / 4) * 2 + h) * 4);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      part[j][0] = fmaf(w.x, relu(x[j][i + 0]), part[j][0]);
      part[j][0] = fmaf(w.y, relu(x[j][i + 1]), part[j][0]);
      part[j][0] = fmaf(w.z, relu(x[j][i + 2]), part[j][0]);
      part[j][0] = fmaf(w.w, relu(x[j][i + 3]), part[j][0]);
    }
  }
}

// ---- one net's forward for NT 32-env tiles at once (all 64 lanes). X^T fragments:
// xb[j][s] = x[env = lane&31 of tile j][2 s + (lane>>5)]. Returns the NOUT head outputs of env
// lane&31 of every tile (both lane halves get them). The NT tiles share every LDS weight fragment,
// and their MFMA chains interleave, so consecutive MFMAs are independent.
template <int NOUT, int NT>
__device__ __forceinline__ void net_forward(const float* __restrict__ L, const float (&xb)[NT][6],
                                            float (&out)[NT][NOUT]) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  f32x16 h1[NT][4];
#pragma unroll
  for (int n = 0; n < 4; n++) {
    f32x16 b;
    bias_init(b, L, NET_B1 + (n * 2 + h) * 16);
    const float4 wa = ld4(L, NET_W1 + (n * 64 + lane) * 8), wb = ld4(L, NET_W1 + (n * 64 + lane) * 8 + 4);
    const float w[6] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y};
    f32x16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = b;
#pragma unroll
    for (int s = 0; s < 6; s++)
#pragma unroll
      for (int j = 0; j < NT; j++) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[s], xb[j][s], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NT; j++) {
#pragma unroll
      for (int r = 0; r < 16; r++) acc[j][r] = relu(acc[j][r]);
      h1[j][n] = acc[j];
    }
  }
  float part[NT][NOUT];
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int o = 0; o < NOUT; o++) part[j][o] = 0.f;
  // Layer 2 in four 32-neuron blocks m. The VALU head of block m-1 is issued inside block m's MFMA
  // chain (independent work), so it runs in the matrix pipe's shadow instead of after it.
  f32x16 prev[NT];  // block m-1 (zeros before block 0: its head then adds exact zeros)
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int r = 0; r < 16; r++) prev[j][r] = 0.f;
#pragma unroll 1
  for (int m = 0; m < 4; m++) {
    f32x16 acc[NT];
    bias_init(acc[0], L, NET_B2 + (m * 2 + h) * 16);
#pragma unroll
    for (int j = 1; j < NT; j++) acc[j] = acc[0];
    // A fragments double-buffered: fragment i+1 is in flight while the MFMAs of fragment i issue
    // (one register quad would make each ds_read wait for the last MFMA that reads it)
    const int wbase = NET_W2 + (m * 16 * 64 + lane) * 4;
    float4 a4 = ld4(L, wbase);
#pragma unroll
    for (int i = 0; i < 16; i++) {  // i = 4 n + q
      const int n = i / 4, q = i % 4;
      float4 nx;
      if (i < 15) nx = ld4(L, wbase + (i + 1) * 64 * 4);
      const float w[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < NT; j++)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[k], h1[j][n][4 * q + k], acc[j], 0, 0, 0);
      head_part<NOUT, NT>(L, prev, m > 0 ? m - 1 : 0, i, h, part);  // 1/16 of block m-1's head
      if (i < 15) a4 = nx;
    }
#pragma unroll
    for (int j = 0; j < NT; j++) prev[j] = acc[j];
  }
#pragma unroll
  for (int i = 0; i < 16; i++) head_part<NOUT, NT>(L, prev, 3, i, h, part);
  // lanes l and l ^ 32 hold the two halves of the same env's neurons; both lanes form the same sum
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int o = 0; o < NOUT; o++) {
      const float other = __shfl_xor(part[j][o], 32);
      out[j][o] = ((h ? other : part[j][o]) + (h ? part[j][o] : other)) + L[NET_W3 + NOUT * 128 + o];
    }
}

// 152 KB global -> LDS per block: batches of 13 float4 loads in flight per thread (a serial
// load -> store loop would pay ~38 round trips of L2/MALL latency)
template <int BLK>
__device__ __forceinline__ void stage_lds(float* lds, const float* __restrict__ packed) {
  constexpr int NV = LDS_F / 4, PER = (NV + BLK - 1) / BLK, BATCH = BLK >= 512 ? 10 : 13;
  const float4* src = reinterpret_cast<const float4*>(packed);
  float4* dst = reinterpret_cast<float4*>(lds);
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += BATCH) {
    float4 v[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; j++) {
      const int k = (b0 + j) * BLK + threadIdx.x;
      v[j] = src[k < NV ? k : NV - 1];  // clamped: every element defined, stays in VGPRs
    }
#pragma unroll
    for (int j = 0; j < BATCH; j++) {
      const int k = (b0 + j) * BLK + threadIdx.x;
      if (b0 + j < PER && k < NV) dst[k] = v[j];
    }
  }
  __syncthreads();
}

// Box-Muller on Philox(seed; env, step, 0x200) -> 4 standard normals
__device__ __forceinline__ void gauss4(uint64_t seed, uint64_t env, uint32_t step, float z[4]) {
  uint32_t c[4] = {uint32_t(env), uint32_t(env >> 32), step, 0x200u};
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const float u1 = (float(c[2 * k] >> 8) + 1.0f) * 0x1p-24f;  // (0, 1]
    const float u2 = float(c[2 * k + 1] >> 8) * 0x1p-24f;
    // hardware log2 / sqrt / sin / cos (sin and cos take revolutions: u2 in [0, 1) is the angle
    // 2 pi u2 directly) instead of the libm sequences (~130 VALU for the four normals); within
    // the 1e-5 (1 + |a|) bar of the float64 Box-Muller (tests/test_gpu_policy.py)
    const float r = __builtin_amdgcn_sqrtf(-1.38629436111989061f * __builtin_amdgcn_logf(u1));  // -2 ln u1
    z[2 * k] = r * __builtin_amdgcn_cosf(u2);
    z[2 * k + 1] = r * __builtin_amdgcn_sinf(u2);
  }
}

}  // namespace quadenv
