// policy_net.h -- the rollout policy's MLP on MFMA (device only), shared by the policy kernel
// (policy.hip) and the fused rollout kernel (rollout.hip). See policy.hip for the layout trick.
//
// Arithmetic: bf16 MFMA (v_mfma_f32_32x32x16_bf16) over three-piece splits of every f32 operand,
// the learner's scheme (learner_x3.hip): x = x0 + x1 + x2, each piece the round-to-nearest bf16 of
// what the previous pieces leave (exact), and a product a*b as the six MFMAs a2b0 + a1b1 + a0b2 +
// a1b0 + a0b1 + a0b0 accumulated in f32; the dropped a1b2 + a2b1 + a2b2 are <= ~2^-23 |ab|. One
// 16-deep k-step costs 6 x 32 matrix cycles instead of 8 x 64 with v_mfma_f32_32x32x2_f32 (2.7x
// less). The activations (X^T, relu(h1)^T) are split once per layer. W2 is pre-split once per
// policy update (k_policy_pack appends the pieces to the packed image, 96 KB per net) and read from
// L2 two k-steps ahead; W1, biases and head weights are staged in LDS as f32 (21 KB; W1 split at
// use). Until round 3 the f32 W2 sat in LDS too (both nets' three-piece W2 would be 192 KB against
// 160) and was split at every step: ~45 VALU per k-step against 12 MFMAs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "quad_physics.h"

namespace quadenv {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int H = 128, OBS = 12, ACT = 4;
constexpr int TILE = 32;     // envs per MFMA tile (one wave holds one tile at a time)
constexpr int PBLOCK = 256;  // 4 waves (k_rollout_post; k_policy_act takes BLK)

// packed net image (floats); NOUT = 4 (actor) or 1 (critic). Operand element j of lane l (r = l & 31,
// h = l >> 5) is k = 8h + j of the 32x32x16 MFMA (cdna_hip_programming.md, bf16 lane maps):
//   W1: [4 n][64 lane][8]               A[neuron 32n + r][feature 8h + j] (features 12..15 zero)
//   W2: [4 m][4 n][2 t][64 lane][8]     A[neuron 32m + r][input 32n + acc_row(8t + j, h)]: k-step
//                                       (n, t) consumes registers 8t .. 8t + 7 of relu(h1) block n
//   B1, B2: [4 tile][2 half][16 reg]    biases in accumulator order
//   W3 actor:  [4 m][16 reg][2 half][4 out]   head weights in accumulator order
//   W3 critic: [4 m][4 rq][2 half][4 r]       (reg = 4 rq + r)
//   B3: [4]
constexpr int W1_F = 4 * 64 * 8, W2_F = 4 * 4 * 2 * 64 * 8, B_F = 4 * 2 * 16;
constexpr int NET_W1 = 0, NET_W2 = NET_W1 + W1_F, NET_B1 = NET_W2 + W2_F, NET_B2 = NET_B1 + B_F;
constexpr int NET_W3 = NET_B2 + B_F;
constexpr int ACTOR_F = NET_W3 + ACT * 128 + 4;
constexpr int CRITIC_F = NET_W3 + 128 + 4;
constexpr int LDS_F = ACTOR_F + CRITIC_F;  // 38,024 floats = 152 KB
constexpr int PACKED_F = LDS_F + 4;        // + log_std[4]
static_assert(ACTOR_F % 4 == 0 && LDS_F % 4 == 0, "float4 staging");
// then the W2 fragments pre-split into three bf16 pieces (k_policy_pack), read from HBM / L2 by
// the MLP pipeline instead of splitting the f32 fragments from LDS at every step:
// [net][k-step g 0..31][piece 0..2][lane 0..63] x 16 bytes = 96 KB per net
constexpr int PIECES_F = 2 * 32 * 3 * 64 * 4;
// then W1 the same way: [net][block n 0..3][piece][lane] x 16 bytes = 12 KB per net
constexpr int W1PIECES_F = 2 * 4 * 3 * 64 * 4;
constexpr int PACKED_ALL_F = PACKED_F + PIECES_F + W1PIECES_F;
static_assert(PACKED_F % 4 == 0, "16-byte aligned pieces");

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
// (o3 = NET_W3 + 4h: the lane's part of the head-weight region)
// The actor head's four FMAs per hidden value as two v_pk_fma_f32 (each lane of a packed FMA is the
// same fused multiply-add, so the same bits as four v_fma_f32, tools/env_digest.py). Round 4 A/B
// (k_rollout, 65,536 envs): 27.63 / 27.74 vs 27.73 / 27.93 us per step for the four plain FMAs
template <int NOUT, int NT>
__device__ __forceinline__ void head_part(const float* __restrict__ L, const f32x16 (&x)[NT], int m, int i,
                                          int o3, float (&part)[NT][NOUT]) {
  if constexpr (NOUT == ACT) {
    const float4 w = ld4(L, o3 + (m * 16 + i) * 8);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const float v = relu(x[j][i]);
      const f32x2 vv = {v, v}, w01 = {w.x, w.y}, w23 = {w.z, w.w};
      f32x2 p01 = {part[j][0], part[j][1]}, p23 = {part[j][2], part[j][3]};
      p01 = __builtin_elementwise_fma(w01, vv, p01);
      p23 = __builtin_elementwise_fma(w23, vv, p23);
      part[j][0] = p01[0]; part[j][1] = p01[1]; part[j][2] = p23[0]; part[j][3] = p23[1];
    }
  } else {
    if (i % 4 != 0) return;
    const float4 w = ld4(L, o3 + (m * 4 + i / 4) * 8);
#pragma unroll
    for (int j = 0; j < NT; j++) {
      part[j][0] = fmaf(w.x, relu(x[j][i + 0]), part[j][0]);
      part[j][0] = fmaf(w.y, relu(x[j][i + 1]), part[j][0]);
      part[j][0] = fmaf(w.z, relu(x[j][i + 2]), part[j][0]);
      part[j][0] = fmaf(w.w, relu(x[j][i + 3]), part[j][0]);
    }
  }
}

// ---- three-piece operands
struct P3 {
  bf16x8 p[3];  // x = p[0] + p[1] + p[2]
};
__device__ __forceinline__ P3 split8(const float (&v)[8]) {
  u32x4 q0, q1, q2;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const f32x2 x = {v[2 * k], v[2 * k + 1]};
    const bf16x2 p0 = __builtin_convertvector(x, bf16x2);
    const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
    const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
    const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
    const bf16x2 p2 = __builtin_convertvector(r2, bf16x2);
    q0[k] = __builtin_bit_cast(uint32_t, p0);
    q1[k] = __builtin_bit_cast(uint32_t, p1);
    q2[k] = __builtin_bit_cast(uint32_t, p2);
  }
  P3 o;
  o.p[0] = __builtin_bit_cast(bf16x8, q0);
  o.p[1] = __builtin_bit_cast(bf16x8, q1);
  o.p[2] = __builtin_bit_cast(bf16x8, q2);
  return o;
}
// acc += a * b, small terms first
__device__ __forceinline__ f32x16 mfma6(const P3& a, const P3& b, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}
__device__ __forceinline__ P3 ld_split8(const float* L, int off) {
  const float4 a = ld4(L, off), b = ld4(L, off + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return split8(v);
}

// ---- the MLP forward for NT 32-env tiles at once (all 64 lanes). Input fragments:
// xq[j][k] = x[env = lane&31 of tile j][feature 8 (lane>>5) + k] (zero past feature 11). Outputs: the
// NOUT head outputs of env lane&31 of every tile (both lane halves get them). The NT tiles share
// every weight split, and their MFMA chains interleave.
// Order: per input block n, layer 1 makes relu(h1) block n as pieces, and its two k-steps go into
// all four layer-2 output blocks (m) at once, so only two blocks of pieces are ever live (all four
// would be 192 VGPRs at NT = 2); the layer-2 accumulators (128 registers) sit in AGPRs. Software
// pipeline over the 32 layer-2 k-steps g = 8n + s (s = 4t + m): the W2 fragment of step g + 2 is
// read from LDS and the one of g + 1 split while step g's 6 x NT MFMAs issue; during block n,
// layer 1 of the NEXT block runs too (its W1 split at s = 0, its MFMAs at s = 1, its ReLU + split in
// 16 pair-chunks over s = 2..7), so the matrix pipe never waits for a layer-1 result. When the
// actor is followed by the critic (net_forward2), the critic's block 0 and first W2 fragments are
// that next block: the pipeline runs through both nets. Each step is one scheduling region (fence)
// with its VALU interleaved between the MFMAs.

// per-net LDS offsets of this lane (floats), opaque to the compiler: every read is one of these
// plus an immediate (< 64 KB). Left to itself it hoists one address register per distinct offset out
// of the callers' step loops (the critic's image starts 76 KB into the LDS) -- ~100 of them, spilled.
// VALU per MFMA in each step's interleave (measured on tools/diag/net_bench.hip builds; the
// scheduler's own order without the group barriers was slower)
constexpr int NF_VPG = 5;
typedef __attribute__((address_space(1))) const bf16x8 gbf16x8;  // global loads, not flat
struct NetOff {
  int w1, w2, b, w3;
  gbf16x8* wp;   // this net's pre-split W2 pieces, this lane's unit
  gbf16x8* w1p;  // and W1's
  int lpa, lpb;  // LDS byte offsets of this lane's unit of the actor's W2 pieces (stage_pieces)
};
// The actor's pre-split W2 pieces in LDS (k_rollout: staged once per launch, read by ds_read_b128
// instead of three global loads per k-step): the f32 W2 regions of the image are not staged since
// round 3, so the 96 KB go into the actor's (k-steps 0 .. LP_SPLIT - 1, 3 KB each) and the
// critic's (the rest). The critic's pieces stay in L2 (both nets' would be 192 KB).
constexpr int LP_SPLIT = 21;
constexpr int LP_A = NET_W2 * 4, LP_B = (ACTOR_F + NET_W2) * 4;
static_assert(LP_SPLIT * 3072 <= W2_F * 4 && (32 - LP_SPLIT) * 3072 <= W2_F * 4, "pieces fit the W2 regions");
static_assert(LP_A % 16 == 0 && LP_B % 16 == 0, "16-byte aligned LDS pieces");
// `packed`: the global packed image; its scalar base is made opaque per call, so the compiler
// cannot hoist the pieces' loads out of the callers' step loops (hundreds of VGPRs)
__device__ __forceinline__ NetOff net_off(int base, const float* packed, int net) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  uint64_t pb = reinterpret_cast<uint64_t>(packed + PACKED_F);
  asm volatile("" : "+s"(pb));
  NetOff o{base + NET_W1 + lane * 8, base + NET_W2 + lane * 8, base + NET_B1 + h * 16, base + NET_W3 + h * 4,
           reinterpret_cast<gbf16x8*>(pb) + net * (32 * 3 * 64) + lane,
           reinterpret_cast<gbf16x8*>(pb) + 2 * (32 * 3 * 64) + net * (4 * 3 * 64) + lane,
           LP_A + lane * 16, LP_B + lane * 16};
  asm volatile("" : "+v"(o.w1), "+v"(o.w2), "+v"(o.b), "+v"(o.w3), "+v"(o.lpa), "+v"(o.lpb));
  return o;
}
// the pre-split W1 fragment of layer-1 block n (k_policy_pack; the same pieces as ld_split8 of the
// LDS f32, which the four waves of a block would each redo per step)
__device__ __forceinline__ P3 w1_pieces(const NetOff& o, int n) {
  P3 x;
#pragma unroll
  for (int p = 0; p < 3; p++) x.p[p] = o.w1p[(n * 3 + p) * 64];
  return x;
}
// the pre-split W2 fragment of layer-2 k-step g (three dwordx4 loads; LP: three ds_read_b128 of
// the actor's pieces staged in LDS)
template <bool LP = false>
__device__ __forceinline__ P3 w2_pieces(const float* L, const NetOff& o, int g) {
  P3 x;
  if constexpr (LP) {
    const char* Lc = reinterpret_cast<const char*>(L);
#pragma unroll
    for (int p = 0; p < 3; p++)
      x.p[p] = *reinterpret_cast<const bf16x8*>(Lc + (g < LP_SPLIT ? o.lpa + (g * 3 + p) * 1024
                                                                   : o.lpb + ((g - LP_SPLIT) * 3 + p) * 1024));
  } else {
#pragma unroll
    for (int p = 0; p < 3; p++) x.p[p] = o.wp[(g * 3 + p) * 64];
  }
  return x;
}
// W2 fragment of layer-2 k-step g = 8n + 4t + m
__device__ __forceinline__ int w2_frag(const NetOff& o, int g) {
  return o.w2 + (((g & 3) * 4 + (g >> 3)) * 2 + ((g >> 2) & 1)) * 512;
}

struct Q3 {  // three pieces as raw 32-bit words (filled a pair at a time)
  u32x4 q[3];
  __device__ __forceinline__ P3 p() const {
    P3 o;
#pragma unroll
    for (int k = 0; k < 3; k++) o.p[k] = __builtin_bit_cast(bf16x8, q[k]);
    return o;
  }
};
// pieces of the pair (x0, x1) into word `k` of each piece (one quarter of split8)
__device__ __forceinline__ void split_pair(float x0, float x1, Q3& o, int k) {
  const f32x2 x = {x0, x1};
  const bf16x2 p0 = __builtin_convertvector(x, bf16x2);
  const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
  const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
  const bf16x2 p2 = __builtin_convertvector(r2, bf16x2);
  o.q[0][k] = __builtin_bit_cast(uint32_t, p0);
  o.q[1][k] = __builtin_bit_cast(uint32_t, p1);
  o.q[2][k] = __builtin_bit_cast(uint32_t, p2);
}

template <int NT>
struct Pipe {
  Q3 h1[2][NT][2];   // relu(h1) pieces: block n in buffer n & 1 (block 0 of the next net: buffer 0)
  P3 wr[3];          // pre-split W2 fragments: ring over the global step count (net 32 + g) % 3,
                     // step g's loaded two steps ahead
};

// block 0 of a net before its pipeline starts (the first net of a call)
template <int NT, bool LP = false>
__device__ __forceinline__ void pipe_start(const float* __restrict__ L, const NetOff& o, const P3 (&xp)[NT],
                                           Pipe<NT>& st) {
  f32x16 b;
  bias_init(b, L, o.b);
  const P3 w1 = w1_pieces(o, 0);
#pragma unroll
  for (int j = 0; j < NT; j++) {
    const f32x16 a1 = mfma6(w1, xp[j], b);
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int k = 0; k < 4; k++)
        split_pair(relu(a1[8 * t + 2 * k]), relu(a1[8 * t + 2 * k + 1]), st.h1[0][j][t], k);
  }
  st.wr[0] = w2_pieces<LP>(L, o, 0);
  st.wr[1] = w2_pieces<LP>(L, o, 1);
  __builtin_amdgcn_sched_barrier(0);
}

// a caller's work for the issue gaps of layer-2 step g (none by default): called inside step g's
// scheduling region, so its VALU interleaves with that step's MFMAs (the fused rollout hangs the env
// step on the critic's steps, rollout.hip)
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
};

// one net's 32 layer-2 steps (+ layer 1 of its blocks 1..3, and with NEXT the next net's block 0
// and first fragments), then its head
// (LP: this net's W2 pieces come from LDS -- the actor in k_rollout; the next net's always from L2)
template <int NOUT, int NT, bool NEXT, int G0, bool LP = false, typename Hook = NoHook>
__device__ __forceinline__ void net_core(const float* __restrict__ L, const NetOff& o, const NetOff& on,
                                         const P3 (&xp)[NT], Pipe<NT>& st, float (&out)[NT][NOUT],
                                         Hook&& hook = Hook{}) {
  const int h = (threadIdx.x >> 5) & 1;
  f32x16 acc[4][NT];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    bias_init(acc[m][0], L, o.b + B_F + m * 32);
#pragma unroll
    for (int j = 1; j < NT; j++) acc[m][j] = acc[m][0];
  }
#pragma unroll
  for (int n = 0; n < 4; n++) {
    const int cb = n & 1, nb = cb ^ 1;
    const bool pre = n < 3 || NEXT;          // layer 1 of the next block during this one
    const NetOff& ol = n < 3 ? o : on;       // whose next block
    const int nn = n < 3 ? n + 1 : 0;
    P3 w1n;
    f32x16 b1n, a1n[NT];
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const int g = 8 * n + s, t = s >> 2, m = s & 3;
      if (g + 2 < 32 || NEXT)  // step g + 2's pieces into the ring slot step g - 1 freed
        st.wr[(G0 + g + 2) % 3] = g + 2 < 32 ? w2_pieces<LP>(L, o, g + 2) : w2_pieces(L, on, g + 2 - 32);
#pragma unroll
      for (int j = 0; j < NT; j++) acc[m][j] = mfma6(st.wr[(G0 + g) % 3], st.h1[cb][j][t].p(), acc[m][j]);
      if (pre && s == 1) {
#pragma unroll
        for (int j = 0; j < NT; j++) a1n[j] = mfma6(w1n, xp[j], b1n);
      }
      if (pre && s == 0) {
        bias_init(b1n, L, ol.b + nn * 32);
        w1n = w1_pieces(ol, nn);
      }
      if (pre && s >= 2) {  // pair-chunks c = 0..15 (tile c >> 3, half (c >> 2) & 1, pair c & 3) over s = 2..7
#pragma unroll
        for (int c = 0; c < 16; c++) {
          if (2 + (c * 6) / 16 != s || (c >> 3) >= NT) continue;
          const int j = c >> 3, tt = (c >> 2) & 1, k = c & 3;
          split_pair(relu(a1n[j][8 * tt + 2 * k]), relu(a1n[j][8 * tt + 2 * k + 1]), st.h1[nb][j][tt], k);
        }
      }
      hook(g);
#pragma unroll
      for (int q = 0; q < 6 * NT; q++) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NF_VPG, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float part[NT][NOUT];
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int q = 0; q < NOUT; q++) part[j][q] = 0.f;
#pragma unroll
  for (int m = 0; m < 4; m++) {
#pragma unroll
    for (int i = 0; i < 16; i++) head_part<NOUT, NT>(L, acc[m], m, i, o.w3, part);
    __builtin_amdgcn_sched_barrier(0);  // one block's accumulators in VGPRs at a time
  }
  // lanes l and l ^ 32 hold the two halves of the same env's neurons; both lanes form the same sum
  // (lower half + upper half: v_permlane32_swap of the partial with itself gives the lower half's
  // value in every lane as the first result, the upper half's as the second -- a VALU swap, not an
  // LDS permute)
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int q = 0; q < NOUT; q++) {
      const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(part[j][q]), __float_as_uint(part[j][q]), false, false);
      out[j][q] = (__uint_as_float(p[0]) + __uint_as_float(p[1])) + L[o.w3 - 4 * h + NOUT * 128 + q];
    }
}

// one net (image at L): NOUT = ACT for the actor, 1 for the critic
template <int NOUT, int NT>
__device__ __forceinline__ void net_forward(const float* __restrict__ L, const float* packed, const float (&xq)[NT][8],
                                            float (&out)[NT][NOUT]) {
  P3 xp[NT];
#pragma unroll
  for (int j = 0; j < NT; j++) xp[j] = split8(xq[j]);
  const NetOff o = net_off(0, packed, NOUT == ACT ? 0 : 1);
  Pipe<NT> st;
  pipe_start<NT>(L, o, xp, st);
  net_core<NOUT, NT, false, 0>(L, o, o, xp, st, out);
}

// actor (image at L) then critic (at L + ACTOR_F) in one pipeline: the same bits as two net_forward
// calls (every tile's operations and their order are the same)
// (ALP: the actor's W2 pieces from LDS, staged by stage_pieces)
template <int NT, bool ALP = false>
__device__ __forceinline__ void net_forward2(const float* __restrict__ L, const float* packed, const float (&xq)[NT][8],
                                             float (&mean)[NT][ACT], float (&val)[NT][1]) {
  P3 xp[NT];
#pragma unroll
  for (int j = 0; j < NT; j++) xp[j] = split8(xq[j]);
  const NetOff oa = net_off(0, packed, 0), oc = net_off(ACTOR_F, packed, 1);
  Pipe<NT> st;
  pipe_start<NT, ALP>(L, oa, xp, st);
  net_core<ACT, NT, true, 0, ALP>(L, oa, oc, xp, st, mean);
  net_core<1, NT, false, 32>(L, oc, oc, xp, st, val);
}

// the packed image global -> LDS per block, without the two f32 W2 regions (the MLP reads the
// pre-split pieces from L2 instead): 21 KB of the 152 KB image, in batches of float4 loads in flight
// per thread (a serial load -> store loop would pay a round trip of L2/MALL latency per float4).
// Compact float4 index k -> image float4 index: [0, NET_W2) | [NET_B1, ACTOR_F + NET_W2) |
// [ACTOR_F + NET_B1, LDS_F)
constexpr int STAGE_V = (LDS_F - 2 * W2_F) / 4;
__device__ __forceinline__ int stage_map(int k) {
  constexpr int A = NET_W2 / 4, B = (ACTOR_F + NET_W2 - NET_B1) / 4 + A;
  return k < A ? k : (k < B ? k + W2_F / 4 : k + W2_F / 2);
}
template <int BLK>
__device__ __forceinline__ void stage_lds(float* lds, const float* __restrict__ packed) {
  constexpr int NV = STAGE_V, PER = (NV + BLK - 1) / BLK, BATCH = PER < 8 ? PER : 8;
  const float4* src = reinterpret_cast<const float4*>(packed);
  float4* dst = reinterpret_cast<float4*>(lds);
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += BATCH) {
    float4 v[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; j++) {
      const int k = (b0 + j) * BLK + threadIdx.x;
      v[j] = src[stage_map(k < NV ? k : NV - 1)];  // clamped: every element defined, stays in VGPRs
    }
#pragma unroll
    for (int j = 0; j < BATCH; j++) {
      const int k = (b0 + j) * BLK + threadIdx.x;
      if (b0 + j < PER && k < NV) dst[stage_map(k)] = v[j];
    }
  }
  __syncthreads();
}

// the actor's 96 KB of pre-split W2 pieces (global [k-step][piece][lane] units of 16 bytes, right
// after the packed image) into the LDS regions LP_A / LP_B (see LP_SPLIT); ends with a barrier
template <int BLK>
__device__ __forceinline__ void stage_pieces(float* lds, const float* __restrict__ packed) {
  constexpr int NV = 32 * 3 * 64, PER = NV / BLK, BATCH = PER % 8 == 0 ? 8 : 4;
  static_assert(NV % BLK == 0 && PER % BATCH == 0, "whole batches");
  const float4* src = reinterpret_cast<const float4*>(packed + PACKED_F);
  char* Lc = reinterpret_cast<char*>(lds);
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += BATCH) {
    float4 v[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; j++) v[j] = src[(b0 + j) * BLK + threadIdx.x];
#pragma unroll
    for (int j = 0; j < BATCH; j++) {
      const int u = (b0 + j) * BLK + int(threadIdx.x), g = u / 192;  // unit (g, p, lane) = (g * 3 + p) * 64 + lane
      const int off = g < LP_SPLIT ? LP_A + u * 16 : LP_B + (u - LP_SPLIT * 192) * 16;
      *reinterpret_cast<float4*>(Lc + off) = v[j];
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
