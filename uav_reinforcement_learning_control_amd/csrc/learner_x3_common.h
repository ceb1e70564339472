// learner_x3_common.h -- the bf16x3 arithmetic of the PPO minibatch gradient (learner_x3.hip,
// k_ppo_grad_x3), kept apart from the kernel so A/B forms of it (round 5: a 32-row-round, two-
// blocks-per-CU cut) build on the same pieces: the three-piece splits, the split
// products on v_mfma_f32_32x32x16_bf16, the LDS image addressing and reads, the pre-split W2 image.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "learner.h"

namespace quadenv {
namespace lrn {

// k_x3_prep (learner_x3.hip): the W2 split (+ the advantage statistics when adv_stats != NULL)
int launch_prep(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv);

namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

struct X3 {
  bf16x8 p[3];  // x = p[0] + p[1] + p[2]
};
struct X3h {
  bf16x4 p[3];
};

constexpr int RS = 272;  // row stride (bytes) of the bf16 [row][128 neuron] images: 256 + 16

// byte offset of 16-byte chunk `ch` of image row `row`. Padded rows (68 dwords) instead of an XOR
// swizzle: every address is affine in the k-step / tile / block indices, so each read takes one
// base register and an immediate offset (the XOR form held ~100 hoisted address VGPRs, and spilled);
// the 16-byte row reads are conflict-free, and so are dW2's transposed reads (rows 4 apart, see
// trblk); the relu'(h1) reads (4 consecutive rows: the accumulator's row order) are 4-way.
// round barriers (QD_X3_NOBAR: cost-ablation builds only -- wrong results)
#if defined(QD_X3_NOBAR)
#define X3_BAR() ((void)0)
#else
#define X3_BAR() __syncthreads()
#endif

// scheduling fence between k-steps (bounds how far the compiler hoists operand reads)
#if defined(QD_X3_NOSB)
#define X3_SB() ((void)0)
#else
#define X3_SB() __builtin_amdgcn_sched_barrier(0)
#endif

// The next k-step's operand reads interleaved with the first MFMAs of this one (scheduling groups
// of the region between two X3_SB fences: `n_rd` LDS reads, `n_mfma` MFMAs). Left to itself the
// scheduler sinks the reads behind all but the last MFMA (their registers are the ones the current
// MFMAs read), so each k-step waited out the LDS latency: 1.5 % of the kernel (QD_X3_NOPIPE:
// A/B builds only)
#if !defined(QD_X3_NOPIPE)
#define X3_PIPE(n_rd, n_mfma)                                                   \
  do {                                                                          \
    for (int i_ = 0; i_ < (n_rd) / 2; i_++) {                                   \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                        \
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                        \
    }                                                                           \
    __builtin_amdgcn_sched_group_barrier(0x008, (n_mfma) - (n_rd) / 2, 0);      \
  } while (0)
#else
#define X3_PIPE(n_rd, n_mfma) ((void)0)
#endif
// the same with `n_vm` global loads (the pre-split weight pieces two k-steps ahead) issued first
#if !defined(QD_X3_NOPIPE)
#define X3_PIPE_V(n_vm, n_rd, n_mfma)                                           \
  do {                                                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, (n_vm), 0);                     \
    X3_PIPE(n_rd, n_mfma);                                                      \
  } while (0)
#else
#define X3_PIPE_V(n_vm, n_rd, n_mfma) ((void)0)
#endif

__device__ __forceinline__ int soff(int row, int ch) { return RS * row + 16 * ch; }

// three-piece split of two floats (exact residuals: x - bf16(x) is representable in f32)
__device__ __forceinline__ void split2(float a, float b, bf16x2& p0, bf16x2& p1, bf16x2& p2) {
  const f32x2 x = {a, b};
  p0 = __builtin_convertvector(x, bf16x2);
#if defined(QD_X3_NOSPLIT)  // cost-ablation builds only: one piece
  p1 = p2 = bf16x2{};
  return;
#endif
  const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
  p1 = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
  p2 = __builtin_convertvector(r2, bf16x2);
}

__device__ __forceinline__ X3h split4(const float (&v)[4]) {
  bf16x2 a0, a1, a2, b0, b1, b2;
  split2(v[0], v[1], a0, a1, a2);
  split2(v[2], v[3], b0, b1, b2);
  X3h o;
  o.p[0] = __builtin_shufflevector(a0, b0, 0, 1, 2, 3);
  o.p[1] = __builtin_shufflevector(a1, b1, 0, 1, 2, 3);
  o.p[2] = __builtin_shufflevector(a2, b2, 0, 1, 2, 3);
  return o;
}

__device__ __forceinline__ X3 split8(const float (&v)[8]) {
  const float lo[4] = {v[0], v[1], v[2], v[3]}, hi[4] = {v[4], v[5], v[6], v[7]};
  const X3h a = split4(lo), b = split4(hi);
  X3 o;
#pragma unroll
  for (int p = 0; p < 3; p++) o.p[p] = __builtin_shufflevector(a.p[p], b.p[p], 0, 1, 2, 3, 4, 5, 6, 7);
  return o;
}

__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// a*b over one K-step of 16 at f32 accuracy (small terms first)
__device__ __forceinline__ f32x16 mma3(const X3& a, const X3& b, f32x16 c) {
  c = mfma16(a.p[2], b.p[0], c);
  c = mfma16(a.p[1], b.p[1], c);
  c = mfma16(a.p[0], b.p[2], c);
  c = mfma16(a.p[1], b.p[0], c);
  c = mfma16(a.p[0], b.p[1], c);
  return mfma16(a.p[0], b.p[0], c);
}

// The W2 fragments a wave multiplies with, as bf16 pieces in HBM (L2-resident, 96 KB per net),
// split once per launch by k_x3_prep: unit (16 bytes) of (net, wave w, use u, k-step s, piece p,
// lane). Use 0 = A of L2: W2[n_own][kk]; use 1 = B of dh1: W2[kk][n_own]; kk = 8s + 64h + j for
// lane half h, element j (n_own = 32w + lane % 32). Loading the pieces (3 dwordx4 per k-step)
// replaces re-splitting f32 slices held in registers each round (~45 VALU per k-step and operand,
// and the slices' 128 VGPRs); same pieces, so the same bits.
__device__ __forceinline__ int wimg_unit(int net, int w, int u, int s, int p, int lane) {
  return ((((net * 4 + w) * 2 + u) * 8 + s) * 3 + p) * 64 + lane;
}
static_assert(int64_t(2 * 4 * 2 * 8 * 3 * 64) * 16 == WIMG_BYTES, "pre-split image size");

// the same product with the five small terms in their own accumulator `sm` (magnitude ~2^-8 of the
// sum): the bf16 MFMA truncates what falls below its f32 result (tools/diag/mfma_rounding.hip, a
// small negative bias per instruction); five tiny-term MFMAs per k-step onto the full-size running
// sum gave the forward outputs a systematic bias of up to ~48 ulp over a 128-deep product, which
// the minibatch sums of the bias / head gradients accumulate linearly. The caller adds sm once.
__device__ __forceinline__ void mma3s(const X3& a, const X3& b, f32x16& big, f32x16& sm) {
  sm = mfma16(a.p[2], b.p[0], sm);
  sm = mfma16(a.p[1], b.p[1], sm);
  sm = mfma16(a.p[0], b.p[2], sm);
  sm = mfma16(a.p[1], b.p[0], sm);
  sm = mfma16(a.p[0], b.p[1], sm);
  big = mfma16(a.p[0], b.p[0], big);
}

__device__ __forceinline__ bf16x8 rd16(const char* L, int off) { return *reinterpret_cast<const bf16x8*>(L + off); }

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / columns 4p..4p+3 of a 4 x 16
// block; lane i receives column i of the 4 rows (row q in element q)
__device__ __forceinline__ s16x4 rdtr(const char* L, int off) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(L + off));
}

// x(lane) + x(lane ^ 32) in every lane (v_permlane32_swap of x with itself: the first result holds
// lanes 0-31's values in every lane, the second lanes 32-63's; the sum is the same either order)
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[1]) + __uint_as_float(p[0]);
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(bf16x8, s16x8(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7)));
}

}  // namespace x3
}  // namespace lrn
}  // namespace quadenv
