// learner_x3.hip -- the PPO minibatch gradient (row P) on bf16 MFMA with three-piece splits
// (k_ppo_grad_x3): f32 accuracy at the bf16 matrix rate.
//
// Every f32 operand x of the three 128-deep products (L2, dW2, dh1) and of L1 / dW1 is split into
// three bf16 pieces x = x0 + x1 + x2, each the round-to-nearest bf16 of what the previous pieces
// leave (exact: x0 takes the top 8 significant bits, the f32 residual x - x0 has at most 16, the
// second residual at most 8, so the three pieces hold x exactly outside the subnormal range). A
// product a*b is formed as the six MFMAs a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0 accumulated in f32
// (v_mfma_f32_32x32x16_bf16: exact bf16 products, f32 sums); the dropped a1b2 + a2b1 + a2b2 are
// <= ~2^-23 |ab|, one f32 rounding of the product. So each K-step of 16 costs 6 x 32 cycles instead
// of 8 x 64 cycles of v_mfma_f32_32x32x2_f32 (2.7x less matrix time) at f32-level error; the
// accuracy bar is the same as the f32 form's (tests/test_gpu_learner.py, both forms).
//
// Structure (per block: one net, 4 waves, wave w owns neurons 32w..32w+31 of both hidden layers,
// rounds of 64 minibatch rows = two 32-row tiles; the loss math is learner.hip's):
//   L1   h1^T = W1 x^T        E form (neurons in registers, rows on lanes)  -> H1 pieces image
//   L2   h2^T = W2 h1^T       E form: A = W2 rows (pre-split pieces from HBM, k_x3_prep), B = H1 row reads
//   head / loss / dL/dmean    VALU, as learner.hip
//   dh2  E form               -> DH2 pieces image; dW3 += dmean^T relu(h2) per lane (f32 FMAs in
//        registers, rows = lanes; the 32 lanes of each half are summed once at the end of the launch)
//   dW2  = dh2^T h1 (K = rows)  A = DH2, B = H1, both by transposed reads (ds_read_b64_tr_b16);
//        db2 per lane in f32 (VALU adds of the unsplit dh2, summed over the lanes at the end): the
//        MFMA-with-ones form accumulated over K = rows with the bf16 MFMA's truncating sums
//   dh1  R form (rows in registers): A = DH2 row reads, B = W2 columns (pre-split pieces); relu'(h1)
//        from the H1 image by transposed reads
//   dW1  = dh1^T x            the dh1 accumulator split in registers is the A operand; B = the
//        observation image by transposed reads; its column 12 is 1.0, so dW1's column 12 is db1
// The [64 row][128 neuron] bf16 images have 272-byte rows (see soff).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "../../include/quadenv.h"
#include "learner.h"
#include "learner_x3_common.h"

namespace quadenv {

int set_error(int code, const char* msg);  // quadenv.hip

namespace lrn {
namespace {

using namespace x3;


// LDS (bytes)
constexpr int IMG = RND * RS;                  // one [64 row][128 neuron] bf16 piece
constexpr int XROW = 32;                       // observation image row: 12 features, 1.0, 3 zeros (bf16)
constexpr int XIMG = RND * XROW;
constexpr int B_H1P = 0;                       // 3 pieces
constexpr int B_DH2P = B_H1P + 3 * IMG;        // 3 pieces
constexpr int B_XO = B_DH2P + 3 * IMG;         // [2 round buffers][3 pieces][64][16] bf16
constexpr int B_ZERO = B_XO + 2 * 3 * XIMG;    // 64 zero bytes: dW1's padded columns 16..31
constexpr int B_SC = B_ZERO + 64;              // f32 [2][64][8] row scalars: action 4, old logp, adv, return
constexpr int B_PART = B_SC + 2 * RND * 8 * 4; // f32 [4 waves][64][4] head partial sums
constexpr int B_W3T = B_PART + 4 * RND * 16;   // f32 [128][4] head weights, neuron-major
constexpr int B_B1 = B_W3T + H * 16, B_B2 = B_B1 + H * 4;
constexpr int B_TOTAL = B_B2 + H * 4;          // 162,368 B
static_assert(B_TOTAL <= 160 * 1024, "LDS budget");
static_assert(B_XO % 16 == 0 && B_SC % 16 == 0 && B_W3T % 16 == 0, "alignment");
static_assert(2 * LB * 8 <= 3 * IMG, "the advantage reduction aliases the DH2 image");




// k_x3_prep: blocks 0..31 split W2 (four (net, w, u, s) units of 64 lanes per 256-thread block);
// with adv != NULL blocks 32.. are the advantage-statistics blocks (adv_stats_block) -- one launch
// for both pre-passes of the gradient kernel
__device__ __forceinline__ void split_w2_unit(const float* __restrict__ wa, const float* __restrict__ wc,
                                              bf16x8* __restrict__ img, int b) {
  const int s = b & 7, u = (b >> 3) & 1, w = (b >> 4) & 3, net = b >> 6;
  const int lane = threadIdx.x & 63, h = lane >> 5, n_own = 32 * w + (lane & 31);
  const float* w1 = net ? wc : wa;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int kk = 8 * s + 64 * h + j;
    v[j] = u == 0 ? w1[n_own * H + kk] : w1[kk * H + n_own];
  }
  const X3 x = split8(v);
#pragma unroll
  for (int p = 0; p < 3; p++) img[wimg_unit(net, w, u, s, p, lane)] = x.p[p];
}
constexpr int SPLIT_BLOCKS = 128 / 4;
__global__ __launch_bounds__(256) void k_x3_prep(const float* __restrict__ wa, const float* __restrict__ wc,
                                                 bf16x8* __restrict__ img, const float* __restrict__ adv,
                                                 const int64_t* __restrict__ idx, int batch, double* __restrict__ part) {
  __shared__ double red[2][256];
  if (int(blockIdx.x) < SPLIT_BLOCKS) {
    split_w2_unit(wa, wc, img, 4 * blockIdx.x + (threadIdx.x >> 6));
    return;
  }
  adv_stats_block(adv, idx, batch, part, blockIdx.x - SPLIT_BLOCKS, red);
}



// The schedule below is the one measured best (round 5, profiles/r05/learner_*_ab.txt; the not-kept
// alternatives were A/B builds and are gone from the product source): L1 issues both tiles' MFMAs
// before either tile's ReLU / split / image writes; the loss terms run one row per lane; tile 1's dh2
// is computed in dW2's first k-steps (741-743 vs 755-759 us per 524,288-row minibatch same-box, the
// same gradient bits); relu'(h1)'s mask reads are issued in dh1's last k-step.

// how many k-steps ahead L2 / dh1 load their pre-split W2 pieces (global loads, L2-resident); round 5
// A/B (profiles/r05/learner_wpf_ab.txt): 3 is 5 % slower (register pressure), 1 the same as 2
constexpr int WPF = 2, WRING = WPF + 1;
static_assert(WPF >= 1 && WPF <= 3, "prefetch distance");

// QD_LPROBE (tools/probe/probe_learner.py builds only, never the product): the dump build records
// per-wave s_memtime stamps at the phase boundaries of round 2 into g.dump instead of the hidden
// pre-activations (sched barriers around each stamp: the probe build is slower; use the shares)
#if defined(QD_LPROBE)
#define LP(k)                                        \
  do {                                               \
    if (DUMP && rd == 2) {                           \
      __builtin_amdgcn_sched_barrier(0);             \
      stp[k] = __builtin_amdgcn_s_memtime();         \
      __builtin_amdgcn_sched_barrier(0);             \
    }                                                \
  } while (0)
#define LP_DUMP(x) ((void)0)
#else
#define LP(k) ((void)0)
#define LP_DUMP(x) x
#endif

template <int NOUT, bool DUMP = false>
__device__ __forceinline__ void body(const GArgs& g, char* __restrict__ L, int blk) {
  const NetW& W = NOUT == ACT ? g.actor : g.critic;
  float* const Lf = reinterpret_cast<float*>(L);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int n_own = 32 * w + l32;
  // transposed-read roles: lane 4 gq + gp of its 16-lane group; ghi = which 16 columns of a 32-block
  const int gq = (lane & 15) >> 2, gp = lane & 3, ghi = (lane >> 4) & 1;
  const int tr_col = 2 * ghi + (gp >> 1), tr_half = 8 * (gp & 1);

  // ---- advantage statistics of the minibatch (actor): fixed-order tree over the pre-pass partials
  float adv_mu = 0.f, adv_den = 1.f;
  if (NOUT == ACT && g.adv_part) {
    double* red = reinterpret_cast<double*>(L + B_DH2P);  // [2][LB], before the DH2 image is used
    red[tid] = g.adv_part[2 * tid];
    red[LB + tid] = g.adv_part[2 * tid + 1];
    __syncthreads();
    for (int o = LB / 2; o > 0; o >>= 1) {
      if (tid < o) { red[tid] += red[tid + o]; red[LB + tid] += red[LB + tid + o]; }
      __syncthreads();
    }
    const double n = double(g.batch), s = red[0], s2 = red[LB];
    const double var = fmax((s2 - s * s / n) / (n - 1.0), 0.0);
    adv_mu = float(s / n);
    adv_den = float(sqrt(var)) + 1e-8f;
  }
  const float adv_rden = 1.f / adv_den;

  // ---- small weights in LDS; the wave's W1 fragment split in registers
  for (int i = tid; i < H; i += LB) {
    Lf[B_B1 / 4 + i] = W.b0[i];
    Lf[B_B2 / 4 + i] = W.b1[i];
#pragma unroll
    for (int k = 0; k < 4; k++) Lf[B_W3T / 4 + 4 * i + k] = k < NOUT ? W.w2[k * H + i] : 0.f;
  }
  if (tid < 16) Lf[B_ZERO / 4 + tid] = 0.f;
  float b3[NOUT];
#pragma unroll
  for (int k = 0; k < NOUT; k++) b3[k] = W.b2[k];
  X3 w1x;  // A of L1: W1[n_own][f = 8h + j] (f >= 12: 0)
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = 8 * h + j < OBS ? W.w0[n_own * OBS + 8 * h + j] : 0.f;
    w1x = split8(v);
  }
  // this wave's pre-split W2 fragments (k_x3_prep); the base is made opaque each round so the
  // compiler cannot hoist the 48 loads out of the round loop (their 192 VGPRs would spill)
  const int wunit0 = wimg_unit(NOUT == ACT ? 0 : 1, w, 0, 0, 0, lane);
  float ls[ACT], sd[ACT], isd[ACT];  // isd: the row loop multiplies (a full-precision division is ~10 VALU)
  if constexpr (NOUT == ACT) {
#pragma unroll
    for (int k = 0; k < ACT; k++) { ls[k] = g.log_std[k]; sd[k] = expf(ls[k]); isd[k] = 1.f / sd[k]; }
  }

  // accumulators (whole launch)
  f32x16 dW2[4], dW1, dW1b, dW1s;  // dW1b / dW1s: the last round's dW1 (big / small terms)
  float dW3[NOUT][16];  // per lane: sum over this lane's rows of dL/dout[k] * relu(h2) of register r's neuron
  float dB2[16];  // per lane: sum over this lane's rows of dh2 of neuron 32w + acc_row(r, h)
#pragma unroll
  for (int r = 0; r < 16; r++) {
    dW1[r] = dW1b[r] = dW1s[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j++) dW2[j][r] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; r++)
#pragma unroll
    for (int k = 0; k < NOUT; k++) dW3[k][r] = 0.f;
#pragma unroll
  for (int r = 0; r < 16; r++) dB2[r] = 0.f;
  float db3[NOUT], dls[ACT], st[3] = {0.f, 0.f, 0.f};  // st: pg sum, vf sum, clipped count
#pragma unroll
  for (int k = 0; k < NOUT; k++) db3[k] = 0.f;
#pragma unroll
  for (int k = 0; k < ACT; k++) dls[k] = 0.f;

  const int per_block = NOUT == ACT ? g.per_block : g.per_block_c;
  const int s0 = blk * per_block;
  const int s1 = min(g.batch, s0 + per_block);
  const int rounds = s1 > s0 ? (s1 - s0 + RND - 1) / RND : 0;
  // Row staging, one round ahead: threads 0..191 gather the observation rows (float4 each),
  // threads 192..255 the row scalars; the minibatch indices are loaded two rounds ahead.
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
  // features 12..15 of every observation image row: 1.0 (dW1's column 12 is db1), 0, 0, 0 -- both
  // buffers, once (the per-round staging writes features 0..11 only)
  if (tid < 2 * RND) {
    const bf16x4 one = {__bf16(1.f), __bf16(0.f), __bf16(0.f), __bf16(0.f)}, zero = {};
    char* const XO = L + B_XO + (tid / RND) * 3 * XIMG + (tid % RND) * XROW + 24;
    *reinterpret_cast<bf16x4*>(XO) = one;
    *reinterpret_cast<bf16x4*>(XO + XIMG) = zero;
    *reinterpret_cast<bf16x4*>(XO + 2 * XIMG) = zero;
  }
  gather(index_of(0));
  int64_t next_row = index_of(1);
  __syncthreads();

#if defined(QD_LPROBE)
  uint64_t stp[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
  for (int rd = 0; rd < rounds; rd++) {
    const int base = s0 + rd * RND;
    uint64_t wbase = reinterpret_cast<uint64_t>(g.wimg);
    asm volatile("" : "+s"(wbase));
    typedef __attribute__((address_space(1))) const bf16x8 gbf16x8;  // global, not flat: no lgkmcnt
    gbf16x8* const WI = reinterpret_cast<gbf16x8*>(wbase) + wunit0;
    auto ldw = [&](int u, int s) {
      X3 x;
#pragma unroll
      for (int p = 0; p < 3; p++) x.p[p] = WI[((u * 8 + s) * 3 + p) * 64];
      return x;
    };
#define WLOAD(u, s) ldw(u, s)
    X3 wr[WRING];  // L2's first WPF k-steps: in flight through L1
#pragma unroll
    for (int k = 0; k < WPF; k++) wr[k] = WLOAD(0, k);
    LP(0);
    char* const XO = L + B_XO + (rd & 1) * 3 * XIMG;
    float* const SCI = Lf + B_SC / 4 + (rd & 1) * RND * 8;
    // threads 0..191 = waves 0-2, 192..255 = wave 3: a wave-uniform role (a scalar branch); the
    // constant columns 12..15 are written once before the loop, so no lane branches here (the
    // kernel's 8 spilled VGPRs went to 0)
    if (__builtin_amdgcn_readfirstlane(tid) < 3 * RND) {
      const float v[4] = {pf.x, pf.y, pf.z, pf.w};
      const X3h x = split4(v);
      const int c = tid % 3;
#pragma unroll
      for (int p = 0; p < 3; p++) *reinterpret_cast<bf16x4*>(XO + p * XIMG + srow * XROW + 8 * c) = x.p[p];
    } else {
      *reinterpret_cast<float4*>(SCI + srow * 8) = pf;
      SCI[srow * 8 + 4] = pfs[0]; SCI[srow * 8 + 5] = pfs[1]; SCI[srow * 8 + 6] = pfs[2];
    }
    bool valid[2];
#pragma unroll
    for (int t = 0; t < 2; t++) valid[t] = base + 32 * t + l32 < s1;
    X3_BAR();  // B1: observation image complete; the previous round's readers are done
    LP(1);

    // ---- L1 (E form): h1^T block w of both tiles -> H1 pieces
    // both tiles' operand reads and MFMAs first, then their ReLU / split / image writes (in program
    // order per tile the compiler kept tile 1's reads behind tile 0's image stores)
    f32x16 acc1[2];
    {
      X3 xb[2];
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int p = 0; p < 3; p++) xb[t].p[p] = rd16(XO, p * XIMG + (32 * t + l32) * XROW + 16 * h);
      f32x16 sm[2];
#pragma unroll
      for (int r = 0; r < 16; r++) {
        acc1[0][r] = Lf[B_B1 / 4 + 32 * w + acc_row(r, h)];
        sm[0][r] = 0.f;
      }
      acc1[1] = acc1[0];
      sm[1] = sm[0];
#pragma unroll
      for (int t = 0; t < 2; t++) mma3s(w1x, xb[t], acc1[t], sm[t]);
#pragma unroll
      for (int t = 0; t < 2; t++) acc1[t] += sm[t];
    }
#pragma unroll
    for (int t = 0; t < 2; t++) {
      f32x16& acc = acc1[t];
      if constexpr (DUMP) {
        LP_DUMP(if (valid[t])
          for (int r = 0; r < 16; r++) dump_pre(g.dump, NOUT == ACT ? 0 : 1, g.batch, base + 32 * t + l32, 0, 32 * w + acc_row(r, h), acc[r]));
      }
#pragma unroll
      for (int gg = 0; gg < 4; gg++) {  // registers 4gg.. = neurons 32w + 8gg + 4h + 0..3
        const float v[4] = {relu(acc[4 * gg]), relu(acc[4 * gg + 1]), relu(acc[4 * gg + 2]), relu(acc[4 * gg + 3])};
        const X3h x = split4(v);
        const int off = soff(32 * t + l32, 4 * w + gg) + 8 * h;
#pragma unroll
        for (int p = 0; p < 3; p++) *reinterpret_cast<bf16x4*>(L + B_H1P + p * IMG + off) = x.p[p];
      }
    }
    LP(2);
    X3_BAR();  // B2: H1 image complete
    LP(3);

#if !defined(QD_X3_NOL2)
    // ---- L2 (E form): h2^T block w, A = W2 rows (pre-split pieces), B = H1 row reads
    f32x16 h2[2];
#pragma unroll
    for (int r = 0; r < 16; r++) h2[0][r] = Lf[B_B2 / 4 + 32 * w + acc_row(r, h)];
    h2[1] = h2[0];
    f32x16 h2s[2];
#pragma unroll
    for (int r = 0; r < 16; r++) { h2s[0][r] = 0.f; h2s[1][r] = 0.f; }
    {  // software pipeline: step s's MFMAs with step s + 1's reads and step s + 2's weight pieces in flight
      X3 b[2];
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int p = 0; p < 3; p++) b[t].p[p] = rd16(L, B_H1P + p * IMG + soff(32 * t + l32, 8 * h));
#pragma unroll
      for (int s = 0; s < 8; s++) {
        X3 bn[2];
        if (s + WPF < 8) wr[(s + WPF) % WRING] = WLOAD(0, s + WPF);
        if (s < 7) {
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int p = 0; p < 3; p++) bn[t].p[p] = rd16(L, B_H1P + p * IMG + soff(32 * t + l32, s + 1 + 8 * h));
        }
#pragma unroll
        for (int t = 0; t < 2; t++) mma3s(wr[s % WRING], b[t], h2[t], h2s[t]);
        if (s + WPF < 8) X3_PIPE_V(3, 6, 12);
        else if (s < 7) X3_PIPE(6, 12);
        X3_SB();
        if (s < 7) { b[0] = bn[0]; b[1] = bn[1]; }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; t++) h2[t] += h2s[t];
#else
    f32x16 h2[2];
    for (int r = 0; r < 16; r++) { h2[0][r] = Lf[r]; h2[1][r] = Lf[r + 16]; }
#endif
    // Row staging for round rd + 1, issued after L2's weight-piece loads: vmcnt retires in issue
    // order, so a gather issued before them would expose its HBM latency at L2's first wait; from
    // here it has the rest of the round (the dh1 pieces are waited ~10k cycles later)
    gather(next_row);
    next_row = index_of(rd + 2);
    LP(4);
    if constexpr (DUMP) {
      LP_DUMP(for (int t = 0; t < 2; t++)
        if (valid[t])
          for (int r = 0; r < 16; r++) dump_pre(g.dump, NOUT == ACT ? 0 : 1, g.batch, base + 32 * t + l32, 1, 32 * w + acc_row(r, h), h2[t][r]));
    }
    // head partial sums over the wave's 32 neurons (the two lane halves hold 16 each): the 2 x NOUT
    // chains (each in neuron order) interleaved, so a dependent FMA waits on no other; the halves'
    // sum by v_permlane32_swap (a VALU swap; the shuffle was an LDS round trip per output)
    {
      float part[2][NOUT];
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int k = 0; k < NOUT; k++) part[t][k] = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const float4 w3 = *reinterpret_cast<const float4*>(Lf + B_W3T / 4 + 4 * (32 * w + acc_row(r, h)));
        const float wk[4] = {w3.x, w3.y, w3.z, w3.w};
#pragma unroll
        for (int t = 0; t < 2; t++) h2[t][r] = relu(h2[t][r]);
#pragma unroll
        for (int k = 0; k < NOUT; k++)
#pragma unroll
          for (int t = 0; t < 2; t++) part[t][k] = fmaf(wk[k], h2[t][r], part[t][k]);
      }
      // both halves hold the same sum (lo + hi == hi + lo) and write it to the same word
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int k = 0; k < NOUT; k++) Lf[B_PART / 4 + (w * RND + 32 * t + l32) * 4 + k] = xhalf_sum(part[t][k]);
    }
    LP(5);
    X3_BAR();  // B3: head partials complete
    LP(6);

    // ---- per-row loss terms and dL/d(head output) (every wave, identical arithmetic)
    float d[2][NOUT];
    // one row per lane (row = lane: tile h, row l32), then both tiles' d on every lane by one
    // v_permlane32_swap per output; the per-row sums accumulate on every lane of wave 0
    {
      const int e = lane;
      const bool vrow = h ? valid[1] : valid[0];
      const bool acc = w == 0 && vrow;
      float dd[NOUT];
      const float* PT = Lf + B_PART / 4;
      float out[NOUT];
#pragma unroll
      for (int k = 0; k < NOUT; k++)
        out[k] = (((PT[e * 4 + k] + PT[(RND + e) * 4 + k]) + PT[(2 * RND + e) * 4 + k]) + PT[(3 * RND + e) * 4 + k]) +
                 b3[k];
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
        const float dlp = vrow ? -g.inv_batch * A * (w1 + (1.f - w1) * inr) * r : 0.f;
#pragma unroll
        for (int k = 0; k < ACT; k++) dd[k] = dlp * z[k] * isd[k];
        // the row sums as selects, not branches (the same operations on the accumulating lanes)
        st[0] = acc ? st[0] + -fminf(sa, sb) : st[0];
        st[2] = acc ? st[2] + (fabsf(r - 1.f) > g.clip ? 1.f : 0.f) : st[2];
#pragma unroll
        for (int k = 0; k < ACT; k++) dls[k] = acc ? dls[k] + dlp * (z[k] * z[k] - 1.f) : dls[k];
      } else {
        const float diff = out[0] - SCI[e * 8 + 6];
        dd[0] = vrow ? 2.f * g.vf_coef * g.inv_batch * diff : 0.f;
        st[1] = acc ? st[1] + diff * diff : st[1];
      }
#pragma unroll
      for (int k = 0; k < NOUT; k++) {
        db3[k] = w == 0 ? db3[k] + dd[k] : db3[k];
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(dd[k]), __float_as_uint(dd[k]), false, false);
        d[0][k] = __uint_as_float(p[0]);  // lanes 0-31's value (tile 0's row) in every lane
        d[1][k] = __uint_as_float(p[1]);  // lanes 32-63's (tile 1's)
      }
    }
    LP(7);
    // ---- dh2 (E form) -> DH2 pieces; dW3 per lane
    // (one 4-neuron chunk of tile t: dh2 = relu'(h2) (d W3), dW3 / db2 per lane, the DH2 pieces)
    auto dh2_chunk = [&](int t, int gg) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = 4 * gg + u;
        const float4 w3 = *reinterpret_cast<const float4*>(Lf + B_W3T / 4 + 4 * (32 * w + acc_row(r, h)));
        const float wk[4] = {w3.x, w3.y, w3.z, w3.w};
        float gsum = 0.f;
#pragma unroll
        for (int k = 0; k < NOUT; k++) gsum = fmaf(wk[k], d[t][k], gsum);
        v[u] = h2[t][r] > 0.f ? gsum : 0.f;
#pragma unroll
        for (int k = 0; k < NOUT; k++) dW3[k][r] = fmaf(d[t][k], h2[t][r], dW3[k][r]);  // h2: relu'd
        dB2[r] += v[u];
      }
      const X3h x = split4(v);
      const int off = soff(32 * t + l32, 4 * w + gg) + 8 * h;
#pragma unroll
      for (int p = 0; p < 3; p++) *reinterpret_cast<bf16x4*>(L + B_DH2P + p * IMG + off) = x.p[p];
    };
    // dW2 reads only this wave's own DH2 columns (its neurons) and the H1 image (complete since
    // B2), so it needs no barrier: tile 0's dh2 first, then dW2's first two k-steps (rows 0..31 =
    // tile 0) with tile 1's dh2 chunks in their issue gaps, written before the k-step-2 reads of
    // rows 32..47 are issued (program order within the wave); B4 (every wave's DH2 columns) then
    // guards dh1's row reads. Per register r the dW3 / db2 sums keep the order tile 0, tile 1.
#pragma unroll
    for (int gg = 0; gg < 4; gg++) dh2_chunk(0, gg);
    LP(8);
    LP(9);

    X3 wr1[WRING];  // dh1's W2 pieces (ring, WPF k-steps ahead)
#if defined(QD_X3_NODW2)  // QD_X3_NO*: cost-ablation builds only (tools/x3_build.sh)
    // without dW2 tile 1's dh2 still has to be written before B4 (dh1 reads its rows)
#pragma unroll
    for (int gg = 0; gg < 4; gg++) dh2_chunk(1, gg);
#else
    // ---- dW2 slab (rows 32w..): K = the round's 64 rows, both operands by transposed reads
    {  // 20 operand blocks (per k-step s: A, then B of jb = 0..3), each read one unit ahead
      // The K order over the rows is free (both operands use it): the 4-row blocks of the transposed
      // reads take rows 4 apart (k-step s, lane half h: element j is row 16s + 2h + (j >> 2) + 4(j & 3)),
      // so a block's rows sit 16 banks apart on the 272-byte rows and a 32-lane half covers the 64
      // banks once (consecutive rows were 4-way conflicts)
      auto trblk = [&](int img, int s, int chunk) {
        const int r0 = 16 * s + 2 * h + 4 * gq;
        X3 x;
#pragma unroll
        for (int p = 0; p < 3; p++) {
          const char* I = L + img + p * IMG;
          x.p[p] = cat_tr(rdtr(I, soff(r0, chunk) + tr_half), rdtr(I, soff(r0 + 1, chunk) + tr_half));
        }
        return x;
      };
      X3 a = trblk(B_DH2P, 0, 4 * w + tr_col), b = trblk(B_H1P, 0, tr_col);
#pragma unroll
      for (int s = 0; s < 4; s++) {
#pragma unroll
        for (int jb = 0; jb < 4; jb++) {
          X3 an, bn;
          if (jb < 3) bn = trblk(B_H1P, s, 4 * (jb + 1) + tr_col);
          else if (s < 3) { an = trblk(B_DH2P, s + 1, 4 * w + tr_col); bn = trblk(B_H1P, s + 1, tr_col); }
          dW2[jb] = mma3(a, b, dW2[jb]);
          if (s < 2 && (jb & 1) == 0) dh2_chunk(1, 2 * s + (jb >> 1));  // before (s = 1, jb = 3)'s k-step-2 reads
          if (jb < 3) X3_PIPE(6, 6);
          else if (s < 3) X3_PIPE(12, 6);
          X3_SB();
          if (jb < 3) b = bn;
          else if (s < 3) { a = an; b = bn; }
        }
      }
    }
#endif
    X3_BAR();  // B4: every wave's DH2 columns (dh1 reads whole rows)
#pragma unroll
    for (int k = 0; k < WPF; k++) wr1[k] = WLOAD(1, k);
    LP(10);
#if !defined(QD_X3_NODH1)
    // ---- dh1 (R form) = relu'(h1) . (dh2 W2[:, block w]); then the dW1 slab (+ db1 in column 12)
    f32x16 dh1[2];
#pragma unroll
    for (int r = 0; r < 16; r++) { dh1[0][r] = 0.f; dh1[1][r] = 0.f; }
    f32x16 dh1s[2] = {dh1[0], dh1[1]};
    s16x4 rmask[2][4];
    {  // software pipeline as L2: A = DH2 row reads, B = pre-split W2 columns
      X3 a[2];
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int p = 0; p < 3; p++) a[t].p[p] = rd16(L, B_DH2P + p * IMG + soff(32 * t + l32, 8 * h));
#pragma unroll
      for (int s = 0; s < 8; s++) {
        X3 an[2];
        if (s + WPF < 8) wr1[(s + WPF) % WRING] = WLOAD(1, s + WPF);
        if (s < 7) {
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int p = 0; p < 3; p++) an[t].p[p] = rd16(L, B_DH2P + p * IMG + soff(32 * t + l32, s + 1 + 8 * h));
        }
        if (s == 7) {  // relu'(h1)'s mask reads under the last k-step's MFMAs
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int gg = 0; gg < 4; gg++)
              rmask[t][gg] = rdtr(L + B_H1P, soff(32 * t + 8 * gg + 4 * h + gq, 4 * w + tr_col) + tr_half);
        }
#pragma unroll
        for (int t = 0; t < 2; t++) {
          mma3s(a[t], wr1[s % WRING], dh1[t], dh1s[t]);
        }
        if (s + WPF < 8) X3_PIPE_V(3, 6, 12);
        else if (s < 7) X3_PIPE(6, 12);
        X3_SB();
        if (s < 7) { a[0] = an[0]; a[1] = an[1]; }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; t++) dh1[t] += dh1s[t];
    LP(11);
    // this round's dW1 in fresh accumulators (big / small terms), added to the launch total with
    // round-to-nearest VALU adds: one MFMA chain over every row of the block drifted by the
    // truncation bias (mma3s). The previous round's are added here, a round after their MFMAs
    // issued (no wait on them). Costs ~2.5 % of the launch (the flush's ~130 AGPR moves and adds
    // per round; flushing every 4th round under a branch spilled); buys first-layer gradients
    // within torch fp32's error (tests/test_gpu_learner.py)
    dW1 += dW1b + dW1s;
#pragma unroll
    for (int r = 0; r < 16; r++) { dW1b[r] = 0.f; dW1s[r] = 0.f; }
#pragma unroll
    for (int t = 0; t < 2; t++) {
      f32x16& acc = dh1[t];
      // register r: row 32t + acc_row(r, h), neuron n_own; relu'(h1) from the top piece of h1
      // (h1 >= 0 after the ReLU: its top piece is > 0 exactly when h1 is a positive normal)
#pragma unroll
      for (int gg = 0; gg < 4; gg++) {
        const s16x4 m = rmask[t][gg];
#pragma unroll
        for (int q = 0; q < 4; q++) acc[4 * gg + q] = m[q] > 0 ? acc[4 * gg + q] : 0.f;
      }
      // dW1[n][f] += sum_rows dh1[row][n] x[row][f]: registers 8s2.. are the A^T fragment of k-step
      // s2, rows 32t + 16 s2 + 8(j >> 2) + 4h + (j & 3); B from the observation image (zeros past f 15)
#pragma unroll
      for (int s2 = 0; s2 < 2; s2++) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = acc[8 * s2 + j];
        const X3 a = split8(v);
        const int rr = 32 * t + 16 * s2 + 4 * h + gq;
        X3 b;
#pragma unroll
        for (int p = 0; p < 3; p++) {
          const int o0 = ghi ? B_ZERO - B_XO - (rd & 1) * 3 * XIMG + 8 * gp : p * XIMG + rr * XROW + 8 * gp;
          const int o1 = ghi ? o0 : o0 + 8 * XROW;
          b.p[p] = cat_tr(rdtr(XO, o0), rdtr(XO, o1));
        }
        mma3s(a, b, dW1b, dW1s);
      }
    }
  #endif
    LP(12);
}
  dW1 += dW1b + dW1s;
#if defined(QD_LPROBE)
  if (DUMP && lane == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(g.dump) + (size_t(blockIdx.x) * 8 + (NOUT == ACT ? 0 : 4) + size_t(w)) * 16;
    for (int k = 0; k < 13; k++) o[k] = stp[k];
    o[15] = NOUT;
  }
#endif

  // ---- block partials in the parameter layout
  float* P = g.part + size_t(blk + (NOUT == ACT ? 0 : g.nb)) * PSTRIDE;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int n = 32 * w + acc_row(r, h);
    if (l32 < OBS) P[P_W1 + n * OBS + l32] = dW1[r];
    if (l32 == OBS) P[P_B1 + n] = dW1[r];
#pragma unroll
    for (int j = 0; j < 4; j++) P[P_W2 + n * H + 32 * j + l32] = dW2[j][r];
  }
  // dW3: sum the per-lane partials over the 32 lanes (rows) of each half; lane 0 of the half holds
  // neurons 32w + acc_row(r, h)
#pragma unroll
  for (int r = 0; r < 16; r++) {
#pragma unroll
    for (int k = 0; k < NOUT; k++) {
      float x = dW3[k][r];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o);
      if (l32 == 0) P[P_W3 + k * H + 32 * w + acc_row(r, h)] = x;
    }
  }
#pragma unroll
  for (int r = 0; r < 16; r++) {  // db2: the same lane sum
    float x = dB2[r];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (l32 == 0) P[P_B2 + 32 * w + acc_row(r, h)] = x;
  }
  if (w == 0) {  // the per-row sums (one row per lane: every lane of wave 0 holds some)
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

// block b: the actor over its rows, then the critic over the same rows (layout_both)
__global__ __launch_bounds__(LB, 1) void k_ppo_grad_x3(GArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds_x3[];
  body<ACT>(g, lds_x3, blockIdx.x);
  __syncthreads();  // the critic's first writes reuse LDS the actor's last round still reads
  body<1>(g, lds_x3, blockIdx.x);
}

// small minibatches (2 nb <= X3_BLOCKS: at most 128 rounds, 8,192 rows): the actor's and the critic's
// rounds of the same rows in separate blocks of one launch (blocks [0, nb) actor, [nb, 2 nb) critic),
// so a block runs one net and the launch lasts half as long -- the same rows per block and net as
// k_ppo_grad_x3, the same partial slots, so the same bits. train.py's minibatches of 128 rows are two
// rounds: two blocks each running both nets left 254 of the 256 CUs idle for both nets' latency.
__global__ __launch_bounds__(LB, 1) void k_ppo_grad_x3_sep(GArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds_x3s[];
  if (int(blockIdx.x) < g.nb)
    body<ACT>(g, lds_x3s, blockIdx.x);
  else
    body<1>(g, lds_x3s, blockIdx.x - g.nb);
}

// diagnostics: the same body with the hidden pre-activations recorded (quad_ppo_hidden)
__global__ __launch_bounds__(LB, 1) void k_ppo_grad_x3_dump(GArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds_x3d[];
  body<ACT, true>(g, lds_x3d, blockIdx.x);
  __syncthreads();
  body<1, true>(g, lds_x3d, blockIdx.x);
}

// one net per kernel (QUADENV_LEARNER_SPLIT=1): each gets its own register allocation; the two
// launch on two streams (fork / join by events) so their blocks share the chip
template <int NOUT>
__global__ __launch_bounds__(LB, 1) void k_ppo_grad_x3_net(GArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds_x3n[];
  body<NOUT>(g, lds_x3n, blockIdx.x);
}

}  // namespace

int launch_prep(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv) {
  hipLaunchKernelGGL(k_x3_prep, dim3(SPLIT_BLOCKS + (adv_stats ? ADV_BLOCKS : 0)), dim3(256), 0, s, g.actor.w1,
                     g.critic.w1, const_cast<bf16x8*>(static_cast<const bf16x8*>(g.wimg)), adv, g.idx, g.batch,
                     adv_stats);
  if (hipGetLastError() != hipSuccess) return set_error(QUAD_EHIP, "k_x3_prep launch failed");
  return QUAD_OK;
}

int launch_ppo_grad_x3(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv) {
  static bool opted[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return set_error(QUAD_EHIP, "hipGetDevice failed");
  if (!opted[dev]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_x3), hipFuncAttributeMaxDynamicSharedMemorySize,
                            B_TOTAL) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_x3_sep),
                            hipFuncAttributeMaxDynamicSharedMemorySize, B_TOTAL) != hipSuccess)
      return set_error(QUAD_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    opted[dev] = true;
  }
  if (int rc = launch_prep(g, s, adv_stats, adv)) return rc;
  const char* sp = std::getenv("QUADENV_LEARNER_SPLIT");
  if (sp && std::atoi(sp) != 0) {
    static hipStream_t s2[64] = {};
    static hipEvent_t ev[64][2] = {};
    static bool ready[64] = {};
    if (!ready[dev]) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_x3_net<ACT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, B_TOTAL) != hipSuccess ||
          hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_x3_net<1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, B_TOTAL) != hipSuccess ||
          hipStreamCreateWithFlags(&s2[dev], hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&ev[dev][0], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&ev[dev][1], hipEventDisableTiming) != hipSuccess)
        return set_error(QUAD_EHIP, "learner split: stream / event setup failed");
      ready[dev] = true;
    }
    if (hipEventRecord(ev[dev][0], s) != hipSuccess || hipStreamWaitEvent(s2[dev], ev[dev][0], 0) != hipSuccess)
      return set_error(QUAD_EHIP, "learner split: fork failed");
    hipLaunchKernelGGL(k_ppo_grad_x3_net<ACT>, dim3(g.nb), dim3(LB), B_TOTAL, s, g);
    GArgs gc = g;  // the critic kernel numbers its blocks from 0; its partials follow the actor's
    gc.part = g.part + size_t(g.nb) * PSTRIDE;
    gc.nb = 0;
    hipLaunchKernelGGL(k_ppo_grad_x3_net<1>, dim3(g.nbc), dim3(LB), B_TOTAL, s2[dev], gc);
    if (hipGetLastError() != hipSuccess) return set_error(QUAD_EHIP, "k_ppo_grad_x3_net launch failed");
    if (hipEventRecord(ev[dev][1], s2[dev]) != hipSuccess || hipStreamWaitEvent(s, ev[dev][1], 0) != hipSuccess)
      return set_error(QUAD_EHIP, "learner split: join failed");
    return QUAD_OK;
  }
  if (2 * g.nb <= X3_BLOCKS && g.nbc == g.nb)
    hipLaunchKernelGGL(k_ppo_grad_x3_sep, dim3(2 * g.nb), dim3(LB), B_TOTAL, s, g);
  else
    hipLaunchKernelGGL(k_ppo_grad_x3, dim3(g.nb), dim3(LB), B_TOTAL, s, g);
  if (hipGetLastError() != hipSuccess) return set_error(QUAD_EHIP, "k_ppo_grad_x3 launch failed");
  return QUAD_OK;
}

int launch_ppo_grad_x3_dump(const GArgs& g, hipStream_t s, double* adv_stats, const float* adv) {
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ppo_grad_x3_dump), hipFuncAttributeMaxDynamicSharedMemorySize,
                          B_TOTAL) != hipSuccess)
    return set_error(QUAD_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  if (int rc = launch_prep(g, s, adv_stats, adv)) return rc;
  hipLaunchKernelGGL(k_ppo_grad_x3_dump, dim3(g.nb), dim3(LB), B_TOTAL, s, g);
  if (hipGetLastError() != hipSuccess) return set_error(QUAD_EHIP, "k_ppo_grad_x3_dump launch failed");
  return QUAD_OK;
}

}  // namespace lrn
}  // namespace quadenv
