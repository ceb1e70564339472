// valu_policy.hip -- comparison kernel (tools only, not product): the rollout policy's forward
// (SB3 ActorCritic of train.py: actor and critic MLPs 12 -> 128 -> 128, ReLU, heads 4 and 1) as a
// plain LDS-tiled f32 VALU kernel, the baseline the north star names for the MFMA policy kernel
// (csrc/policy.hip): "the tiny policy GEMM on MFMA only if rocprof shows it beating a plain
// LDS-tiled kernel". Classic register-blocked SGEMM tiling: a 256-thread block owns a 128-env tile
// and one net; thread (tx, ty) computes envs 8ty..8ty+7 x neurons 8tx..8tx+7 (64 accumulators),
// reading per k one float4 pair of activations ([k][env] image) and one of weights ([k][neuron]
// image) from LDS: 64 FMAs per 4 ds_read_b128. Blocks are persistent over env tiles so each stages
// its net's transposed weights (70 KB) once.
#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef VP_NAME
#define VP_NAME valu_policy_forward
#endif

namespace {

constexpr int H = 128, OBS = 12, TE = 128, LB = 256;
// LDS (floats)
constexpr int L_W2T = 0;                      // [k][n]
constexpr int L_H1 = L_W2T + H * H;           // [k][env]
constexpr int L_W1T = L_H1 + H * TE;          // [f][n]
constexpr int L_X = L_W1T + OBS * H;          // [f][env]
constexpr int L_B1 = L_X + OBS * TE, L_B2 = L_B1 + H, L_W3 = L_B2 + H;  // W3 [4][n]
constexpr int L_TOTAL = L_W3 + 4 * H;          // 35,840 floats = 140 KB

struct NetP {
  const float *w0, *b0, *w1, *b1, *w2, *b2;
};
struct Args {
  NetP net[2];
  const float* obs;
  float* mean;   // [n,4]
  float* value;  // [n]
  int n, ntiles;
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int NOUT>
__device__ __forceinline__ void run(const Args& a, const NetP& P, float* __restrict__ L) {
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  for (int i = tid; i < H * H; i += LB) L[L_W2T + (i % H) * H + i / H] = P.w1[i];  // W2T[k][n] = W2[n][k]
  for (int i = tid; i < H * OBS; i += LB) L[L_W1T + (i % OBS) * H + i / OBS] = P.w0[i];
  for (int i = tid; i < H; i += LB) {
    L[L_B1 + i] = P.b0[i];
    L[L_B2 + i] = P.b1[i];
#pragma unroll
    for (int o = 0; o < 4; o++) L[L_W3 + o * H + i] = o < NOUT ? P.w2[o * H + i] : 0.f;
  }
  float b3[NOUT];
#pragma unroll
  for (int o = 0; o < NOUT; o++) b3[o] = P.b2[o];
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int e0 = tile * TE;
    for (int i = tid; i < TE * OBS; i += LB) {
      const int e = i / OBS, f = i % OBS;
      L[L_X + f * TE + e] = e0 + e < a.n ? a.obs[size_t(e0) * OBS + i] : 0.f;
    }
    __syncthreads();  // weights (first tile), observation image
    float acc[8][8];
    {
      const float4 ba = ld4(L + L_B1 + 8 * tx), bb = ld4(L + L_B1 + 8 * tx + 4);
      const float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) acc[i][j] = bv[j];
    }
#pragma unroll
    for (int f = 0; f < OBS; f++) {
      const float4 xa = ld4(L + L_X + f * TE + 8 * ty), xb = ld4(L + L_X + f * TE + 8 * ty + 4);
      const float4 wa = ld4(L + L_W1T + f * H + 8 * tx), wb = ld4(L + L_W1T + f * H + 8 * tx + 4);
      const float x[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
      const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) acc[i][j] = fmaf(x[i], w[j], acc[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {  // relu(h1) -> [k = neuron][env]
      float* dst = L + L_H1 + (8 * tx + j) * TE + 8 * ty;
      *reinterpret_cast<float4*>(dst) = make_float4(fmaxf(acc[0][j], 0.f), fmaxf(acc[1][j], 0.f),
                                                    fmaxf(acc[2][j], 0.f), fmaxf(acc[3][j], 0.f));
      *reinterpret_cast<float4*>(dst + 4) = make_float4(fmaxf(acc[4][j], 0.f), fmaxf(acc[5][j], 0.f),
                                                        fmaxf(acc[6][j], 0.f), fmaxf(acc[7][j], 0.f));
    }
    __syncthreads();
    {
      const float4 ba = ld4(L + L_B2 + 8 * tx), bb = ld4(L + L_B2 + 8 * tx + 4);
      const float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) acc[i][j] = bv[j];
    }
#ifndef VP_UNROLL
#define VP_UNROLL 4
#endif
#if defined(VP_PIPE)
    float4 nxa = ld4(L + L_H1 + 8 * ty), nxb = ld4(L + L_H1 + 8 * ty + 4);
    float4 nwa = ld4(L + L_W2T + 8 * tx), nwb = ld4(L + L_W2T + 8 * tx + 4);
#endif
#pragma unroll VP_UNROLL
    for (int k = 0; k < H; k++) {
#if defined(VP_PIPE)
      const float4 xa = nxa, xb = nxb, wa = nwa, wb = nwb;
      const int kn = k + 1 < H ? k + 1 : k;
      nxa = ld4(L + L_H1 + kn * TE + 8 * ty); nxb = ld4(L + L_H1 + kn * TE + 8 * ty + 4);
      nwa = ld4(L + L_W2T + kn * H + 8 * tx); nwb = ld4(L + L_W2T + kn * H + 8 * tx + 4);
#else
      const float4 xa = ld4(L + L_H1 + k * TE + 8 * ty), xb = ld4(L + L_H1 + k * TE + 8 * ty + 4);
      const float4 wa = ld4(L + L_W2T + k * H + 8 * tx), wb = ld4(L + L_W2T + k * H + 8 * tx + 4);
#endif
      const float x[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
      const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#if defined(VP_PACKED)
      const f32x2 w2[4] = {{w[0], w[1]}, {w[2], w[3]}, {w[4], w[5]}, {w[6], w[7]}};
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const f32x2 xx = {x[i], x[i]};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          f32x2 c = {acc[i][2 * j], acc[i][2 * j + 1]};
          c = __builtin_elementwise_fma(xx, w2[j], c);
          acc[i][2 * j] = c.x; acc[i][2 * j + 1] = c.y;
        }
      }
#else
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) acc[i][j] = fmaf(x[i], w[j], acc[i][j]);
#endif
    }
    // heads: partial sums over the thread's 8 neurons, then over the 16 tx lanes of each env group
    float part[8][NOUT];
#pragma unroll
    for (int o = 0; o < NOUT; o++) {
      const float4 wa = ld4(L + L_W3 + o * H + 8 * tx), wb = ld4(L + L_W3 + o * H + 8 * tx + 4);
      const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
      for (int i = 0; i < 8; i++) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) s = fmaf(fmaxf(acc[i][j], 0.f), w[j], s);
        part[i][o] = s;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int o = 0; o < NOUT; o++) {
        float s = part[i][o];
#pragma unroll
        for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m);
        part[i][o] = s + b3[o];
      }
    if (tx == 0) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int e = e0 + 8 * ty + i;
        if (e < a.n) {
          if (NOUT == 4) *reinterpret_cast<float4*>(a.mean + size_t(e) * 4) =
              make_float4(part[i][0], part[i][NOUT > 1 ? 1 : 0], part[i][NOUT > 2 ? 2 : 0], part[i][NOUT > 3 ? 3 : 0]);
          else a.value[e] = part[i][0];
        }
      }
    }
    __syncthreads();  // the next tile overwrites the images
  }
}

__global__ __launch_bounds__(LB, 1) void k_valu_policy(Args a) {
  extern __shared__ float L[];
  if (blockIdx.y == 0) run<4>(a, a.net[0], L);
  else run<1>(a, a.net[1], L);
}

}  // namespace

extern "C" int VP_NAME(const float* const* p, const float* obs, int n, float* mean, float* value,
                                   int blocks_per_net, void* stream) {
  Args a{};
  for (int t = 0; t < 2; t++) a.net[t] = NetP{p[6 * t], p[6 * t + 1], p[6 * t + 2], p[6 * t + 3], p[6 * t + 4], p[6 * t + 5]};
  a.obs = obs; a.mean = mean; a.value = value; a.n = n; a.ntiles = (n + TE - 1) / TE;
  static bool opted = false;
  if (!opted) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_valu_policy), hipFuncAttributeMaxDynamicSharedMemorySize,
                            L_TOTAL * 4) != hipSuccess) return -1;
    opted = true;
  }
  const int nb = blocks_per_net < a.ntiles ? blocks_per_net : a.ntiles;
  hipLaunchKernelGGL(k_valu_policy, dim3(nb, 2), dim3(LB), L_TOTAL * 4, static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
