// Profiling tool (not product): memory floor of the step's access shape at large N on the TILED
// layout (tiles of 64 envs x 34 fields x 4 B, as csrc/env_tiles.h): the 26 state fields read and
// written, the action float4 read, obs rows (48 B) + reward + 2 flags written, trivial compute.
// Variants: (dword) one dword load/store per field per lane, as k_step_g<1>; (lds) the wave moves
// its 8.7 KB tile with dwordx4 loads/stores staged through LDS, lanes read/write their env's
// fields from LDS; (copy) a plain dwordx4 streaming copy of the same byte counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NF = 26, TF = 34, TILE_FLOATS = TF * 64;  // 8,704 B per tile

template <int BLK>
__global__ __launch_bounds__(BLK) void k_dword(float* __restrict__ T, const float4* __restrict__ act, float* __restrict__ obs,
                                               float* __restrict__ rew, unsigned char* __restrict__ fl, int n) {
  __shared__ float4 lds[BLK * 3];
  const int i = blockIdx.x * BLK + threadIdx.x;
  float* tile = T + size_t(i >> 6) * TILE_FLOATS + (i & 63);
  float x[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) x[f] = tile[f * 64];
  const float4 a = act[i];
  const float s = a.x + a.y + a.z + a.w;
#pragma unroll
  for (int f = 0; f < NF; f++) x[f] = x[f] * 0.999f + s * 1e-3f;
  rew[i] = x[0];
  fl[i] = x[1] > 100.f;
  fl[n + i] = x[2] > 100.f;
#pragma unroll
  for (int f = 0; f < NF; f++) tile[f * 64] = x[f];
  const int t = threadIdx.x;
  lds[3 * t] = make_float4(x[0], x[1], x[2], x[3]);
  lds[3 * t + 1] = make_float4(x[4], x[5], x[6], x[7]);
  lds[3 * t + 2] = make_float4(x[8], x[9], x[10], x[11]);
  __syncthreads();
  float4* dst = reinterpret_cast<float4*>(obs + size_t(blockIdx.x) * BLK * 12);
  for (int j = 0; j < 3; j++) dst[j * BLK + t] = lds[j * BLK + t];
}

// each wave stages its tile: 9 dwordx4 loads per lane (8,704 B = 544 float4; 64 lanes x 9 = 576)
template <int BLK>
__global__ __launch_bounds__(BLK) void k_lds(float* __restrict__ T, const float4* __restrict__ act, float* __restrict__ obs,
                                             float* __restrict__ rew, unsigned char* __restrict__ fl, int n) {
  __shared__ float4 lds[BLK * 3];
  __shared__ float4 tl[BLK / 64][TILE_FLOATS / 4];
  const int i = blockIdx.x * BLK + threadIdx.x, l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float4* tile4 = reinterpret_cast<float4*>(T + size_t(i >> 6) * TILE_FLOATS);
  float4 v[9];
#pragma unroll
  for (int k = 0; k < 9; k++) { const int q = k * 64 + l; v[k] = q < NF * 16 ? tile4[q] : make_float4(0, 0, 0, 0); }
#pragma unroll
  for (int k = 0; k < 9; k++) { const int q = k * 64 + l; if (q < NF * 16) tl[wv][q] = v[k]; }
  const float* tf = reinterpret_cast<const float*>(tl[wv]);
  float x[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) x[f] = tf[f * 64 + l];
  const float4 a = act[i];
  const float s = a.x + a.y + a.z + a.w;
#pragma unroll
  for (int f = 0; f < NF; f++) x[f] = x[f] * 0.999f + s * 1e-3f;
  rew[i] = x[0];
  fl[i] = x[1] > 100.f;
  fl[n + i] = x[2] > 100.f;
  float* tw = reinterpret_cast<float*>(tl[wv]);
#pragma unroll
  for (int f = 0; f < NF; f++) tw[f * 64 + l] = x[f];
#pragma unroll
  for (int k = 0; k < 9; k++) { const int q = k * 64 + l; if (q < NF * 16) tile4[q] = tl[wv][q]; }
  const int t = threadIdx.x;
  lds[3 * t] = make_float4(x[0], x[1], x[2], x[3]);
  lds[3 * t + 1] = make_float4(x[4], x[5], x[6], x[7]);
  lds[3 * t + 2] = make_float4(x[8], x[9], x[10], x[11]);
  __syncthreads();
  float4* dst = reinterpret_cast<float4*>(obs + size_t(blockIdx.x) * BLK * 12);
  for (int j = 0; j < 3; j++) dst[j * BLK + t] = lds[j * BLK + t];
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4r, size_t n4w) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x, stride = size_t(gridDim.x) * 256;
  for (size_t k = i; k < n4w; k += stride) dst[k] = k < n4r ? src[k] : make_float4(1, 2, 3, 4);
}

template <typename F>
float timed(F launch, int reps) {
  hipStream_t s; CK(hipStreamCreate(&s));
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < reps; k++) launch(s, k);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 3; r++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / (3 * reps);
}

int main() {
  for (int n : {65536, 1048576, 4194304}) {
    float *T, *obs, *rew; float4* act; unsigned char* fl;
    CK(hipMalloc(&T, size_t(n / 64) * TILE_FLOATS * 4)); CK(hipMalloc(&obs, size_t(n) * 48)); CK(hipMalloc(&rew, size_t(n) * 4));
    CK(hipMalloc(&act, size_t(n) * 16 * 4)); CK(hipMalloc(&fl, size_t(n) * 2));
    CK(hipMemset(T, 0, size_t(n / 64) * TILE_FLOATS * 4)); CK(hipMemset(act, 0, size_t(n) * 64));
    const int reps = n >= 1048576 ? 50 : 200;
    const double bytes = 278.0 * n;
    auto rep = [&](const char* name, float us) { printf("n=%d %-14s %8.2f us  %6.0f GB/s\n", n, name, us, bytes / us / 1e3); };
    rep("dword/256", timed([&](hipStream_t s, int k) { hipLaunchKernelGGL(k_dword<256>, dim3(n / 256), dim3(256), 0, s, T, act + size_t(k % 4) * n, obs, rew, fl, n); }, reps));
    rep("dword/64", timed([&](hipStream_t s, int k) { hipLaunchKernelGGL(k_dword<64>, dim3(n / 64), dim3(64), 0, s, T, act + size_t(k % 4) * n, obs, rew, fl, n); }, reps));
    rep("lds/256", timed([&](hipStream_t s, int k) { hipLaunchKernelGGL(k_lds<256>, dim3(n / 256), dim3(256), 0, s, T, act + size_t(k % 4) * n, obs, rew, fl, n); }, reps));
    rep("lds/64", timed([&](hipStream_t s, int k) { hipLaunchKernelGGL(k_lds<64>, dim3(n / 64), dim3(64), 0, s, T, act + size_t(k % 4) * n, obs, rew, fl, n); }, reps));
    // streaming copy with the same read / write byte counts (120 B read, 158 B written per env)
    const size_t n4r = size_t(n) * 120 / 16, n4w = size_t(n) * 158 / 16;
    float4 *src, *dst; CK(hipMalloc(&src, n4w * 16)); CK(hipMalloc(&dst, n4w * 16));
    rep("copy", timed([&](hipStream_t s, int) { hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, s, src, dst, n4r, n4w); }, reps));
    (void)hipFree(src); (void)hipFree(dst);
    (void)hipFree(T); (void)hipFree(obs); (void)hipFree(rew); (void)hipFree(act); (void)hipFree(fl);
  }
  return 0;
}
