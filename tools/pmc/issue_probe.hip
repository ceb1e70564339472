// Profiling tool (not product): does a lone wave use the whole SIMD's VALU? The same 65,536
// independent 4-chain FMA streams (ILP 4) run as (a) 1,024 full waves (one per SIMD), (b) 2,048
// waves with only lanes 0-31 active (two per SIMD), (c) 2,048 full waves (131,072 streams, two per
// SIMD). If (b) takes ~half of (a), one wave issues VALU at half the SIMD's rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void chains(float* out, int iters, int active) {
  const int lane = threadIdx.x & 63;
  if (lane >= active) return;
  float c0 = threadIdx.x, c1 = c0 + 1.f, c2 = c0 + 2.f, c3 = c0 + 3.f;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      c0 = __builtin_fmaf(c0, 0.9999f, 1e-4f); c1 = __builtin_fmaf(c1, 0.9999f, 1e-4f);
      c2 = __builtin_fmaf(c2, 0.9999f, 1e-4f); c3 = __builtin_fmaf(c3, 0.9999f, 1e-4f);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
}

float run(int blocks, int active, int iters) {
  float* out; CK(hipMalloc(&out, size_t(blocks) * 256 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chains, dim3(blocks), dim3(256), 0, 0, out, iters, active);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 10; r++) hipLaunchKernelGGL(chains, dim3(blocks), dim3(256), 0, 0, out, iters, active);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipFree(out);
  return ms * 1e3f / 10;
}

int main() {
  const int iters = 200;  // 200 x 8 x 4 = 6,400 FMAs per lane
  const float a = run(256, 64, iters), b = run(512, 32, iters), c = run(512, 64, iters);
  printf("(a) 1024 full waves: %.1f us  (b) 2048 half waves: %.1f us  (c) 2048 full waves: %.1f us\n", a, b, c);
  printf("cycles per wave64 FMA at 2.2 GHz, (a): %.2f\n", a * 1e-6 * 2.2e9 / (iters * 32));
  return 0;
}
