// PMC calibration (profiling tool, not product): a coalesced dword-per-lane copy, the access
// shape of k_step's SoA loads/stores, over a known byte count. Run under rocprofv3 --pmc
// FETCH_SIZE / WRITE_SIZE to get bytes-per-counter-unit for this pattern on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void calib_copy_dword(const float* __restrict__ a, float* __restrict__ b, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = a[i] * 1.0001f;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : (64 << 20);  // floats per buffer (256 MiB default)
  float *a, *b;
  if (hipMalloc(&a, size_t(n) * 4) != hipSuccess || hipMalloc(&b, size_t(n) * 4) != hipSuccess) return 1;
  (void)hipMemset(a, 0, size_t(n) * 4);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(calib_copy_dword, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, n);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("calib: %d floats, %zu bytes read + %zu written per launch\n", n, size_t(n) * 4, size_t(n) * 4);
  (void)hipFree(a); (void)hipFree(b);
  return 0;
}
