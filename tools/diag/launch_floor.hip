// Diagnostic (not product): the fixed cost of one launch on MI355X -- an empty kernel at the step
// kernel's launch shapes (256 blocks x 512 threads = k_step_h at 65,536 envs; 64 x 128; 1024 x 256),
// a kernel whose waves only write one dword each, and one that writes the step's 8 MB of state +
// obs rows -- graph-replayed back to back like bench.py, HIP events around 20 x 100 launches.
// Build: hipcc --offload-arch=gfx950 -O3 -o launch_floor launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_empty(float*, int) {}
__global__ void k_one(float* p, int) {
  if ((threadIdx.x & 63) == 0) p[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = 1.f;
}
// every thread writes `per` dwords, coalesced (the step writes ~30 dwords per env)
__global__ void k_write(float* p, int per) {
  const size_t n = size_t(gridDim.x) * blockDim.x, i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (int k = 0; k < per; k++) p[size_t(k) * n + i] = float(k);
}
// every thread reads `per` dwords and writes them back (a copy of per x 4 B per thread)
__global__ void k_copy(float* p, int per) {
  const size_t n = size_t(gridDim.x) * blockDim.x, i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  float v[64];
#pragma unroll
  for (int k = 0; k < 64; k++) if (k < per) v[k] = p[size_t(k) * n + i];
#pragma unroll
  for (int k = 0; k < 64; k++) if (k < per) p[size_t(k) * n + i] = v[k] + 1.f;
}

typedef void (*KF)(float*, int);

float time_kernel(KF f, int grid, int block, float* buf, int per) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < 100; k++) hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, s, buf, per);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 5; w++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < 20; r++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return ms * 1e3f / 2000.f;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, size_t(256) << 20));
  CK(hipMemset(buf, 0, size_t(256) << 20));
  struct { const char* name; KF f; int grid, block, per; } cases[] = {
      {"empty 256x512", k_empty, 256, 512, 0},   {"empty 256x256", k_empty, 256, 256, 0},
      {"empty 64x128", k_empty, 64, 128, 0},     {"empty 1024x256", k_empty, 1024, 256, 0},
      {"empty 2048x64", k_empty, 2048, 64, 0},   {"one-dword 256x512", k_one, 256, 512, 0},
      {"write 30 dw/env 256x256 (7.9 MB)", k_write, 256, 256, 30},
      {"write 30 dw/env 512x128 (7.9 MB)", k_write, 512, 128, 30},
      {"copy 35 dw/env 256x256 (2 x 9.2 MB)", k_copy, 256, 256, 35},
      {"copy 35 dw/env 1024x64 (2 x 9.2 MB)", k_copy, 1024, 64, 35},
  };
  for (int rep = 0; rep < 2; rep++)
    for (auto& c : cases) printf("%-40s %.3f us/launch\n", c.name, time_kernel(c.f, c.grid, c.block, buf, c.per));
  CK(hipFree(buf));
  return 0;
}
