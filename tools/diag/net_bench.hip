// Diagnostic tool (not product): throughput of policy_net.h's net_forward (actor + critic) on
// LDS-staged weights, without the rollout around it -- one block per CU, each wave evaluating its
// NT tile(s) ITERS times (inputs perturbed per iteration so nothing is hoisted). Prints us per
// iteration and the wave-level matrix floor (6 x 32 cycles per 16-deep k-step and tile).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "policy_net.h"

using namespace quadenv;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int NT, int BLK>
__global__ __launch_bounds__(BLK) void k_nf(const float* __restrict__ packed, float* out, int iters) {
  extern __shared__ float lds[];
  stage_lds<BLK>(lds, packed);
  const int lane = threadIdx.x & 63;
  float xq[NT][8];
  for (int j = 0; j < NT; j++)
    for (int k = 0; k < 8; k++) xq[j][k] = 0.01f * float((lane * 7 + j * 3 + k) % 13) - 0.05f;
  float accum = 0.f;
  for (int it = 0; it < iters; it++) {
    float mean[NT][4], val[NT][1];
    net_forward2<NT>(lds, packed, xq, mean, val);
    for (int j = 0; j < NT; j++) {
      accum += mean[j][0] + mean[j][3] + val[j][0];
      xq[j][it & 7] += 1e-3f * mean[j][1];
    }
  }
  out[blockIdx.x * BLK + threadIdx.x] = accum;
}

template <int NT, int BLK>
void run(const float* packed, float* out, int iters) {
  const int bytes = LDS_F * 4;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nf<NT, BLK>), hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_nf<NT, BLK>), dim3(256), dim3(BLK), bytes, 0, packed, out, 2);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_nf<NT, BLK>), dim3(256), dim3(BLK), bytes, 0, packed, out, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const int envs_per_block = BLK / 64 * NT * 32;
  // matrix floor per SIMD per iteration: (4 L1 + 32 L2) k-steps x 6 MFMAs x 32 cycles x 2 nets x tiles per SIMD
  const double cyc = 36.0 * 6 * 32 * 2 * (envs_per_block / 4 / 32);
  printf("NT=%d BLK=%d: %.2f us per iteration (%d envs per CU); matrix floor %.0f cycles = %.2f us at 2.4 GHz\n", NT, BLK,
         best * 1e3 / iters, envs_per_block, cyc, cyc / 2400.0);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 32;
  std::vector<float> h(PACKED_ALL_F);  // (the pieces region holds arbitrary bf16 bits: timing only)
  for (int i = 0; i < PACKED_ALL_F; i++) h[i] = 0.05f * float((i * 2654435761u >> 7) % 2001) / 1000.f - 0.05f;
  float *packed, *out;
  CK(hipMalloc(&packed, PACKED_ALL_F * 4)); CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMemcpy(packed, h.data(), PACKED_ALL_F * 4, hipMemcpyHostToDevice));
  run<2, 256>(packed, out, iters);
  run<1, 512>(packed, out, iters);
  run<1, 256>(packed, out, iters);
  return 0;
}
