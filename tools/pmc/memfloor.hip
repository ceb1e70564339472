// Profiling tool (not product): the memory floor of one k_step launch -- the same SoA loads,
// action load, LDS-staged obs rows, reward/flag and state stores, with the physics replaced by
// a trivial update -- graph-replayed like bench.py. Variants: plain stores, write-through (sc1)
// stores of the state. Prints us/launch for N envs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <bool WT>
__global__ __launch_bounds__(256) void pass(float* __restrict__ S, int* __restrict__ stepc, const float4* __restrict__ act,
                                            float* __restrict__ obs, float* __restrict__ rew, unsigned char* __restrict__ term,
                                            unsigned char* __restrict__ trunc, int n, int chain) {
  __shared__ float4 lds[256 * 3];
  const int i = blockIdx.x * 256 + threadIdx.x;
  float x[25];
  float acc = 0.f;
  if (i < n) {
#pragma unroll
    for (int f = 0; f < 25; f++) { x[f] = S[size_t(f) * n + i]; }
    const float4 a = act[i];
    acc = a.x + a.y + a.z + a.w;
#pragma unroll
    for (int f = 0; f < 25; f++) { x[f] = x[f] * 0.999f + acc * 1e-3f; }
    // dependent compute chains (4 independent chains -> ILP 4), `chain` FMAs each
    float c0 = x[0], c1 = x[1], c2 = x[2], c3 = x[3];
    for (int k = 0; k < chain; k++) {
      c0 = __builtin_fmaf(c0, 0.9999f, 1e-4f); c1 = __builtin_fmaf(c1, 0.9999f, 1e-4f);
      c2 = __builtin_fmaf(c2, 0.9999f, 1e-4f); c3 = __builtin_fmaf(c3, 0.9999f, 1e-4f);
    }
    x[0] = c0; x[1] = c1; x[2] = c2; x[3] = c3;
    int st = stepc[i] + 1;
    rew[i] = x[0];
    term[i] = x[1] > 100.f;
    trunc[i] = st > 1000000;
#pragma unroll
    for (int f = 0; f < 25; f++) {
      if (WT) __hip_atomic_store(&S[size_t(f) * n + i], x[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else S[size_t(f) * n + i] = x[f];
    }
    stepc[i] = st;
  }
  const int t = threadIdx.x;
  lds[3 * t] = make_float4(x[0], x[1], x[2], x[3]);
  lds[3 * t + 1] = make_float4(x[4], x[5], x[6], x[7]);
  lds[3 * t + 2] = make_float4(x[8], x[9], x[10], x[11]);
  __syncthreads();
  const int first = blockIdx.x * 256, rows = min(256, n - first);
  float4* dst = reinterpret_cast<float4*>(obs + size_t(first) * 12);
  for (int j = 0; j < 3; j++) { const int idx = j * 256 + t; if (idx < rows * 3) dst[idx] = lds[idx]; }
}

template <bool WT>
float run(int n, int launches, int chain = 0) {
  float *S, *obs, *rew; int* st; float4* act; unsigned char *te, *tr;
  CK(hipMalloc(&S, size_t(n) * 28 * 4)); CK(hipMalloc(&obs, size_t(n) * 48)); CK(hipMalloc(&rew, size_t(n) * 4));
  CK(hipMalloc(&st, size_t(n) * 4)); CK(hipMalloc(&act, size_t(n) * 16 * 8)); CK(hipMalloc(&te, n)); CK(hipMalloc(&tr, n));
  CK(hipMemset(S, 0, size_t(n) * 28 * 4)); CK(hipMemset(st, 0, size_t(n) * 4)); CK(hipMemset(act, 0, size_t(n) * 16 * 8));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < launches; k++)
    hipLaunchKernelGGL(pass<WT>, dim3((n + 255) / 256), dim3(256), 0, s, S, st, act + size_t(k % 8) * n, obs, rew, te, tr, n, chain);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 4; r++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipFree(S); (void)hipFree(obs); (void)hipFree(rew); (void)hipFree(st); (void)hipFree(act); (void)hipFree(te); (void)hipFree(tr);
  return ms * 1e3f / (4 * launches);
}

int main() {
  for (int chain : {0, 100, 250, 500, 1000}) {
    const float t = run<false>(65536, 100, chain);
    printf("n=65536 chain=%d x4 FMAs: %.2f us\n", chain, t);
  }
  for (int n : {4096, 65536, 262144, 1048576}) {
    const float a = run<false>(n, 100), b = run<true>(n, 100);
    const double bytes = 278.0 * n;
    printf("n=%d plain %.2f us (%.0f GB/s)  write-through %.2f us (%.0f GB/s)\n", n, a, bytes / a / 1e3, b, bytes / b / 1e3);
  }
  return 0;
}
