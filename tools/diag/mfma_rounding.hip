// Diagnostic tool (not product): how v_mfma_f32_32x32x16_bf16 rounds its f32 accumulation on
// gfx950 -- D = C + sum_k a_k b_k with every output element given the same 16 products (all rows
// of A equal, all columns of B equal, so the fragment layout does not matter). Prints D next to the
// round-to-nearest-even and round-toward-zero values of the exact sum, and the result of adding the
// same products one at a time with RNE (an fmaf chain), for cases that tell the rules apart.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_case(const float* a16, const float* b16, float c, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; j++) {
    a[j] = __bf16(a16[8 * (lane >> 5) + j]);
    b[j] = __bf16(b16[8 * (lane >> 5) + j]);
  }
  f32x16 acc;
  for (int r = 0; r < 16; r++) acc[r] = c;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

static float rz(double x) {  // round toward zero to float
  float f = float(x);
  if (std::fabs(double(f)) > std::fabs(x)) f = std::nextafter(f, 0.0f);
  return f;
}

int main() {
  float *da, *db, *dout;
  if (hipMalloc(&da, 64) || hipMalloc(&db, 64) || hipMalloc(&dout, 4)) return 1;
  struct Case { const char* name; float c; std::vector<float> a, b; };
  const float u = std::ldexp(1.0f, -23);  // ulp of 1.0
  std::vector<Case> cases = {
      {"C=1 + 0.25ulp", 1.f, {0.25f * u}, {1.f}},
      {"C=1 + 0.5ulp (tie to even)", 1.f, {0.5f * u}, {1.f}},
      {"C=1 + 0.75ulp", 1.f, {0.75f * u}, {1.f}},
      {"C=1 + 1.5ulp (tie)", 1.f, {1.5f * u}, {1.f}},
      {"C=1 - 0.25ulp/2", 1.f, {-0.125f * u}, {1.f}},
      {"C=1 - 0.75ulp/2", 1.f, {-0.375f * u}, {1.f}},
      {"C=-1 - 0.75ulp", -1.f, {-0.75f * u}, {1.f}},
      {"C=1 + 16 x 0.25ulp", 1.f, std::vector<float>(16, 0.25f * u), std::vector<float>(16, 1.f)},
      {"C=1 + 16 x 0.0625ulp", 1.f, std::vector<float>(16, 0.0625f * u), std::vector<float>(16, 1.f)},
      {"C=0: 1 + 2^-30 (small after big)", 0.f, {1.f, std::ldexp(1.f, -30)}, {1.f, 1.f}},
      {"C=0: 8 x (1 + 1/128) x (1 + 1/128)", 0.f, std::vector<float>(8, 1.f + 1.f / 128), std::vector<float>(8, 1.f + 1.f / 128)},
      {"C=1e-8, products 1 and -1", 1e-8f, {1.f, -1.f}, {1.f, 1.f}},
      {"C=3, 0.3ulp3 x 4", 3.f, std::vector<float>(4, 0.3f * 2 * u), std::vector<float>(4, 1.f)},
      // the accumulation window: C = 1 plus 16 equal terms of +-2^-k (exact sum 1 +- 2^(4-k))
      {"C=1 + 16 x 2^-25", 1.f, std::vector<float>(16, std::ldexp(1.f, -25)), std::vector<float>(16, 1.f)},
      {"C=1 + 16 x 2^-26", 1.f, std::vector<float>(16, std::ldexp(1.f, -26)), std::vector<float>(16, 1.f)},
      {"C=1 + 16 x 2^-27", 1.f, std::vector<float>(16, std::ldexp(1.f, -27)), std::vector<float>(16, 1.f)},
      {"C=1 + 16 x 2^-28", 1.f, std::vector<float>(16, std::ldexp(1.f, -28)), std::vector<float>(16, 1.f)},
      {"C=1 - 16 x 2^-25", 1.f, std::vector<float>(16, -std::ldexp(1.f, -25)), std::vector<float>(16, 1.f)},
      {"C=1 - 16 x 2^-26", 1.f, std::vector<float>(16, -std::ldexp(1.f, -26)), std::vector<float>(16, 1.f)},
      {"C=1 - 16 x 2^-27", 1.f, std::vector<float>(16, -std::ldexp(1.f, -27)), std::vector<float>(16, 1.f)},
      {"C=1 - 16 x 2^-28", 1.f, std::vector<float>(16, -std::ldexp(1.f, -28)), std::vector<float>(16, 1.f)},
      {"C=1 - 16 x 2^-30", 1.f, std::vector<float>(16, -std::ldexp(1.f, -30)), std::vector<float>(16, 1.f)},
      {"C=1, 8 x +2^-27 and 8 x -2^-27", 1.f,
       {std::ldexp(1.f, -27), std::ldexp(1.f, -27), std::ldexp(1.f, -27), std::ldexp(1.f, -27), std::ldexp(1.f, -27),
        std::ldexp(1.f, -27), std::ldexp(1.f, -27), std::ldexp(1.f, -27), -std::ldexp(1.f, -27), -std::ldexp(1.f, -27),
        -std::ldexp(1.f, -27), -std::ldexp(1.f, -27), -std::ldexp(1.f, -27), -std::ldexp(1.f, -27), -std::ldexp(1.f, -27),
        -std::ldexp(1.f, -27)}, std::vector<float>(16, 1.f)},
      {"C=2^-20, 1 and -1 (C under big terms)", std::ldexp(1.f, -20), {1.f, -1.f}, {1.f, 1.f}},
      {"C=2^-24, 1 and -1", std::ldexp(1.f, -24), {1.f, -1.f}, {1.f, 1.f}},
      {"C=-2^-24, 1 and -1", -std::ldexp(1.f, -24), {1.f, -1.f}, {1.f, 1.f}},
      {"C=2^-26, 1 and -1", std::ldexp(1.f, -26), {1.f, -1.f}, {1.f, 1.f}},
      {"C=1+2^-22, 1 and -1", 1.f + std::ldexp(1.f, -22), {1.f, -1.f}, {1.f, 1.f}},
      {"C=0: 1 + 3 x 2^-25 (non-multiple)", 0.f, {1.f, std::ldexp(1.f, -25), std::ldexp(1.f, -25), std::ldexp(1.f, -25)},
       {1.f, 1.f, 1.f, 1.f}},
      {"C=0: -1 - 3 x 2^-25", 0.f, {-1.f, -std::ldexp(1.f, -25), -std::ldexp(1.f, -25), -std::ldexp(1.f, -25)},
       {1.f, 1.f, 1.f, 1.f}},
  };
  for (auto& cs : cases) {
    float a[16] = {0}, b[16] = {0};
    for (size_t k = 0; k < cs.a.size(); k++) {
      a[k] = float(__bf16(cs.a[k]));  // what the MFMA sees
      b[k] = float(__bf16(cs.b[k]));
    }
    if (hipMemcpy(da, a, 64, hipMemcpyHostToDevice) || hipMemcpy(db, b, 64, hipMemcpyHostToDevice)) return 2;
    hipLaunchKernelGGL(k_case, dim3(1), dim3(64), 0, 0, da, db, cs.c, dout);
    float d = 0;
    if (hipMemcpy(&d, dout, 4, hipMemcpyDeviceToHost)) return 3;
    long double exact = cs.c;
    for (int k = 0; k < 16; k++) exact += (long double)a[k] * b[k];
    float chain = cs.c;
    for (int k = 0; k < 16; k++) chain = std::fmaf(a[k], b[k], chain);
    const float rne = float(double(exact));
    printf("%-40s D=%.9g (%a)  RNE=%.9g  RZ=%.9g  fmaf-chain=%.9g  -> %s\n", cs.name, d, d, rne, rz(double(exact)), chain,
           d == rne ? "RNE" : (d == rz(double(exact)) ? "RZ" : (d == chain ? "chain" : "other")));
  }
  return 0;
}
