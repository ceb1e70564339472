// quad_lanes.h -- cross-lane primitives for the 4-lanes-per-env kernels (device only).
//
// An env is owned by a quad: lanes 4e..4e+3 of a wave (16 envs per wave64). Reductions and
// broadcasts inside the quad use DPP quad_perm, i.e. a VALU modifier: no LDS, no extra latency
// beyond the consuming instruction. Every call site is reached by all four lanes of a quad
// (validity and the auto-reset branch are quad-uniform), which DPP needs.
#pragma once

#include <hip/hip_runtime.h>

namespace quadenv {

// quad_perm selectors: lane j of a quad reads lane sel[j]; encoding sel0 | sel1<<2 | ...
constexpr int QP_XOR1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // [1,0,3,2]
constexpr int QP_XOR2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // [2,3,0,1]
template <int K>
constexpr int qp_bcast() { return K | (K << 2) | (K << 4) | (K << 6); }

template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, x)));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long v = __builtin_bit_cast(long long, x);
  const int lo = dpp_i<CTRL>(int(v)), hi = dpp_i<CTRL>(int(v >> 32));
  return __builtin_bit_cast(double, (long long)((unsigned long long)(unsigned)lo |
                                                ((unsigned long long)(unsigned)hi << 32)));
}

__device__ __forceinline__ float qsum(float x) {
  x += dpp_f<QP_XOR1>(x);
  return x + dpp_f<QP_XOR2>(x);
}
__device__ __forceinline__ double qsum(double x) {
  x += dpp_d<QP_XOR1>(x);
  return x + dpp_d<QP_XOR2>(x);
}
__device__ __forceinline__ int qor(int x) {
  x |= dpp_i<QP_XOR1>(x);
  return x | dpp_i<QP_XOR2>(x);
}
template <int K>
__device__ __forceinline__ float qbc(float x) { return dpp_f<qp_bcast<K>()>(x); }
template <int K>
__device__ __forceinline__ unsigned qbcu(unsigned x) { return unsigned(dpp_i<qp_bcast<K>()>(int(x))); }

// Lane groups of G = 1, 2 or 4 lanes per env (groups never straddle a quad).
// group_sum / group_or reduce over the G lanes; group_bc<K> broadcasts lane K of the group.
template <int G> __device__ __forceinline__ float group_sum(float x) {
  if (G >= 2) x += dpp_f<QP_XOR1>(x);
  if (G >= 4) x += dpp_f<QP_XOR2>(x);
  return x;
}
template <int G> __device__ __forceinline__ int group_or(int x) {
  if (G >= 2) x |= dpp_i<QP_XOR1>(x);
  if (G >= 4) x |= dpp_i<QP_XOR2>(x);
  return x;
}
template <int G, int K> constexpr int group_bc_ctrl() {
  return G == 4 ? qp_bcast<K>() : (K | (K << 2) | ((K + 2) << 4) | ((K + 2) << 6));
}
template <int G, int K> __device__ __forceinline__ float group_bc(float x) {
  if constexpr (G == 1) return x;
  else return dpp_f<group_bc_ctrl<G, K>()>(x);
}
template <int G, int K> __device__ __forceinline__ unsigned group_bcu(unsigned x) {
  if constexpr (G == 1) return x;
  else return unsigned(dpp_i<group_bc_ctrl<G, K>()>(int(x)));
}

// select the lane-p entry of a 4-vector held identically by every lane (p = lane & 3)
template <typename T>
__device__ __forceinline__ T pick4(int p, T a, T b, T c, T d) {
  return p == 0 ? a : (p == 1 ? b : (p == 2 ? c : d));
}

}  // namespace quadenv
