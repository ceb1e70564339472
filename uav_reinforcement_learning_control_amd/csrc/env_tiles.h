// env_tiles.h -- the env-state tiles in HBM and the per-env load/store of one step (device
// only), shared by the step kernels (quadenv.hip) and the fused rollout kernel (rollout.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "quad_physics.h"

namespace quadenv {

// Env state layout in HBM: tiles of 64 envs (one wave), each tile NFT fields x 64 lanes of 4 B
// (8,704 B). Field f of env i lives at (i / 64) * TILE_BYTES + f * 256 + (i % 64) * 4: a wave's
// accesses to one field are 256 contiguous bytes, and every field is an immediate offset from one
// per-lane byte offset (see Tiles).
constexpr int F_QPOS = 0, F_QVEL = 11, F_VOLT = 21, F_TGT = 22, F_RINT = 25, F_PREV = 28;
constexpr int F_STEP = 32, F_EP = 33;  // int32 step count, uint32 episode counter
constexpr int NFT = 34;
constexpr uint32_t TILE_BYTES = NFT * 64 * 4;

// The step kernels take the constant block as a separate `const KConsts<float>* __restrict__`
// argument and copy it into p.kc: the argument's noalias lets the compiler keep every constant read
// a scalar load even after the kernel's first global store. Read through a plain struct member it
// could not rule out a clobber, and constants read after a store became VMEM loads whose vmcnt
// waits (gfx9 counts stores too) drained the stores already issued.
struct KParams {
  const KConsts<float>* __restrict__ kc;  // per-handle constant block in device memory
  float* tiles;         // env state tiles (layout above)
  uint32_t tile_bytes;  // bytes of all tiles (< 4 GiB: one buffer resource)
  int32_t n;      // envs in the handle
  int32_t first;  // step launches cover envs [first, first + count)
  int32_t count;
  int32_t auto_reset;
  uint64_t seed;
  uint64_t gid_base;
};

// ---- addressing. All env state goes through ONE buffer resource and one per-lane byte offset
// (env_off); the field offset f * 256 splits into the instruction's 12-bit immediate and a constant
// SGPR (0 / 4096 / 8192), so a step's 60 state loads and stores need no address arithmetic and
// no address registers. (Plain [field][n] indexing gave each field a 64-bit VGPR address, computed
// for the load burst and held until the matching store: ~54 VGPRs and 2 waves per SIMD.) Other
// per-env arrays use the global saddr form: uniform base + 32-bit byte offset.
__device__ __forceinline__ uint32_t env_off(uint32_t i) { return (i >> 6) * TILE_BYTES + (i & 63u) * 4u; }
// Cache policy of the state loads and stores (AUX: 0 = default, 2 = nt): a template parameter of
// the step kernel, chosen by batch size at launch (quad_step_range). A step reads and writes each
// env's fields once; at the DRAM-bound sizes nt keeps them out of L2 and the Infinity Cache (2M envs
// 97 vs 149 us, 4M 268 vs 317, 8M 546 vs 634 for k_step_h), at 65,536 envs it spares the
// end-of-launch write-back of the dirty state lines (5.60-5.81 vs 5.83-5.92 us), and from 4,096 to
// 1M envs, where the next step reads the state back from the Infinity Cache, it costs 0-17 %
// (profiles/r04/r4_step_forms_nt.txt, r4_step_nt_sizes.txt). nt loads alone were slower.
template <int AUX>
struct TilesA {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit TilesA(const KParams& p)
      : r(__builtin_amdgcn_make_buffer_rsrc(p.tiles, 0, int(p.tile_bytes), 0x00020000)) {}
  // f must fold to a constant (unrolled loops): a lane-varying f would make the SGPR part divergent
  __device__ __forceinline__ uint32_t ldu(int f, uint32_t vo) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, vo + uint32_t(f & 15) * 256u, uint32_t(f >> 4) * 4096u, AUX);
  }
  __device__ __forceinline__ void stu(int f, uint32_t vo, uint32_t x) const {
    __builtin_amdgcn_raw_buffer_store_b32(x, r, vo + uint32_t(f & 15) * 256u, uint32_t(f >> 4) * 4096u, AUX);
  }
  __device__ __forceinline__ float ld(int f, uint32_t vo) const { return __builtin_bit_cast(float, ldu(f, vo)); }
  __device__ __forceinline__ void st(int f, uint32_t vo, float x) const { stu(f, vo, __builtin_bit_cast(uint32_t, x)); }
};
using Tiles = TilesA<0>;
template <typename T>
__device__ __forceinline__ T ldo(const T* b, uint32_t off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(b) + off);
}
template <typename T>
__device__ __forceinline__ void sto(T* b, uint32_t off, T v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(b) + off) = v;
}

template <int AUX = 0>
__device__ __forceinline__ void load_env(const KParams& p, int i, EnvRegs<float>& e, bool ctbr) {
  const TilesA<AUX> S(p);
  const uint32_t o = env_off(uint32_t(i));
#pragma unroll
  for (int j = 0; j < 3; j++) e.pos[j] = S.ld(F_QPOS + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.q[j] = S.ld(F_QPOS + 3 + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.th[j] = S.ld(F_QPOS + 7 + j, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.v[j] = S.ld(F_QVEL + j, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.w[j] = S.ld(F_QVEL + 3 + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.s[j] = S.ld(F_QVEL + 6 + j, o);
  e.volt = S.ld(F_VOLT, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.target[j] = S.ld(F_TGT + j, o);
  if (ctbr) {
#pragma unroll
    for (int j = 0; j < 3; j++) e.rint[j] = S.ld(F_RINT + j, o);
  } else {
    e.rint[0] = e.rint[1] = e.rint[2] = 0.f;
  }
  e.step = int32_t(S.ldu(F_STEP, o));
}

// the fields the physics and the observation need (not the voltage / CTBR integral: k_step_h's
// helper waves own the control path)
template <int AUX = 0>
__device__ __forceinline__ void load_env_motion(const KParams& p, int i, EnvRegs<float>& e) {
  const TilesA<AUX> S(p);
  const uint32_t o = env_off(uint32_t(i));
#pragma unroll
  for (int j = 0; j < 3; j++) e.pos[j] = S.ld(F_QPOS + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.q[j] = S.ld(F_QPOS + 3 + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.th[j] = S.ld(F_QPOS + 7 + j, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.v[j] = S.ld(F_QVEL + j, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.w[j] = S.ld(F_QVEL + 3 + j, o);
#pragma unroll
  for (int j = 0; j < 4; j++) e.s[j] = S.ld(F_QVEL + 6 + j, o);
#pragma unroll
  for (int j = 0; j < 3; j++) e.target[j] = S.ld(F_TGT + j, o);
  e.step = int32_t(S.ldu(F_STEP, o));
}

// A per-lane offset made opaque in the block that uses it (fresh_off): the field offsets o + f * 256
// are then formed in THIS basic block, where instruction selection folds them into the store's
// immediate. Without it the compiler CSEs them with the load burst's (a different block), and
// since selection folds addressing modes only within one block, each store took its own
// materialized address: 15 v_add held across the step (15 VGPRs -- k_step_hd spilled) and 15 VALU.
__device__ __forceinline__ uint32_t fresh_off(uint32_t o) {
  asm volatile("" : "+v"(o));
  return o;
}

template <int AUX = 0>
__device__ __forceinline__ void store_env(const KParams& p, int i, const EnvRegs<float>& e,
                                          bool ctbr) {
  const TilesA<AUX> S(p);
  const uint32_t o = fresh_off(env_off(uint32_t(i)));
#pragma unroll
  for (int j = 0; j < 3; j++) S.st(F_QPOS + j, o, e.pos[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) S.st(F_QPOS + 3 + j, o, e.q[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) S.st(F_QPOS + 7 + j, o, e.th[j]);
#pragma unroll
  for (int j = 0; j < 3; j++) S.st(F_QVEL + j, o, e.v[j]);
#pragma unroll
  for (int j = 0; j < 3; j++) S.st(F_QVEL + 3 + j, o, e.w[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) S.st(F_QVEL + 6 + j, o, e.s[j]);
  S.st(F_VOLT, o, e.volt);
#pragma unroll
  for (int j = 0; j < 3; j++) S.st(F_TGT + j, o, e.target[j]);
  if (ctbr) {
#pragma unroll
    for (int j = 0; j < 3; j++) S.st(F_RINT + j, o, e.rint[j]);
  }
  S.stu(F_STEP, o, uint32_t(e.step));
}

// Mark a loaded value as consumed here, before the step's first store. gfx9's vmcnt retires
// loads and stores in issue order: a value first read AFTER stores were issued (the episode
// counter, read only by the reset branch) makes its s_waitcnt drain those stores too -- a store
// round trip on every wave that resets.
__device__ __forceinline__ void settle(uint32_t x) { asm volatile("" ::"v"(x)); }

}  // namespace quadenv
