// quadenv.hip -- gfx950 kernels + the extern "C" ABI declared in include/quadenv.h.
//
// Data layout in HBM (one allocation per handle, field-major SoA, stride N):
//   soa[f * N + i], f = 0..10 qpos, 11..20 qvel, 21 voltage, 22..24 target, 25..27 CTBR integral
//   step[N] int32, episode[N] uint32
// One thread owns one env for a whole step; every per-field access of a wave is a coalesced
// 256-B line. The [N,12] row-major observation rows (48 B per env, what the policy GEMM wants)
// are transposed through LDS so that each wave-store instruction writes 1 KiB contiguously.
//
// Kernels
//   k_step<KIND, CTBR>   fused: (CTBR) -> mixer -> voltage -> mj_step -> obs -> reward ->
//                        termination/truncation -> SB3 auto-reset -> obs (LDS transpose)
//   k_reset<KIND>        HoverEnv.reset for all / masked envs
//   k_observe            HoverEnv._get_obs of the current state
//   k_random_actions     action_space.sample() stand-in (Philox), config 2
//   k_gae                SB3 GAE(lambda) reverse scan, one thread per env
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "../../include/quadenv.h"
#include "quad_lanes.h"
#include "quad_model.h"
#include "quad_physics.h"
#include "env_tiles.h"
#include "kconsts_default.h"
#include "rollout.h"

using namespace quadenv;

namespace {

constexpr int BLOCK = 256;

thread_local std::string g_err;

}  // namespace

namespace quadenv {
// shared with policy.hip: one last-error slot per thread for the whole library
int set_error(int code, const char* msg) {
  g_err = msg;
  return code;
}
}  // namespace quadenv

namespace {

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(QUAD_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
// wrapper kinds: the RelPosActWrapper output stage (obs7) and the CTBR action path
inline bool wrap_relpos(int32_t w) { return w == QUAD_WRAP_RELPOS || w == QUAD_WRAP_CTBR_RELPOS; }
inline bool wrap_ctbr(int32_t w) { return w == QUAD_WRAP_CTBR || w == QUAD_WRAP_CTBR_RELPOS; }

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e__ = (expr);                           \
    if (e__ != hipSuccess) return hip_fail(e__, #expr); \
  } while (0)

// The reset draw of episode `ep` (the env's counter, loaded by the caller with the state; the
// caller stores ep + 1).
template <int KIND>
__device__ __forceinline__ void reset_env(const KParams& p, int i, EnvRegs<float>& e, float obs[12],
                                          uint32_t ep) {
  float init12[12], tgt[3], s12[12];
  reset_draw(p.kc->init_lo, p.kc->init_span, p.kc->tgt_lo, p.kc->tgt_span, p.seed, p.gid_base + uint64_t(i),
             ep, init12, tgt);
  env_reset_from<float, KIND>(*p.kc, e, init12, tgt, obs, s12);
}

// The reset draws of a wave's resetting envs, compacted: each resetting lane publishes (env,
// episode) under its rank among them, every lane of the wave then computes one (env, block) Philox
// item, and the resetting lanes read back their 16 words. With <= 16 resets per wave (the common
// case) that is one Philox pass for the wave instead of four serial ones per resetting lane: a
// Philox block is 20 quarter-rate v_mad_u64_u32, and the draw was half the reset branch.
// Identical words to reset_draw (same counters), handed back as the uniforms u01(word): converted
// by the lane that made the block, 4 per lane instead of 16 in each resetting lane's stream.
// Called by every active lane of the wave.
struct ResetLds {
  uint32_t env[4][64], ep[4][64];
  float4 words[4][256];  // [wave][rank * 4 + block]
};
__device__ __forceinline__ void reset_words_wave(const KParams& p, ResetLds& L, uint32_t i, uint32_t ep,
                                                 bool rs, float u16[16]) {
  const uint64_t m = __ballot(rs);
  if (m == 0) return;
  const int w = threadIdx.x >> 6, lane = __lane_id();
  const int nres = __popcll(m);
  const int rank = __popcll(m & __lanemask_lt());
  if (rs) { L.env[w][rank] = i; L.ep[w][rank] = ep; }
  __builtin_amdgcn_wave_barrier();
  const int passes = (nres * 4 + 63) >> 6;
  for (int t = 0; t < passes; t++) {
    const int item = t * 64 + lane, rr = item >> 2;
    if (rr < nres) {
      uint32_t c[4];
      reset_block(p.seed, p.gid_base + uint64_t(L.env[w][rr]), L.ep[w][rr], uint32_t(item & 3), c);
      L.words[w][item] = make_float4(u01(c[0]), u01(c[1]), u01(c[2]), u01(c[3]));
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (rs) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const float4 v = L.words[w][rank * 4 + b];
      u16[4 * b] = v.x; u16[4 * b + 1] = v.y; u16[4 * b + 2] = v.z; u16[4 * b + 3] = v.w;
    }
  }
}

// One 12-float row per lane: three 16-byte stores when the row base is 16-byte aligned (a uniform
// test), else twelve dword stores. Row-per-lane stores are issue-bound: 12 scattered dword
// stores per lane cost the wave far more issue time than 3 dwordx4.
__device__ __forceinline__ void store_row12(float* __restrict__ base, uint32_t i, const float v[12]) {
  if ((reinterpret_cast<uintptr_t>(base) & 15u) == 0) {
    float4* b4 = reinterpret_cast<float4*>(base);
#pragma unroll
    for (int j = 0; j < 3; j++)
      sto(b4, 48u * i + 16u * j, make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]));
  } else {
#pragma unroll
    for (int j = 0; j < 12; j++) sto(base, 48u * i + 4u * j, v[j]);
  }
}

// Stage the block's [256,12] obs rows through LDS; write them as contiguous float4.
__device__ __forceinline__ void store_obs_rows(float4* lds, const float obs[12], float* out,
                                               int block_first, int n) {
  const int t = threadIdx.x;
  lds[3 * t + 0] = make_float4(obs[0], obs[1], obs[2], obs[3]);
  lds[3 * t + 1] = make_float4(obs[4], obs[5], obs[6], obs[7]);
  lds[3 * t + 2] = make_float4(obs[8], obs[9], obs[10], obs[11]);
  __syncthreads();
  const int rows = min(BLOCK, n - block_first);
  const int nf4 = rows * 3;
  float4* dst = reinterpret_cast<float4*>(out + size_t(block_first) * 12);
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int idx = j * BLOCK + t;
    if (idx < nf4) dst[idx] = lds[idx];
  }
}

// info["target", "target_vel", "target_acc"] of the step just taken (before any auto-reset);
// `ep` is the episode counter as loaded (the running episode is ep - 1)
template <int KIND>
__device__ __forceinline__ void target_info_of(const KConsts<float>& K, const KParams& p, int i,
                                               const EnvRegs<float>& e, uint32_t ep, float o[9]) {
  o[0] = e.target[0]; o[1] = e.target[1]; o[2] = e.target[2];
#pragma unroll
  for (int j = 3; j < 9; j++) o[j] = 0.f;
  if (KIND == QUAD_ENV_TRAJ)  // the target register holds the start position (= traj_pos[0])
    traj_spline_info(K, p.seed, p.gid_base + uint64_t(i), ep - 1u, e.target, e.step, o);
}

__device__ __forceinline__ void store_target_info(float* __restrict__ out, int i, const float o[9]) {
#pragma unroll
  for (int j = 0; j < 9; j++) sto(out, uint32_t(i) * 36u + 4u * j, o[j]);
}

// The step of one env per thread; K is the handle's constant block (k_step's SPEC form passes a
// compile-time copy of the default block, so every constant is an immediate).
template <int KIND, bool CTBR>
__device__ __forceinline__ void step_body(const KConsts<float>& K, KParams p, const float4* __restrict__ act,
                                          QuadStepOut out, float4* lds, ResetLds& rl) {
  const int block_first = p.first + blockIdx.x * BLOCK;
  const int end = p.first + p.count;
  // Every thread runs the step: the reset draws are computed by the whole wave (reset_words_wave),
  // so lanes past the last env shadow it (in-range loads) and store nothing.
  const bool live = block_first + int(threadIdx.x) < end;
  const int i = live ? block_first + int(threadIdx.x) : end - 1;
  float obs[12];
#if defined(QD_PROBE)
  uint64_t stamp_buf[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t* stamps = out.target_info ? stamp_buf : nullptr;  // probe builds: target_info = stamp buffer
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  bool rs_probe = false;
#else
  uint64_t* stamps = nullptr;
#endif
  QD_STAMP(stamps, 0);
  {
    EnvRegs<float> e;
    load_env(p, i, e, CTBR);
    const Tiles S(p);
    const uint32_t vo = env_off(uint32_t(i));
    const uint32_t ep = S.ldu(F_EP, vo);
    const float4 a4 = act[i];
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
#if defined(QD_PROBE)
    if (stamps) {  // stamp 1: every load of the step has landed
      settle(ep); settle(__builtin_bit_cast(uint32_t, a4.x)); settle(__builtin_bit_cast(uint32_t, e.volt));
      settle(__builtin_bit_cast(uint32_t, e.s[3])); settle(uint32_t(e.step)); settle(__builtin_bit_cast(uint32_t, e.target[2]));
    }
#endif
    QD_STAMP(stamps, 1);
    StepRes r;
    env_step<float, CTBR>(K, e, a, r, stamps);
    QD_STAMP(stamps, 5);
    settle(ep);
    const uint32_t o = uint32_t(i) * 4u;
#if defined(QD_PROBE)
    if (live && !stamps) {
#else
    if (live) {
#endif
      sto(out.reward, o, r.reward);
      sto(out.terminated, uint32_t(i), uint8_t(r.term));
      sto(out.truncated, uint32_t(i), uint8_t(r.trunc));
      if (out.motor_commands)
        sto(reinterpret_cast<float4*>(out.motor_commands), 4u * o,
            make_float4(r.motor[0], r.motor[1], r.motor[2], r.motor[3]));
      if (out.voltage_scale) sto(out.voltage_scale, o, r.vscale);
      if (out.state12) store_row12(out.state12, uint32_t(i), r.state12);
      if (out.target_info) {
        float info[9];
        target_info_of<KIND>(K, p, i, e, ep, info);
        store_target_info(out.target_info, i, info);
      }
    }
#pragma unroll
    for (int j = 0; j < 12; j++) obs[j] = r.obs[j];
#if defined(QD_ABL_NORESET)
    const bool rs = false;
#else
    const bool rs = live && (r.term || r.trunc) && p.auto_reset;
#endif
#if defined(QD_PROBE)
    rs_probe = rs;
#endif
    float u16[16];
#if defined(QD_ABL_NODRAW)  // cost ablation (tools only): the reset without its Philox draw / LDS hand-off
#pragma unroll
    for (int j = 0; j < 16; j++) u16[j] = 0.5f;
#else
    reset_words_wave(p, rl, uint32_t(i), ep, rs, u16);
#endif
    if (stamps && rs) QD_PIN_N(u16, 16);
    QD_STAMP(stamps, 8);
    if (rs) {
      if (out.terminal_obs) store_row12(out.terminal_obs, uint32_t(i), r.obs);
      QD_STAMP(stamps, 9);
      float init12[12], tgt[3], s12[12];
      reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
      env_reset_from<float, KIND>(K, e, init12, tgt, obs, s12);
      if (stamps) { QD_PIN_N(obs, 12); QD_PIN_N(e.q, 4); }
      QD_STAMP(stamps, 10);
      S.stu(F_EP, vo, ep + 1u);
    }
    if (stamps) { QD_PIN_N(obs, 12); QD_PIN_N(e.q, 4); QD_PIN_N(e.pos, 3); }
    QD_STAMP(stamps, 6);
    if (live) store_env(p, i, e, CTBR);
  }
  store_obs_rows(lds, obs, out.obs, block_first, p.first + p.count);
#if defined(QD_PROBE)
  QD_STAMP(stamps, 7);
  if (stamps && (threadIdx.x & 63) == 0) {
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
    uint64_t* dst = reinterpret_cast<uint64_t*>(out.target_info) + size_t(block_first + int(threadIdx.x)) / 64 * 16;
#pragma unroll
    for (int k = 0; k < 12; k++) dst[k] = stamp_buf[k];
    dst[12] = rt0; dst[13] = rt1;
    dst[14] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID (id 20)
    dst[15] = __popcll(__ballot(rs_probe));
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// k_step_h<KIND, CTBR, SPEC>: the step with HELPER waves. A block of 2 x HB threads owns HB envs:
// the first HB/64 waves step one env per lane; as many helper waves (one per SIMD, beside a step
// wave) take the two parts of HoverEnv.step that do not depend on the rigid-body state:
//   (C) the control path -- env_control: CTBR, denormalize, mixer, voltage sag, voltage update --
//       and its motor wrench (wrench_of), handed to the step wave through LDS, plus the
//       motor_commands / voltage_scale outputs. Meanwhile the step wave checks the state
//       (mj_checkPos/Vel) and accumulates gravity, base drag and prop drags (forward_base), which
//       need no controls; after barrier (C) it adds the wrench and finishes mj_step. Same
//       functions in the same order as env_step, so the same bits as the one-wave forms.
//   (R) every env's NEXT reset (the Philox words of its episode counter, the affine map, the
//       quaternion, the reset observation: reset_block / reset_affine_u / env_reset_from) into an
//       LDS image; after barrier (1) a resetting step lane only copies its row.
// With one step wave per SIMD (65,536 envs) the step wave's chain is the launch: the helpers run
// in the issue slots it leaves. HB = envs per block (one step wave + its helper wave per 64).
// Small batches take 64: at 4,096 envs 3.79 vs 4.24 us per launch with 256 (the batch spreads over
// 64 CUs instead of 16, and each barrier joins two waves instead of eight); at 65,536 the two
// measured equal (5.84-5.87 vs 5.83-5.87 us) and 128 slower (6.10), so batches above H_SMALL keep
// 256 (profiles/r02/ab_step_h_block.txt).
constexpr int H_SMALL = 32768;
#ifndef QD_H_PRE
#define QD_H_PRE 1  // Philox blocks of the helper's reset draw issued before barrier (C): 1 measured best (below)
#endif
// Small batches (64-env blocks, default cache policy: up to H_SMALL envs): each step lane stores its
// own obs row (three 16-byte stores; the non-resetting lanes before barrier 1, under the helper's
// reset draw) instead of the block's LDS transpose + barrier 2 + the shared copy -- 3.38 vs 3.45-3.46
// us at 4,096 envs; at 65,536 (256-env blocks) 6.43-6.54 vs 5.60-5.77, at 1M 54.5 vs 52.2-52.3, at 4M
// (k_step_hd) 262 vs 248-249, so those keep the transpose (profiles/r05/step_obs_direct_ab.txt)
template <int HB, bool NT>
constexpr bool obs_direct() { return HB == 64 && !NT; }
// Without CTBR, the helper image H and the control block CT as env-major 16-byte rows: the helper
// writes an env's 28 image words as seven 16-byte stores (and its control words as two) and a
// resetting step lane reads its row back the same way, instead of one word per field; same bits,
// 4,096 envs 3.32 vs 3.36 us, 4M 249.8-250.6 vs 253.8-254.6, 65,536 and 1M unchanged
// (profiles/r05/step_rowmajor_image_ab.txt). QD_H_ROWMAJOR=0: the field-major layout (A/B builds)
#ifndef QD_H_ROWMAJOR
#define QD_H_ROWMAJOR 1
#endif
// H / CT layout: field-major [f][HB], or (QD_H_ROWMAJOR, no CTBR) 16-byte env rows (H: 28 words, CT:
// CT_STRIDE); the CTBR kinds keep the field-major forms (config 5 at 65,536 envs measured 5.92 vs
// 5.78 us with row-major H)
template <bool CTBR>
constexpr bool ct_rows() { return QD_H_ROWMAJOR && !CTBR; }
constexpr int CT_STRIDE = 8;  // words per env row of CT (6 used)
constexpr int HROW = 28;  // floats per env in the helper image: pos 3, quat 4, v 3, w 3, target 3, obs 12
constexpr int HCTL = 9;   // floats per env from the control helper: Fsum, taum 3, volt, bad ctrl, rint 3
template <int KIND, bool CTBR, int HB, bool NT>
__device__ __forceinline__ void step_h_body(const KConsts<float>& K, KParams p, const float4* __restrict__ act,
                                            QuadStepOut out, float4* lds, float* H, float* CT) {
  constexpr int AUX = NT ? 2 : 0;  // the state tiles' cache policy (env_tiles.h)
  const int tid = threadIdx.x;
  const int block_first = p.first + blockIdx.x * HB;
  const int end = p.first + p.count;
  const int l = tid & (HB - 1);
  const bool live = block_first + l < end;
  const int i = live ? block_first + l : end - 1;
  const TilesA<AUX> S(p);
  const uint32_t vo = env_off(uint32_t(i));
#if defined(QD_PROBE)  // tools/probe/probe_step_h.py: per-wave stamps into the target_info buffer
  uint64_t stamp_buf[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t* stamps = out.target_info ? stamp_buf : nullptr;
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  float* const stamp_out = out.target_info;
  out.target_info = nullptr;
#else
  uint64_t* stamps = nullptr;
#endif
  QD_STAMP(stamps, 0);
  if (tid >= HB) {  // ---- helper
    // the helpers are the younger half of the block, the issue arbitration's losers: raised
    // priority while their control path is on the step wave's path (to barrier C), then back
    // (65,536 envs: 5.92 us vs 6.58 without; priority for the whole helper: 6.62 us)
    __builtin_amdgcn_s_setprio(1);
    // (C) env i's control path and motor wrench
    const uint32_t ep = S.ldu(F_EP, vo);
    const float4 a4 = act[i];
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
    const float volt = S.ld(F_VOLT, vo);
    float w[3] = {0.f, 0.f, 0.f}, ri[3] = {0.f, 0.f, 0.f};
    if (CTBR) {
#pragma unroll
      for (int j = 0; j < 3; j++) { w[j] = S.ld(F_QVEL + 3 + j, vo); ri[j] = S.ld(F_RINT + j, vo); }
    }
    if (stamps) { QD_PIN(ep); QD_PIN(a4.x); QD_PIN(a4.w); QD_PIN(volt); }
    QD_STAMP(stamps, 1);
    const Ctl<float> c = env_control<float, CTBR>(K, volt, w, ri, a);
    const Wrench<float> m = wrench_of<float, true>(K.ph, c.F, false);  // F = clip(., 0, max) * vs >= 0
    if constexpr (ct_rows<CTBR>()) {
      reinterpret_cast<float4*>(CT)[l * (CT_STRIDE / 4)] = make_float4(m.Fsum, m.taum[0], m.taum[1], m.taum[2]);
      reinterpret_cast<float4*>(CT)[l * (CT_STRIDE / 4) + 1] =
          make_float4(c.volt, any_bad_ctrl<float>(c.F) ? 1.f : 0.f, 0.f, 0.f);
    } else {
      CT[0 * HB + l] = m.Fsum;
#pragma unroll
      for (int j = 0; j < 3; j++) CT[(1 + j) * HB + l] = m.taum[j];
      CT[4 * HB + l] = c.volt;
      CT[5 * HB + l] = any_bad_ctrl<float>(c.F) ? 1.f : 0.f;
    }
    if (CTBR) {
#pragma unroll
      for (int j = 0; j < 3; j++) CT[(6 + j) * HB + l] = ri[j];
    }
    if (stamps) { QD_PIN(m.Fsum); QD_PIN(m.taum[0]); QD_PIN(m.taum[1]); QD_PIN(m.taum[2]); QD_PIN(c.volt); }
    QD_STAMP(stamps, 2);
    if (live) {
      const uint32_t o = uint32_t(i) * 4u;
      if (out.motor_commands)
        sto(reinterpret_cast<float4*>(out.motor_commands), 4u * o,
            make_float4(float(c.F[0]), float(c.F[1]), float(c.F[2]), float(c.F[3])));
      if (out.voltage_scale) sto(out.voltage_scale, o, float(c.vs));
    }
    // (R) env i's next reset, into H[f][l]: the first PRE Philox blocks before barrier (C), at
    // normal priority, in the slack the helper has while the step wave accumulates forward_base
    constexpr int PRE = QD_H_PRE;
    float u16[16];
    if (PRE > 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (uint32_t b = 0; b < uint32_t(PRE); b++) {
      uint32_t cw[4];
      reset_block(p.seed, p.gid_base + uint64_t(i), ep, b, cw);
#pragma unroll
      for (int j = 0; j < 4; j++) u16[4 * b + j] = u01(cw[j]);
    }
    __syncthreads();  // (C) the control results are staged
    QD_STAMP(stamps, 3);
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (uint32_t b = uint32_t(PRE); b < 4; b++) {
      uint32_t cw[4];
      reset_block(p.seed, p.gid_base + uint64_t(i), ep, b, cw);
#pragma unroll
      for (int j = 0; j < 4; j++) u16[4 * b + j] = u01(cw[j]);
    }
    float init12[12], tgt[3], obs[12], s12[12];
    reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
    EnvRegs<float> e;
    env_reset_from<float, KIND>(K, e, init12, tgt, obs, s12);
    const float row[HROW] = {e.pos[0], e.pos[1], e.pos[2], e.q[0], e.q[1], e.q[2], e.q[3],
                             e.v[0], e.v[1], e.v[2], e.w[0], e.w[1], e.w[2],
                             e.target[0], e.target[1], e.target[2],
                             obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9],
                             obs[10], obs[11]};
    if constexpr (ct_rows<CTBR>()) {  // env-major rows (112 B, 16-byte aligned): seven 16-byte writes
#pragma unroll
      for (int q = 0; q < HROW / 4; q++)
        reinterpret_cast<float4*>(H)[l * (HROW / 4) + q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
    } else {
#pragma unroll
      for (int f = 0; f < HROW; f++) H[f * HB + l] = row[f];
    }
    QD_STAMP(stamps, 4);
    __syncthreads();  // (1) the image is complete
    QD_STAMP(stamps, 5);
    if constexpr (!obs_direct<HB, NT>()) __syncthreads();  // (2) the obs rows are staged
    QD_STAMP(stamps, 6);
  } else {  // ---- step
    float obs[12];
    EnvRegs<float> e;
#if defined(QD_H_NOCTL)  // A/B builds only: the step wave runs the control path itself (round 2)
    load_env<AUX>(p, i, e, CTBR);
    const uint32_t ep = S.ldu(F_EP, vo);
    const float4 a4 = act[i];
    const float a[4] = {a4.x, a4.y, a4.z, a4.w};
    StepRes r;
    env_step<float, CTBR>(K, e, a, r);
    __syncthreads();  // (C)
#else
    load_env_motion<AUX>(p, i, e);
    const uint32_t ep = S.ldu(F_EP, vo);
    if (stamps) { QD_PIN(ep); QD_PIN_N(e.pos, 3); QD_PIN_N(e.q, 4); QD_PIN_N(e.th, 4); QD_PIN_N(e.v, 3);
                  QD_PIN_N(e.w, 3); QD_PIN_N(e.s, 4); QD_PIN_N(e.target, 3); QD_PIN(e.step); }
    QD_STAMP(stamps, 1);
    // mujoco.mj_step up to the controls: mj_checkPos/Vel, gravity + base + prop drag
    const bool bad = check_state(e);
    float qn[4] = {e.q[0], e.q[1], e.q[2], e.q[3]};
    normalize4(qn);
    ForceAcc<float> fa;
    forward_base(K.ph, qn, e.th, e.v, e.w, e.s, fa);
    if (stamps) { QD_PIN_N(fa.FB, 3); QD_PIN_N(fa.tau, 3); QD_PIN_N(fa.Qs, 4); QD_PIN_N(fa.R, 9); }
    QD_STAMP(stamps, 2);
    __syncthreads();  // (C)
    QD_STAMP(stamps, 3);
    Wrench<float> m;
    float ct_bad;
    if constexpr (ct_rows<CTBR>()) {
      const float4 c0 = reinterpret_cast<const float4*>(CT)[l * (CT_STRIDE / 4)];
      const float4 c1 = reinterpret_cast<const float4*>(CT)[l * (CT_STRIDE / 4) + 1];
      m.Fsum = c0.x; m.taum[0] = c0.y; m.taum[1] = c0.z; m.taum[2] = c0.w;
      e.volt = c1.x;
      ct_bad = c1.y;
    } else {
      m.Fsum = CT[0 * HB + l];
#pragma unroll
      for (int j = 0; j < 3; j++) m.taum[j] = CT[(1 + j) * HB + l];
      e.volt = CT[4 * HB + l];
      ct_bad = CT[5 * HB + l];
    }
    if (CTBR) {
#pragma unroll
      for (int j = 0; j < 3; j++) e.rint[j] = CT[(6 + j) * HB + l];
    } else {
      e.rint[0] = e.rint[1] = e.rint[2] = 0.f;
    }
    if (bad || ct_bad != 0.f) {  // mj_fwdActuation: bad state / bad ctrl -> zero ctrl
      const double z[4] = {0.0, 0.0, 0.0, 0.0};
      m = wrench_of<float, true>(K.ph, z, true);
    }
    physics_finish<float, true>(K.ph, e, qn, fa, m);
    if (stamps) { QD_PIN_N(e.pos, 3); QD_PIN_N(e.q, 4); QD_PIN_N(e.v, 3); QD_PIN_N(e.w, 3); }
    QD_STAMP(stamps, 4);
    StepRes r;
    env_post(K, e, r);
#endif
    if (stamps) { QD_PIN_N(r.obs, 12); QD_PIN(r.reward); QD_PIN(uint32_t(r.term)); }
    QD_STAMP(stamps, 5);
    settle(ep);
    const uint32_t o = uint32_t(i) * 4u;
    if (live) {
      sto(out.reward, o, r.reward);
      sto(out.terminated, uint32_t(i), uint8_t(r.term));
      sto(out.truncated, uint32_t(i), uint8_t(r.trunc));
      if (out.state12) store_row12(out.state12, uint32_t(i), r.state12);
      if (out.target_info) {
        float info[9];
        target_info_of<KIND>(K, p, i, e, ep, info);
        store_target_info(out.target_info, i, info);
      }
    }
#pragma unroll
    for (int j = 0; j < 12; j++) obs[j] = r.obs[j];
    const bool rs = live && (r.term || r.trunc) && p.auto_reset;
    QD_STAMP(stamps, 6);
    if constexpr (obs_direct<HB, NT>()) {
      if (live && !rs) store_row12(out.obs, uint32_t(i), r.obs);  // before (1): under the helper's draw
    }
    __syncthreads();  // (1)
    QD_STAMP(stamps, 7);
    if (rs) {
      if (out.terminal_obs) store_row12(out.terminal_obs, uint32_t(i), r.obs);
      float row[HROW];
      if constexpr (ct_rows<CTBR>()) {
#pragma unroll
        for (int q = 0; q < HROW / 4; q++) {
          const float4 v = reinterpret_cast<const float4*>(H)[l * (HROW / 4) + q];
          row[4 * q] = v.x; row[4 * q + 1] = v.y; row[4 * q + 2] = v.z; row[4 * q + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int f = 0; f < HROW; f++) row[f] = H[f * HB + l];
      }
#pragma unroll
      for (int j = 0; j < 3; j++) {
        e.pos[j] = row[j]; e.v[j] = row[7 + j]; e.w[j] = row[10 + j]; e.target[j] = row[13 + j];
        e.rint[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) { e.q[j] = row[3 + j]; e.th[j] = 0.f; e.s[j] = 0.f; }
#pragma unroll
      for (int j = 0; j < 12; j++) obs[j] = row[16 + j];
      e.volt = float(K.vnom);
      e.step = 0;
      S.stu(F_EP, fresh_off(vo), ep + 1u);
      if constexpr (obs_direct<HB, NT>()) store_row12(out.obs, uint32_t(i), obs);
    }
    if (live) store_env<AUX>(p, i, e, CTBR);
    if constexpr (!obs_direct<HB, NT>()) {
      lds[3 * l + 0] = make_float4(obs[0], obs[1], obs[2], obs[3]);
      lds[3 * l + 1] = make_float4(obs[4], obs[5], obs[6], obs[7]);
      lds[3 * l + 2] = make_float4(obs[8], obs[9], obs[10], obs[11]);
    }
    QD_STAMP(stamps, 8);
    if constexpr (!obs_direct<HB, NT>()) __syncthreads();  // (2)
    QD_STAMP(stamps, 9);
  }
  if constexpr (!obs_direct<HB, NT>()) {
    // the block's [HB,12] obs rows as contiguous float4 stores, shared by all 2 x HB threads
    const int nf4 = min(HB, end - block_first) * 3;
    float4* dst = reinterpret_cast<float4*>(out.obs + size_t(block_first) * 12);
    for (int idx = tid; idx < nf4; idx += 2 * HB) dst[idx] = lds[idx];
  }
#if defined(QD_PROBE)
  QD_STAMP(stamps, 10);
  if (stamps && (tid & 63) == 0) {  // wave (block, w): 16 words
    uint64_t* st = reinterpret_cast<uint64_t*>(stamp_out) + (size_t(blockIdx.x) * (2 * HB / 64) + size_t(tid >> 6)) * 16;
#pragma unroll
    for (int k = 0; k < 11; k++) st[k] = stamp_buf[k];
    st[12] = rt0;
    st[13] = __builtin_amdgcn_s_memrealtime();
    st[14] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    st[15] = tid >= HB ? 1u : 0u;
  }
#endif
}

template <int KIND, bool CTBR, bool SPEC, int HB, bool NT>
__global__ __launch_bounds__(2 * HB) void k_step_h(float* tiles, const float4* __restrict__ act, uint32_t tile_bytes,
                                                      int32_t first, int32_t count,
                                                      const KConsts<float>* __restrict__ kc, KParams p, QuadStepOut out) {
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;  // preloaded (see k_step)
  p.kc = kc;
  __shared__ float4 lds[HB * 3];
  __shared__ __attribute__((aligned(16))) float H[HROW * HB];
  __shared__ __attribute__((aligned(16))) float CT[(ct_rows<CTBR>() ? CT_STRIDE : (CTBR ? HCTL : HCTL - 3)) * HB];
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_h_body<KIND, CTBR, HB, NT>(K, p, act, out, lds, H, CT);
  } else {
    step_h_body<KIND, CTBR, HB, NT>(*kc, p, act, out, lds, H, CT);
  }
}

// k_step_hd: k_step_h's DRAM form (64-env blocks, nt state) with a floor of 7 waves per SIMD on its
// register budget (72 VGPRs, 5 of them spilled, instead of 74-76 and 6 waves). (Round 5: moving the
// step / episode counters to the helper waves removed the spills but cost 13 us at 4M envs -- the
// counters' stores left the step wave's store burst; profiles/r05/step_counters_ab.txt.) More waves keep more
// state bytes in flight where the batch streams from DRAM: 4M envs 250.0-251.6 vs 264.9-265.8 us,
// 8M 511.7-513.0 vs 546.5-547.9; where the Infinity Cache still serves part of it the spills cost
// more than the waves buy (2M 108 vs 95, 3M 161 vs 145; profiles/r04/r4_step_hw7_ab.txt). Same body,
// same bits.
template <int KIND, bool CTBR, bool SPEC>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(7, 8)))
void k_step_hd(float* tiles, const float4* __restrict__ act, uint32_t tile_bytes, int32_t first, int32_t count,
               const KConsts<float>* __restrict__ kc, KParams p, QuadStepOut out) {
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;  // preloaded (see k_step)
  p.kc = kc;
  __shared__ float4 lds[64 * 3];
  __shared__ __attribute__((aligned(16))) float H[HROW * 64];
  __shared__ __attribute__((aligned(16))) float CT[(ct_rows<CTBR>() ? CT_STRIDE : (CTBR ? HCTL : HCTL - 3)) * 64];
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_h_body<KIND, CTBR, 64, true>(K, p, act, out, lds, H, CT);
  } else {
    step_h_body<KIND, CTBR, 64, true>(*kc, p, act, out, lds, H, CT);
  }
}

// k_step: one env per thread. SPEC: the handle's constant block equals the reference default
// (quad_create checks the bytes), so the constants are compiled in -- no scalar loads of the block
// and no waits on them inside the step.
// Kernel-argument preload (csrc/Makefile: -amdgpu-kernarg-preload-count=16): the leading scalar
// arguments -- what the state loads need: tiles, their size, the env range, the actions -- arrive
// in SGPRs at wave launch, so the loads are issued without first waiting on a scalar load of the
// kernarg segment (the KParams / QuadStepOut aggregates behind them are not preloaded).
template <int KIND, bool CTBR, bool SPEC>
__global__ __launch_bounds__(BLOCK) void k_step(float* tiles, const float4* __restrict__ act, uint32_t tile_bytes,
                                                int32_t first, int32_t count, const KConsts<float>* __restrict__ kc,
                                                KParams p, QuadStepOut out) {
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores below (see KParams)
  __shared__ float4 lds[BLOCK * 3];
  __shared__ ResetLds rl;
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_body<KIND, CTBR>(K, p, act, out, lds, rl);
  } else {
    step_body<KIND, CTBR>(*kc, p, act, out, lds, rl);
  }
}


// Config 2 of the scope table -- debug_training.py:111's loop env.step(env.action_space.sample())
// -- as ONE launch: `steps` whole k_step steps per thread with the action of step s drawn in-kernel
// from quad_random_actions' map, Philox(seed; gid, step0 + s, 0x100), and the env state kept in
// registers between steps (read once, written once). Per step every output row goes to HBM as in
// k_step: obs [N,12] through the block's LDS transpose, reward, flags, terminal obs of finishing
// envs, all time-major [steps][N, ...]. Same env_step code as k_step, so the same bits.
template <int KIND, bool CTBR>
__device__ __forceinline__ void step_random_body(const KConsts<float>& K, KParams p, QuadStepOut out,
                                                 float4* __restrict__ act_out, uint32_t step0, int32_t steps,
                                                 float4* lds, ResetLds& rl) {
  const int block_first = blockIdx.x * BLOCK;
  const int n = p.n;
  const bool live = block_first + int(threadIdx.x) < n;
  const int i = live ? block_first + int(threadIdx.x) : n - 1;  // shadow lanes: in-range, store nothing
  EnvRegs<float> e;
  load_env(p, i, e, CTBR);
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  uint32_t ep = S.ldu(F_EP, vo);
  const uint64_t gid = p.gid_base + uint64_t(i);
  for (int t = 0; t < steps; t++) {
    uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), step0 + uint32_t(t), 0x100u};
    philox4x32_10(c, uint32_t(p.seed), uint32_t(p.seed >> 32));
    const float a[4] = {float(c[0] >> 8) * 0x1p-23f - 1.0f, float(c[1] >> 8) * 0x1p-23f - 1.0f,
                        float(c[2] >> 8) * 0x1p-23f - 1.0f, float(c[3] >> 8) * 0x1p-23f - 1.0f};
    StepRes r;
    env_step<float, CTBR>(K, e, a, r);
    const uint32_t row = uint32_t(t) * uint32_t(n) + uint32_t(i);  // time-major row (< 2^32: checked)
    if (live) {
      sto(out.reward, 4u * row, r.reward);
      sto(out.terminated, row, uint8_t(r.term));
      sto(out.truncated, row, uint8_t(r.trunc));
      if (act_out) sto(act_out, 16u * row, make_float4(a[0], a[1], a[2], a[3]));
    }
    float obs[12];
#pragma unroll
    for (int j = 0; j < 12; j++) obs[j] = r.obs[j];
    const bool rs = live && (r.term || r.trunc) && p.auto_reset;
    float u16[16];
    reset_words_wave(p, rl, uint32_t(i), ep, rs, u16);
    if (rs) {
      if (out.terminal_obs) store_row12(out.terminal_obs, row, r.obs);
      float init12[12], tgt[3], s12[12];
      reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
      env_reset_from<float, KIND>(K, e, init12, tgt, obs, s12);
      ep += 1u;
    }
    store_obs_rows(lds, obs, out.obs + size_t(t) * size_t(n) * 12, block_first, n);
    __syncthreads();  // the next step reuses the LDS rows
  }
  if (live) {
    store_env(p, i, e, CTBR);
    S.stu(F_EP, vo, ep);
  }
}

// RB = envs per k_step_random_h block: 64 up to H_SMALL envs (4,096 envs: 2.22 vs 2.40 us per
// step with 256), 256 above (65,536: 3.4 vs 4.5 us with 64); profiles/r02/ab_step_h_block.txt.
// The same with helper waves (see k_step_h): a 512-thread block owns 256 envs; waves 0-3 step them,
// waves 4-7 draw -- two steps ahead -- each env's actions (quad_random_actions' Philox map) into a
// double-buffered LDS slot, and keep each env's next-reset row (k_step_h's image) current: after
// every step they read which envs reset, advance those episode counters and redraw their rows.
// Per step: barrier A (flags known; the image is current) -> resets copied, obs rows staged ->
// barrier B -> obs rows stored by all 512 threads, helpers redraw. Same bits as k_step_random.
template <int KIND, bool CTBR, int RB>
__device__ __forceinline__ void helper_reset_row(const KConsts<float>& K, const KParams& p, int i, uint32_t ep,
                                                 float* H, int l) {
  float u16[16];
#pragma unroll
  for (uint32_t b = 0; b < 4; b++) {
    uint32_t c[4];
    reset_block(p.seed, p.gid_base + uint64_t(i), ep, b, c);
#pragma unroll
    for (int j = 0; j < 4; j++) u16[4 * b + j] = u01(c[j]);
  }
  float init12[12], tgt[3], obs[12], s12[12];
  reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
  EnvRegs<float> e;
  env_reset_from<float, KIND>(K, e, init12, tgt, obs, s12);
  const float row[HROW] = {e.pos[0], e.pos[1], e.pos[2], e.q[0], e.q[1], e.q[2], e.q[3],
                           e.v[0], e.v[1], e.v[2], e.w[0], e.w[1], e.w[2],
                           e.target[0], e.target[1], e.target[2],
                           obs[0], obs[1], obs[2], obs[3], obs[4], obs[5], obs[6], obs[7], obs[8], obs[9],
                           obs[10], obs[11]};
#pragma unroll
  for (int f = 0; f < HROW; f++) H[f * RB + l] = row[f];
}

// a resetting step lane takes its row of the helper image (k_step_h, k_step_random_h)
template <int KIND, int RB>
__device__ __forceinline__ void take_reset_row(const KConsts<float>& K, const float* H, int l, EnvRegs<float>& e,
                                               float obs[12]) {
  float row[HROW];
#pragma unroll
  for (int f = 0; f < HROW; f++) row[f] = H[f * RB + l];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    e.pos[j] = row[j]; e.v[j] = row[7 + j]; e.w[j] = row[10 + j]; e.target[j] = row[13 + j];
    e.rint[j] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) { e.q[j] = row[3 + j]; e.th[j] = 0.f; e.s[j] = 0.f; }
#pragma unroll
  for (int j = 0; j < 12; j++) obs[j] = row[16 + j];
  e.volt = float(K.vnom);
  e.step = 0;
}

__device__ __forceinline__ float4 random_action4(uint64_t seed, uint64_t gid, uint32_t step) {
  uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), step, 0x100u};
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
  return make_float4(float(c[0] >> 8) * 0x1p-23f - 1.0f, float(c[1] >> 8) * 0x1p-23f - 1.0f,
                     float(c[2] >> 8) * 0x1p-23f - 1.0f, float(c[3] >> 8) * 0x1p-23f - 1.0f);
}

template <int KIND, bool CTBR, int RB>
__device__ __forceinline__ void step_random_h_body(const KConsts<float>& K, KParams p, QuadStepOut out,
                                                   float4* __restrict__ act_out, uint32_t step0, int32_t steps,
                                                   float4* lds, float* H, float4* A, uint32_t* R) {
  const int tid = threadIdx.x;
  const int block_first = blockIdx.x * RB;
  const int n = p.n;
  const int l = tid & (RB - 1);
  const bool live = block_first + l < n;
  const int i = live ? block_first + l : n - 1;
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  const uint64_t gid = p.gid_base + uint64_t(i);
  const bool helper = tid >= RB;
  const int nf4 = min(RB, n - block_first) * 3;
  EnvRegs<float> e;
  uint32_t ep = 0;
  if (helper) {
    ep = S.ldu(F_EP, vo);
    A[l] = random_action4(p.seed, gid, step0);
    if (steps > 1) A[RB + l] = random_action4(p.seed, gid, step0 + 1u);
    helper_reset_row<KIND, CTBR, RB>(K, p, i, ep, H, l);
  } else {
    load_env(p, i, e, CTBR);
  }
  __syncthreads();
  for (int t = 0; t < steps; t++) {
    const uint32_t row = uint32_t(t) * uint32_t(n) + uint32_t(i);  // time-major row (< 2^32: checked)
    if (!helper) {
      const float4 a4 = A[(t & 1) * RB + l];
      const float a[4] = {a4.x, a4.y, a4.z, a4.w};
      StepRes r;
      env_step<float, CTBR>(K, e, a, r);
      if (live) {
        sto(out.reward, 4u * row, r.reward);
        sto(out.terminated, row, uint8_t(r.term));
        sto(out.truncated, row, uint8_t(r.trunc));
      }
      float obs[12];
#pragma unroll
      for (int j = 0; j < 12; j++) obs[j] = r.obs[j];
      const bool rs = live && (r.term || r.trunc) && p.auto_reset;
      __syncthreads();  // (A) the image holds every env's next reset
      if (rs) {
        if (out.terminal_obs) store_row12(out.terminal_obs, row, r.obs);
        take_reset_row<KIND, RB>(K, H, l, e, obs);
      }
      R[l] = rs ? 1u : 0u;
      lds[3 * l + 0] = make_float4(obs[0], obs[1], obs[2], obs[3]);
      lds[3 * l + 1] = make_float4(obs[4], obs[5], obs[6], obs[7]);
      lds[3 * l + 2] = make_float4(obs[8], obs[9], obs[10], obs[11]);
      __syncthreads();  // (B) obs rows and reset flags staged
    } else {
      if (act_out && live) sto(act_out, 16u * row, A[(t & 1) * RB + l]);
      __syncthreads();  // (A)
      __syncthreads();  // (B)
      if (R[l]) {  // this env reset at step t: its next episode's row
        ep += 1u;
        helper_reset_row<KIND, CTBR, RB>(K, p, i, ep, H, l);
      }
      if (t + 2 < steps) A[(t & 1) * RB + l] = random_action4(p.seed, gid, step0 + uint32_t(t + 2));
    }
    float4* dst = reinterpret_cast<float4*>(out.obs + (size_t(t) * size_t(n) + size_t(block_first)) * 12);
    for (int idx = tid; idx < nf4; idx += 2 * RB) dst[idx] = lds[idx];
  }
  if (live) {
    if (helper) S.stu(F_EP, vo, ep);
    else store_env(p, i, e, CTBR);
  }
}

template <int KIND, bool CTBR, bool SPEC, int RB>
__global__ __launch_bounds__(2 * RB) void k_step_random_h(const KConsts<float>* __restrict__ kc, KParams p,
                                                             QuadStepOut out, float4* __restrict__ act_out,
                                                             uint32_t step0, int32_t steps) {
  p.kc = kc;
  __shared__ float4 lds[RB * 3];
  __shared__ float H[HROW * RB];
  __shared__ float4 A[2 * RB];
  __shared__ uint32_t R[RB];
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_random_h_body<KIND, CTBR, RB>(K, p, out, act_out, step0, steps, lds, H, A, R);
  } else {
    step_random_h_body<KIND, CTBR, RB>(*kc, p, out, act_out, step0, steps, lds, H, A, R);
  }
}

template <int KIND, bool CTBR, bool SPEC>
__global__ __launch_bounds__(BLOCK) void k_step_random(const KConsts<float>* __restrict__ kc, KParams p,
                                                       QuadStepOut out, float4* __restrict__ act_out,
                                                       uint32_t step0, int32_t steps) {
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
  __shared__ float4 lds[BLOCK * 3];
  __shared__ ResetLds rl;
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_random_body<KIND, CTBR>(K, p, out, act_out, step0, steps, lds, rl);
  } else {
    step_random_body<KIND, CTBR>(*kc, p, out, act_out, step0, steps, lds, rl);
  }
}

// RelPosActWrapper (envs/wrappers.py:13-25) around HoverEnv / TrajectoryFollowEnv: the same step,
// emitting obs7 = [obs[0:3], _prev_action] where _prev_action is the action just taken
// (hover_env.py:166) and zeros after a reset (:212). The previous action is kept in the SoA
// (F_PREV) so quad_observe / get_state stay exact. CTBR: RelPosActWrapper(RateControlWrapper(env))
// -- the action is the rate command the controller maps to torques, and it is also what the
// obs7 carries (rate_wrapper.py:100-106 overwrites _prev_action with it after the base step).
template <int KIND, bool CTBR>
__global__ __launch_bounds__(BLOCK) void k_step_relpos(const KConsts<float>* __restrict__ kc, KParams p,
                                                       const float4* __restrict__ act, QuadStepOut out) {
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
  const int i = p.first + blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.first + p.count) return;
  EnvRegs<float> e;
  load_env(p, i, e, CTBR);
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  const uint32_t ep = S.ldu(F_EP, vo);
  const float4 a4 = act[i];
  const float a[4] = {a4.x, a4.y, a4.z, a4.w};
  StepRes r;
  env_step<float, CTBR>(*p.kc, e, a, r);
  float info[9];
  if (out.target_info) target_info_of<KIND>(*p.kc, p, i, e, ep, info);
  float o7[7] = {r.obs[0], r.obs[1], r.obs[2], a[0], a[1], a[2], a[3]};
  float prev[4] = {a[0], a[1], a[2], a[3]};
  const bool rs = (r.term || r.trunc) && p.auto_reset;
  float obs12[12];
  if (rs) reset_env<KIND>(p, i, e, obs12, ep);
  // ---- outputs (k_step_relpos keeps them after the reset: its 7-wide rows need o7 either way)
  out.reward[i] = r.reward;
  out.terminated[i] = r.term;
  out.truncated[i] = r.trunc;
  if (out.motor_commands)
    reinterpret_cast<float4*>(out.motor_commands)[i] = make_float4(r.motor[0], r.motor[1], r.motor[2], r.motor[3]);
  if (out.voltage_scale) out.voltage_scale[i] = r.vscale;
  if (out.state12) {
#pragma unroll
    for (int j = 0; j < 12; j++) out.state12[size_t(i) * 12 + j] = r.state12[j];
  }
  if (out.target_info) store_target_info(out.target_info, i, info);
  if (rs) {
    if (out.terminal_obs) {
#pragma unroll
      for (int j = 0; j < 7; j++) out.terminal_obs[size_t(i) * 7 + j] = o7[j];
    }
    S.stu(F_EP, vo, ep + 1u);
    o7[0] = obs12[0]; o7[1] = obs12[1]; o7[2] = obs12[2];
#pragma unroll
    for (int j = 0; j < 4; j++) { o7[3 + j] = 0.f; prev[j] = 0.f; }
  }
  store_env(p, i, e, CTBR);
#pragma unroll
  for (int j = 0; j < 4; j++) S.st(F_PREV + j, vo, prev[j]);
#pragma unroll
  for (int j = 0; j < 7; j++) out.obs[size_t(i) * 7 + j] = o7[j];
}

// ---------------------------------------------------------------------------------------------
// k_step_g<KIND, CTBR, G>: the step with one env per GROUP of G lanes (G = 1, 2, 4; 64/G envs
// per wave). Work that is a loop over 4 items in the one-thread form -- the props (hinge state and
// inertia-box drag), the three atan2 of scipy's Euler algorithm, the four obs triples, the four
// Philox blocks of the reset draw, the three half-angle sincos of from_euler -- is spread over the
// group (lane l takes items l, l+G, ...); the rest is evaluated by every lane of the group (one
// wave-instruction either way). Group reductions / broadcasts are DPP quad_perm (quad_lanes.h).
// Why: at 65,536 envs the G = 1 form is one lone wave per SIMD (issue-latency bound); G > 1 buys
// waves per SIMD at the price of the replicated part -- see DESIGN.md "Lane groups".
template <int G, typename T>
__device__ __forceinline__ T grp_pick(int m, const T* v) {  // v[m], m lane-dependent, m < 4
  return pick4(m, v[0], v[1], v[2], v[3]);
}

template <int KIND, bool CTBR, int G>
__device__ __forceinline__ void step_g_body(const KConsts<float>& k, KParams p, const float4* __restrict__ act,
                                            QuadStepOut out) {
  constexpr int NI = 4 / G;  // items per lane
  const unsigned i_raw = unsigned(p.first) + (blockIdx.x * BLOCK + threadIdx.x) / G;
  const int l = G == 1 ? 0 : int(threadIdx.x & (G - 1));
  // G > 1: whole groups leave together. G = 1 keeps every thread (the LDS obs stage has a
  // block barrier); out-of-range threads recompute the last env and store nothing.
  const unsigned end = unsigned(p.first + p.count);
  if (G > 1 && i_raw >= end) return;
  const bool live = i_raw < end;
  const unsigned i = live ? i_raw : end - 1;
  const PhysConsts<float>& c = k.ph;
  const Tiles S(p);
  const uint32_t vo = env_off(i);
  // ---- load: shared fields by every lane; per-prop / per-axis fields by their owner lane
  float pos[3], q[4], v[3], w[3], tgt[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    pos[j] = S.ld(F_QPOS + j, vo);
    v[j] = S.ld(F_QVEL + j, vo);
    w[j] = S.ld(F_QVEL + 3 + j, vo);
    tgt[j] = S.ld(F_TGT + j, vo);
  }
#pragma unroll
  for (int j = 0; j < 4; j++) q[j] = S.ld(F_QPOS + 3 + j, vo);
  float volt = S.ld(F_VOLT, vo);
  int step = int(S.ldu(F_STEP, vo));
  const uint32_t ep = S.ldu(F_EP, vo);  // prefetched: the reset branch must not add a dependent load
  float th[NI], sp[NI];
#pragma unroll
  for (int it = 0; it < NI; it++) {
    const int pr = l + it * G;
    th[it] = G == 1 ? S.ld(F_QPOS + 7 + pr, vo) : S.ldv(F_QPOS + 7 + pr, vo);
    sp[it] = G == 1 ? S.ld(F_QVEL + 6 + pr, vo) : S.ldv(F_QVEL + 6 + pr, vo);
  }
  float ri[3] = {0.f, 0.f, 0.f};
  if (CTBR) {
#pragma unroll
    for (int j = 0; j < 3; j++) ri[j] = S.ld(F_RINT + j, vo);
  }
  const float4 a4 = act[i];
  float a[4] = {a4.x, a4.y, a4.z, a4.w};

  // ---- RateControlWrapper.action (float64): three axes, every lane (cheap, no reduction)
  if (CTBR) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const double err = double(a[1 + j]) * k.rate_max - double(w[j]);
      const double rid = clipn(double(ri[j]) + k.rate_kidt * err, -k.rate_imax, k.rate_imax);
      ri[j] = float(rid);
      a[1 + j] = float(clipn((k.rate_ikd[j] * err + rid) * k.r_max_torque, -1.0, 1.0));
    }
  }
  // ---- denormalize (float32) -> mixer, voltage sag, motor wrench (float64)
  double phys[4];
#pragma unroll
  for (int j = 0; j < 4; j++) phys[j] = double(denorm1(a[j], k.act_lo[j], k.act_span[j]));
  double F[4];
#pragma unroll
  for (int r = 0; r < 4; r++)
    F[r] = clipn(c.mix[4 * r] * phys[0] + c.mix[4 * r + 1] * phys[1] + c.mix[4 * r + 2] * phys[2] +
                     c.mix[4 * r + 3] * phys[3], 0.0, k.max_thrust);
  const double vs = clipn(double(volt) * k.r_vnom, 0.0, 1.0);
#pragma unroll
  for (int r = 0; r < 4; r++) F[r] = clipn(F[r] * vs, 0.0, k.max_thrust * vs);
  volt = float(clipn(double(volt) - (k.vb + k.vl * (((F[0] + F[1] + F[2] + F[3]) * 0.25) * k.r_mx)) * k.dt,
                     k.vmin, k.vnom));
  // ---- mujoco.mj_step: mj_checkPos/Vel, bad ctrl
  int bad = 0;
#pragma unroll
  for (int it = 0; it < NI; it++) bad |= int(isbad(th[it])) | int(isbad(sp[it]));
#pragma unroll
  for (int j = 0; j < 3; j++) bad |= int(isbad(pos[j])) | int(isbad(v[j])) | int(isbad(w[j]));
#pragma unroll
  for (int j = 0; j < 4; j++) bad |= int(isbad(q[j]));
  bad = group_or<G>(bad);
  int badctrl = bad;
#pragma unroll
  for (int r = 0; r < 4; r++) badctrl |= int(isbad(F[r]));
  if (bad) {
#pragma unroll
    for (int j = 0; j < 3; j++) { pos[j] = 0.f; v[j] = 0.f; w[j] = 0.f; }
    q[0] = 1.f; q[1] = q[2] = q[3] = 0.f;
#pragma unroll
    for (int it = 0; it < NI; it++) { th[it] = 0.f; sp[it] = 0.f; }
  }
  double Fc[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const double f = badctrl ? 0.0 : F[r];
    Fc[r] = f < c.ctrl_lo ? c.ctrl_lo : (f > c.ctrl_hi ? c.ctrl_hi : f);
  }
  // ---- forward dynamics (forward_acc in quad_physics.h, props spread over the group)
  float qn[4] = {q[0], q[1], q[2], q[3]};
  normalize4(qn);
  float R[9];
  {
    const float qw = qn[0], qx = qn[1], qy = qn[2], qz = qn[3];
    R[0] = 1.f - 2.f * (qy * qy + qz * qz); R[1] = 2.f * (qx * qy - qw * qz); R[2] = 2.f * (qx * qz + qw * qy);
    R[3] = 2.f * (qx * qy + qw * qz); R[4] = 1.f - 2.f * (qx * qx + qz * qz); R[5] = 2.f * (qy * qz - qw * qx);
    R[6] = 2.f * (qx * qz - qw * qy); R[7] = 2.f * (qy * qz + qw * qx); R[8] = 1.f - 2.f * (qx * qx + qy * qy);
  }
  float vB[3];
#pragma unroll
  for (int j = 0; j < 3; j++) vB[j] = R[j] * v[0] + R[3 + j] * v[1] + R[6 + j] * v[2];
  float FB[3] = {0.f, 0.f, 0.f}, tau[3] = {0.f, 0.f, 0.f}, Qs[NI], Qloc = 0.f, sloc = 0.f;
#pragma unroll
  for (int it = 0; it < NI; it++) {
    const int pr = l + it * G;
    const float pc[3] = {G == 1 ? c.pc[it][0] : pick4(pr, c.pc[0][0], c.pc[1][0], c.pc[2][0], c.pc[3][0]),
                         G == 1 ? c.pc[it][1] : pick4(pr, c.pc[0][1], c.pc[1][1], c.pc[2][1], c.pc[3][1]),
                         G == 1 ? c.pc[it][2] : pick4(pr, c.pc[0][2], c.pc[1][2], c.pc[2][2], c.pc[3][2])};
    float sn, cs;
    q_sincos(th[it], &sn, &cs);
    float wxc[3];
    cross(w, pc, wxc);
    const float ub[3] = {vB[0] + wxc[0], vB[1] + wxc[1], vB[2] + wxc[2]};
    const float wp[3] = {cs * w[0] + sn * w[1], -sn * w[0] + cs * w[1], w[2] + sp[it]};
    const float up[3] = {cs * ub[0] + sn * ub[1], -sn * ub[0] + cs * ub[1], ub[2]};
    float tp[3], fp[3];
    box_drag(wp, up, c.p_kqa, c.p_kva, c.p_kql, c.p_kvl, tp, fp);
    const float f[3] = {cs * fp[0] - sn * fp[1], sn * fp[0] + cs * fp[1], fp[2]};
    const float t[3] = {cs * tp[0] - sn * tp[1], sn * tp[0] + cs * tp[1], tp[2]};
    float rxf[3];
    cross(pc, f, rxf);
#pragma unroll
    for (int j = 0; j < 3; j++) { FB[j] += f[j]; tau[j] += rxf[j] + t[j]; }
    Qs[it] = tp[2];
    Qloc += tp[2];
    sloc += sp[it];
  }
#pragma unroll
  for (int j = 0; j < 3; j++) { FB[j] = group_sum<G>(FB[j]); tau[j] = group_sum<G>(tau[j]); }
  const float Qsum = group_sum<G>(Qloc), ssum = group_sum<G>(sloc);
  {  // motor wrench (float64 -> float32), gravity at the system COM, base inertia-box drag
    FB[2] += float(Fc[0] + Fc[1] + Fc[2] + Fc[3]);
    tau[0] += float(c.syd[0] * Fc[0] + c.syd[1] * Fc[1] + c.syd[2] * Fc[2] + c.syd[3] * Fc[3]);
    tau[1] += float(-(c.sxd[0] * Fc[0] + c.sxd[1] * Fc[1] + c.sxd[2] * Fc[2] + c.sxd[3] * Fc[3]));
    tau[2] += float(c.g5d[0] * Fc[0] + c.g5d[1] * Fc[1] + c.g5d[2] * Fc[2] + c.g5d[3] * Fc[3]);
    const float mg = c.mt * c.gz;
    const float gB[3] = {mg * R[6], mg * R[7], mg * R[8]};
    float tg[3];
    cross(c.cbar, gB, tg);
    float tb[3], fb[3];
    box_drag(w, vB, c.b_kqa, c.b_kva, c.b_kql, c.b_kvl, tb, fb);
#pragma unroll
    for (int j = 0; j < 3; j++) { FB[j] += gB[j] + fb[j]; tau[j] += tg[j] + tb[j]; }
  }
  float vdot[3], wdot[3], sdot[NI];
  {
    float wc[3], wwc[3], fv[3], Iw[3], wIw[3], cxf[3], rhs[3], cxw[3], aB[3];
    cross(w, c.cbar, wc);
    cross(w, wc, wwc);
#pragma unroll
    for (int j = 0; j < 3; j++) fv[j] = FB[j] - c.mt * wwc[j];
#pragma unroll
    for (int j = 0; j < 3; j++) Iw[j] = c.IO[3 * j] * w[0] + c.IO[3 * j + 1] * w[1] + c.IO[3 * j + 2] * w[2];
    cross(w, Iw, wIw);
    cross(c.cbar, fv, cxf);
    rhs[0] = tau[0] - wIw[0] - c.c_ax * ssum * w[1] - cxf[0];
    rhs[1] = tau[1] - wIw[1] + c.c_ax * ssum * w[0] - cxf[1];
    rhs[2] = tau[2] - wIw[2] - Qsum - cxf[2];
#pragma unroll
    for (int j = 0; j < 3; j++) wdot[j] = c.Ainv[3 * j] * rhs[0] + c.Ainv[3 * j + 1] * rhs[1] + c.Ainv[3 * j + 2] * rhs[2];
    cross(c.cbar, wdot, cxw);
#pragma unroll
    for (int j = 0; j < 3; j++) aB[j] = fv[j] * c.inv_mt + cxw[j];
#pragma unroll
    for (int j = 0; j < 3; j++) vdot[j] = R[3 * j] * aB[0] + R[3 * j + 1] * aB[1] + R[3 * j + 2] * aB[2];
#pragma unroll
    for (int it = 0; it < NI; it++) sdot[it] = Qs[it] * c.inv_c_ax - wdot[2];
  }
  {  // mj_checkAcc: reset to qpos0; at rest there qacc is free fall
    int badacc = 0;
#pragma unroll
    for (int it = 0; it < NI; it++) badacc |= int(isbad(sdot[it]));
#pragma unroll
    for (int j = 0; j < 3; j++) badacc |= int(isbad(vdot[j])) | int(isbad(wdot[j]));
    if (group_or<G>(badacc)) {
#pragma unroll
      for (int j = 0; j < 3; j++) { pos[j] = 0.f; v[j] = 0.f; w[j] = 0.f; vdot[j] = 0.f; wdot[j] = 0.f; }
      vdot[2] = c.gz;
      qn[0] = 1.f; qn[1] = qn[2] = qn[3] = 0.f;
#pragma unroll
      for (int it = 0; it < NI; it++) { th[it] = 0.f; sp[it] = 0.f; sdot[it] = 0.f; }
    }
  }
  // ---- mj_Euler: semi-implicit update, MuJoCo quaternion integration
  const float h = c.dt;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    v[j] += h * vdot[j];
    w[j] += h * wdot[j];
    pos[j] += h * v[j];
  }
#pragma unroll
  for (int it = 0; it < NI; it++) {
    sp[it] += h * sdot[it];
    th[it] += h * sp[it];
  }
  {
    const float w2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const float x2 = 0.25f * h * h * w2;
    float qr[4];
    if (x2 < 0.0625f) {
      const float ch = 1.f + x2 * (-0.5f + x2 * (1.f / 24 + x2 * (-1.f / 720 + x2 * (1.f / 40320))));
      const float sc = 1.f + x2 * (-1.f / 6 + x2 * (1.f / 120 + x2 * (-1.f / 5040 + x2 * (1.f / 362880))));
      const float kk = 0.5f * h * sc;
      qr[0] = ch; qr[1] = w[0] * kk; qr[2] = w[1] * kk; qr[3] = w[2] * kk;
    } else {
      const float wn = fsqrt(w2);
      float sh, chh;
      q_sincos(0.5f * h * wn, &sh, &chh);
      const float kk = sh / wn;
      qr[0] = chh; qr[1] = w[0] * kk; qr[2] = w[1] * kk; qr[3] = w[2] * kk;
    }
    q[0] = qn[0] * qr[0] - qn[1] * qr[1] - qn[2] * qr[2] - qn[3] * qr[3];
    q[1] = qn[0] * qr[1] + qn[1] * qr[0] + qn[2] * qr[3] - qn[3] * qr[2];
    q[2] = qn[0] * qr[2] - qn[1] * qr[3] + qn[2] * qr[0] + qn[3] * qr[1];
    q[3] = qn[0] * qr[3] + qn[1] * qr[2] - qn[2] * qr[1] + qn[3] * qr[0];
  }
  step += 1;
  // ---- QuadState (scipy as_euler('xyz')): items 0,1,2 = mid, half_sum, half_diff atan2
  float s12[12];
  {
    const float inv = frsqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const float qw = q[0] * inv, qx = q[1] * inv, qy = q[2] * inv, qz = q[3] * inv;
    const float A = qw - qy, B = qx + qz, Cc = qy + qw, D = qz - qx;
    const float ys[4] = {q_hypot(Cc, D), B, D, D};
    const float xs[4] = {q_hypot(A, B), A, Cc, Cc};
    float at[3];
    if constexpr (G == 1) {
#pragma unroll
      for (int m = 0; m < 3; m++) at[m] = q_atan2(ys[m], xs[m]);
    } else if constexpr (G == 2) {
      const float r0 = q_atan2(l ? ys[1] : ys[0], l ? xs[1] : xs[0]);  // items 0 | 1
      const float r1 = q_atan2(ys[2], xs[2]);                           // item 2 (both lanes)
      at[0] = group_bc<G, 0>(r0); at[1] = group_bc<G, 1>(r0); at[2] = r1;
    } else {
      const float r = q_atan2(grp_pick<G>(l, ys), grp_pick<G>(l, xs));
      at[0] = group_bc<G, 0>(r); at[1] = group_bc<G, 1>(r); at[2] = group_bc<G, 2>(r);
    }
    const float PI = 3.14159265358979323846f;
    const float mid = 2.f * at[0], hs = at[1], hd = at[2];
    const bool case1 = fabsf(mid) <= 1e-7f, case2 = fabsf(mid - PI) <= 1e-7f;
    float e[3];
    if (!(case1 || case2)) { e[0] = hs - hd; e[2] = hs + hd; }
    else { e[2] = 0.f; e[0] = case1 ? 2.f * hs : -2.f * hd; }
    e[1] = mid - PI / 2.f;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      if (e[j] < -PI) e[j] += 2.f * PI;
      else if (e[j] > PI) e[j] -= 2.f * PI;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) { s12[j] = pos[j]; s12[3 + j] = e[j]; s12[6 + j] = v[j]; s12[9 + j] = w[j]; }
  }
  const float reward = reward_of<float>(s12, tgt);
  const bool term = terminated_of(k, s12);
  const bool trunc = step >= k.max_steps;
  // obs triples m = l + it*G (normalize, float32, correctly rounded)
  float ob[NI][3];
  auto obs_triples = [&](const float* st, const float* tg3) {
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int m = l + it * G;
#pragma unroll
      for (int j = 0; j < 3; j++) {
        float x, lo, sp_, rs;
        if constexpr (G == 1) {
          x = st[3 * it + j]; lo = k.obs_lo[3 * it + j]; sp_ = k.obs_span[3 * it + j]; rs = k.obs_rspan[3 * it + j];
        } else {
          x = pick4(m, st[j], st[3 + j], st[6 + j], st[9 + j]);
          lo = pick4(m, k.obs_lo[j], k.obs_lo[3 + j], k.obs_lo[6 + j], k.obs_lo[9 + j]);
          sp_ = pick4(m, k.obs_span[j], k.obs_span[3 + j], k.obs_span[6 + j], k.obs_span[9 + j]);
          rs = pick4(m, k.obs_rspan[j], k.obs_rspan[3 + j], k.obs_rspan[6 + j], k.obs_rspan[9 + j]);
        }
        if (m == 0) x = sub32(tg3[j], x);
        ob[it][j] = norm_obs1(x, lo, sp_, rs);
      }
    }
  };
  obs_triples(s12, tgt);
  settle(ep);
  if (l == 0 && live) {
    out.reward[i] = reward;
    out.terminated[i] = term;
    out.truncated[i] = trunc;
    if (out.voltage_scale) out.voltage_scale[i] = float(vs);
    if (out.motor_commands)
      reinterpret_cast<float4*>(out.motor_commands)[i] = make_float4(float(F[0]), float(F[1]), float(F[2]), float(F[3]));
  }
  if (G == 1 && out.state12 && live) {
    store_row12(out.state12, i, s12);
  } else if (out.state12 && live) {
#pragma unroll
    for (int it = 0; it < NI; it++) {
      const int m = l + it * G;
#pragma unroll
      for (int j = 0; j < 3; j++)
        out.state12[size_t(i) * 12 + 3 * m + j] = G == 1 ? s12[3 * it + j] : pick4(m, s12[j], s12[3 + j], s12[6 + j], s12[9 + j]);
    }
  }
  if (out.target_info && live && l == 0) {  // info target (+ spline velocity / acceleration)
    float o[9] = {tgt[0], tgt[1], tgt[2], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (KIND == QUAD_ENV_TRAJ) traj_spline_info(k, p.seed, p.gid_base + uint64_t(i), ep - 1u, tgt, step, o);
#pragma unroll
    for (int j = 0; j < 9; j++) out.target_info[size_t(i) * 9 + j] = o[j];
  }
  // ---- SB3 auto-reset (group-uniform branch)
  const bool reset = (term || trunc) && p.auto_reset;
  if (reset) {
    if (out.terminal_obs && live) {
      if constexpr (G == 1) {
        const float o12[12] = {ob[0][0], ob[0][1], ob[0][2], ob[1][0], ob[1][1], ob[1][2],
                               ob[2][0], ob[2][1], ob[2][2], ob[3][0], ob[3][1], ob[3][2]};
        store_row12(out.terminal_obs, i, o12);
      } else {
#pragma unroll
        for (int it = 0; it < NI; it++)
#pragma unroll
          for (int j = 0; j < 3; j++) out.terminal_obs[size_t(i) * 12 + 3 * (l + it * G) + j] = ob[it][j];
      }
    }
    const uint64_t gid = p.gid_base + uint64_t(i);
    uint32_t r[NI][4];
#pragma unroll
    for (int it = 0; it < NI; it++) {  // Philox blocks l, l+G, ...
      r[it][0] = uint32_t(gid); r[it][1] = uint32_t(gid >> 32); r[it][2] = ep; r[it][3] = uint32_t(l + it * G);
      philox4x32_10(r[it], uint32_t(p.seed), uint32_t(p.seed >> 32));
    }
    uint32_t wd[15];  // word j of the 16-word draw lives in block j/4 -> lane (j/4)%G, item (j/4)/G
#define QD_W(J) wd[J] = group_bcu<G, ((J) / 4) % G>(r[((J) / 4) / G][(J) % 4]);
    QD_W(0) QD_W(1) QD_W(2) QD_W(3) QD_W(4) QD_W(5) QD_W(6) QD_W(7)
    QD_W(8) QD_W(9) QD_W(10) QD_W(11) QD_W(12) QD_W(13) QD_W(14)
#undef QD_W
    float init12[12], tg[3];
#pragma unroll
    for (int j = 0; j < 12; j++) init12[j] = affine32(k.init_lo[j], u01(wd[j]), k.init_span[j]);
#pragma unroll
    for (int j = 0; j < 3; j++) tg[j] = affine32(k.tgt_lo[j], u01(wd[12 + j]), k.tgt_span[j]);
    // from_euler: half-angle sincos of axes 0..2 spread over the group
    float hsn[3], hcs[3];
    if constexpr (G == 1) {
#pragma unroll
      for (int m = 0; m < 3; m++) q_sincos(init12[3 + m] * 0.5f, &hsn[m], &hcs[m]);
    } else if constexpr (G == 2) {
      float s0, c0;
      q_sincos((l ? init12[4] : init12[3]) * 0.5f, &s0, &c0);
      q_sincos(init12[5] * 0.5f, &hsn[2], &hcs[2]);
      hsn[0] = group_bc<G, 0>(s0); hcs[0] = group_bc<G, 0>(c0);
      hsn[1] = group_bc<G, 1>(s0); hcs[1] = group_bc<G, 1>(c0);
    } else {
      float s0, c0;
      q_sincos(pick4(l, init12[3], init12[4], init12[5], init12[5]) * 0.5f, &s0, &c0);
      hsn[0] = group_bc<G, 0>(s0); hcs[0] = group_bc<G, 0>(c0);
      hsn[1] = group_bc<G, 1>(s0); hcs[1] = group_bc<G, 1>(c0);
      hsn[2] = group_bc<G, 2>(s0); hcs[2] = group_bc<G, 2>(c0);
    }
    {
      const float sr = hsn[0], cr = hcs[0], spp = hsn[1], cp = hcs[1], sy = hsn[2], cy = hcs[2];
      q[0] = cy * cp * cr + sy * spp * sr;
      q[1] = cy * cp * sr - sy * spp * cr;
      q[2] = cy * spp * cr + sy * cp * sr;
      q[3] = sy * cp * cr - cy * spp * sr;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) {
      pos[j] = init12[j];
      v[j] = init12[6 + j];
      w[j] = init12[9 + j];
      tgt[j] = KIND == QUAD_ENV_TRAJ ? init12[j] : tg[j];
      ri[j] = 0.f;
    }
#pragma unroll
    for (int it = 0; it < NI; it++) { th[it] = 0.f; sp[it] = 0.f; }
    volt = float(k.vnom);
    step = 0;
    obs_triples(init12, tgt);  // QuadState round trip of the drawn state == the draw itself
    if (l == 0 && live) S.stu(F_EP, vo, ep + 1u);
  }
  // ---- stores: obs rows. G = 1: staged through LDS so every wave-store writes 1 KiB
  // contiguously; G > 1: one dwordx3 per lane, a wave's rows are already contiguous.
  if constexpr (G == 1) {
    __shared__ float4 lds[BLOCK * 3];
    const float o12[12] = {ob[0][0], ob[0][1], ob[0][2], ob[1][0], ob[1][1], ob[1][2],
                           ob[2][0], ob[2][1], ob[2][2], ob[3][0], ob[3][1], ob[3][2]};
    store_obs_rows(lds, o12, out.obs, p.first + int(blockIdx.x) * BLOCK, int(end));
  } else {
#pragma unroll
    for (int it = 0; it < NI; it++) {
      float* o = out.obs + size_t(i) * 12 + 3 * (l + it * G);
      o[0] = ob[it][0]; o[1] = ob[it][1]; o[2] = ob[it][2];
    }
  }
  if (!live) return;
#pragma unroll
  for (int it = 0; it < NI; it++) {
    const int pr = l + it * G;
    if (G == 1) {
      S.st(F_QPOS + 7 + pr, vo, th[it]);
      S.st(F_QVEL + 6 + pr, vo, sp[it]);
    } else {
      S.stv(F_QPOS + 7 + pr, vo, th[it]);
      S.stv(F_QVEL + 6 + pr, vo, sp[it]);
    }
  }
  if (l == 0) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      S.st(F_QPOS + j, vo, pos[j]);
      S.st(F_QVEL + j, vo, v[j]);
      S.st(F_QVEL + 3 + j, vo, w[j]);
      if (reset) S.st(F_TGT + j, vo, tgt[j]);  // the target only changes on reset
      if (CTBR) S.st(F_RINT + j, vo, ri[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) S.st(F_QPOS + 3 + j, vo, q[j]);
    S.st(F_VOLT, vo, volt);
    S.stu(F_STEP, vo, uint32_t(step));
  }
}

// QD_G_WAVES (A/B builds of tools/probe/build_variant.sh only): a minimum waves-per-SIMD target
#if defined(QD_G_WAVES)
#define QD_G_ATTR __attribute__((amdgpu_waves_per_eu(QD_G_WAVES, 8)))
#else
#define QD_G_ATTR
#endif
template <int KIND, bool CTBR, int G, bool SPEC>
__global__ __launch_bounds__(BLOCK) QD_G_ATTR void k_step_g(float* tiles, const float4* __restrict__ act, uint32_t tile_bytes,
                                                  int32_t first, int32_t count, const KConsts<float>* __restrict__ kc,
                                                  KParams p, QuadStepOut out) {
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;  // preloaded (see k_step)
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
  if constexpr (SPEC) {
    constexpr KConsts<float> K = kdef_block<KIND, CTBR>();
    step_g_body<KIND, CTBR, G>(K, p, act, out);
  } else {
    step_g_body<KIND, CTBR, G>(*kc, p, act, out);
  }
}

template <int KIND, bool RELPOS>
__global__ __launch_bounds__(BLOCK) void k_reset(KParams p, const uint8_t* __restrict__ mask,
                                                 float* __restrict__ obs_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  if (mask && !mask[i]) return;
  EnvRegs<float> e;
  float obs[12];
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  const uint32_t ep = S.ldu(F_EP, vo);
  reset_env<KIND>(p, i, e, obs, ep);
  S.stu(F_EP, vo, ep + 1u);
  store_env(p, i, e, true);
#pragma unroll
  for (int j = 0; j < 4; j++) S.st(F_PREV + j, vo, 0.f);  // hover_env.py:212
  if (obs_out) {
    if (RELPOS) {
#pragma unroll
      for (int j = 0; j < 7; j++) obs_out[size_t(i) * 7 + j] = j < 3 ? obs[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 12; j++) obs_out[size_t(i) * 12 + j] = obs[j];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// brax kinds: one thread per env (obs rows are 84 B, written directly). Auto-reset follows brax's
// AutoResetWrapper: the env returns to the FIRST state of its episode -- regenerated from the draw
// of the last explicit reset (episode counter - 1) instead of being stored.
template <int KIND>
__global__ __launch_bounds__(BLOCK) void k_step_brax(const KConsts<float>* __restrict__ kc, KParams p,
                                                     const float4* __restrict__ act, QuadStepOut out) {
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
  const int i = p.first + blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.first + p.count) return;
  EnvRegs<float> e;
  load_env(p, i, e, true);
  const float4 a4 = act[i];
  const float a[4] = {a4.x, a4.y, a4.z, a4.w};
  float obs[21], reward, motor[4];
  bool term, trunc;
  brax_step<float, KIND>(*p.kc, e, a, obs, reward, term, trunc, motor);
  out.reward[i] = reward;
  out.terminated[i] = term;
  out.truncated[i] = trunc;
  if (out.motor_commands)
    reinterpret_cast<float4*>(out.motor_commands)[i] = make_float4(motor[0], motor[1], motor[2], motor[3]);
  if (out.voltage_scale) out.voltage_scale[i] = 1.0f;
  if (out.target_info) {
#pragma unroll
    for (int j = 0; j < 9; j++) out.target_info[size_t(i) * 9 + j] = j < 3 ? e.target[j] : 0.f;
  }
  if ((term || trunc) && p.auto_reset) {
    if (out.terminal_obs) {
#pragma unroll
      for (int j = 0; j < 21; j++) out.terminal_obs[size_t(i) * 21 + j] = obs[j];
    }
    float u21[21];
    brax_reset_draw(p.kc->bx_noise, p.seed, p.gid_base + uint64_t(i),
                    Tiles(p).ldu(F_EP, env_off(uint32_t(i))) - 1u, u21);
    brax_reset_from<float, KIND>(*p.kc, e, u21, obs, true);
  }
  store_env(p, i, e, true);
#pragma unroll
  for (int j = 0; j < 21; j++) out.obs[size_t(i) * 21 + j] = obs[j];
}

template <int KIND>
__global__ __launch_bounds__(BLOCK) void k_reset_brax(KParams p, const uint8_t* __restrict__ mask,
                                                      float* __restrict__ obs_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  if (mask && !mask[i]) return;
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  const uint32_t ep = S.ldu(F_EP, vo);
  float u21[21], obs[21];
  brax_reset_draw(p.kc->bx_noise, p.seed, p.gid_base + uint64_t(i), ep, u21);
  EnvRegs<float> e;
  brax_reset_from<float, KIND>(*p.kc, e, u21, obs, false);
  S.stu(F_EP, vo, ep + 1u);
  store_env(p, i, e, true);
  if (obs_out) {
#pragma unroll
    for (int j = 0; j < 21; j++) obs_out[size_t(i) * 21 + j] = obs[j];
  }
}

__global__ __launch_bounds__(BLOCK) void k_observe_brax(KParams p, float* __restrict__ obs_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
#pragma unroll
  for (int j = 0; j < 21; j++) obs_out[size_t(i) * 21 + j] = S.ld(F_QPOS + j, vo);  // qpos, qvel
}

template <bool RELPOS>
__global__ __launch_bounds__(BLOCK) void k_observe(KParams p, float* __restrict__ obs_out,
                                                   float* __restrict__ s12_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  EnvRegs<float> e;
  load_env(p, i, e, false);
  float obs[12], s12[12];
  observe(*p.kc, e, obs, s12);
  if (RELPOS) {
#pragma unroll
    for (int j = 0; j < 7; j++)
      obs_out[size_t(i) * 7 + j] = j < 3 ? obs[j] : Tiles(p).ld(F_PREV + j - 3, env_off(uint32_t(i)));
  } else {
#pragma unroll
    for (int j = 0; j < 12; j++) obs_out[size_t(i) * 12 + j] = obs[j];
  }
  if (s12_out) {
#pragma unroll
    for (int j = 0; j < 12; j++) s12_out[size_t(i) * 12 + j] = s12[j];
  }
}

// HoverEnv._is_terminated (hover_env.py:150-157) on caller-given absolute 12-D states: the step
// kernels' own predicate (terminated_of), bounds from the handle's constants
__global__ __launch_bounds__(BLOCK) void k_terminated(const KConsts<float>* __restrict__ kc,
                                                      const float* __restrict__ s12, int32_t n,
                                                      uint8_t* __restrict__ out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  float s[12];
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = s12[size_t(i) * 12 + j];
  out[i] = terminated_of(*kc, s) ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// batched waypoint evaluation (evaluate.py:440-612)
template <bool RELPOS>
__global__ __launch_bounds__(BLOCK) void k_waypoints_begin(KParams p, QuadWaypoints w, QuadWaypointState t,
                                                           float* __restrict__ obs_out) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  const int set = w.set_of ? w.set_of[i] : 0;
  const int cnt = w.counts[set];
  const double* wp = w.points + size_t(set) * w.max_points * 3;
  const int nxt = 1 % cnt;
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
#pragma unroll
  for (int j = 0; j < 3; j++) {
    S.st(F_QPOS + j, vo, float(wp[j]));
    S.st(F_QVEL + j, vo, 0.f);
    S.st(F_QVEL + 3 + j, vo, 0.f);
    S.st(F_TGT + j, vo, float(wp[3 * nxt + j]));  // waypoints[i].astype(np.float32)
    S.st(F_RINT + j, vo, 0.f);
  }
  S.st(F_QPOS + 3, vo, 1.f);
  S.st(F_QPOS + 4, vo, 0.f);
  S.st(F_QPOS + 5, vo, 0.f);
  S.st(F_QPOS + 6, vo, 0.f);
  S.stu(F_STEP, vo, 0u);
  t.wp_idx[i] = nxt;
  t.reached[i] = 0;
  t.laps[i] = 0;
  t.steps[i] = 0;
  t.status[i] = 0;
  t.total_reward[i] = 0.0;
  EnvRegs<float> e;
  load_env(p, i, e, false);
  float obs[12], s12[12];
  observe(*p.kc, e, obs, s12);
  if (RELPOS) {
#pragma unroll
    for (int j = 0; j < 7; j++) obs_out[size_t(i) * 7 + j] = j < 3 ? obs[j] : S.ld(F_PREV + j - 3, vo);
  } else {
#pragma unroll
    for (int j = 0; j < 12; j++) obs_out[size_t(i) * 12 + j] = obs[j];
  }
}

__global__ __launch_bounds__(BLOCK) void k_waypoints_update(KParams p, QuadWaypoints w, QuadWaypointState t,
                                                            const float* __restrict__ s12,
                                                            const float* __restrict__ rew,
                                                            const uint8_t* __restrict__ term,
                                                            const uint8_t* __restrict__ trunc) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n || t.status[i] != 0) return;
  const int set = w.set_of ? w.set_of[i] : 0;
  const int cnt = w.counts[set];
  const double* wp = w.points + size_t(set) * w.max_points * 3;
  t.total_reward[i] += double(rew[i]);
  t.steps[i] += 1;
  int k = t.wp_idx[i];
  // dist_to_wp = float(np.linalg.norm(drone_pos - current_target)): float32 pos minus the
  // float64 waypoint, norm in float64
  double d2 = 0.0;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const double d = double(s12[size_t(i) * 12 + j]) - wp[3 * k + j];
    d2 += d * d;
  }
  int status = 0;
  if (sqrt(d2) < double(w.reach_radius)) {
    t.reached[i] += 1;
    k = (k + 1) % cnt;
    t.wp_idx[i] = k;
    if (k == 0) {
      t.laps[i] += 1;
      status = 1;
    } else {
#pragma unroll
      for (int j = 0; j < 3; j++) Tiles(p).st(F_TGT + j, env_off(uint32_t(i)), float(wp[3 * k + j]));
    }
  }
  if (status == 0 && term[i]) status = 2;
  else if (status == 0 && trunc[i]) status = 3;
  t.status[i] = status;
}

// quad_get_state / quad_set_state: the dense [fields][N] pieces of QuadStateSoA <-> the tiles
struct StateIO {
  uint32_t* ptr[8];  // device pointers (4-byte elements), NULL = piece skipped
  int32_t f0[8], cnt[8];
};
template <bool TO_TILES>
__global__ __launch_bounds__(BLOCK) void k_state_io(KParams p, StateIO u) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= p.n) return;
  const Tiles S(p);
  const uint32_t vo = env_off(uint32_t(i));
  const size_t n = size_t(p.n);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (!u.ptr[k]) continue;
    for (int j = 0; j < u.cnt[k]; j++) {  // f uniform: the SGPR part of the offset stays scalar
      uint32_t* d = u.ptr[k] + size_t(j) * n + i;
      if (TO_TILES) S.stu(u.f0[k] + j, vo, *d);
      else *d = S.ldu(u.f0[k] + j, vo);
    }
  }
}

__global__ __launch_bounds__(BLOCK) void k_fill_field(KParams p, int32_t f, uint32_t x) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i < p.n) Tiles(p).stu(f, env_off(uint32_t(i)), x);
}

__global__ __launch_bounds__(BLOCK) void k_random_actions(int32_t n, uint64_t seed, uint64_t gid_base,
                                                          uint32_t step, float4* __restrict__ act) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const uint64_t gid = gid_base + uint64_t(i);
  uint32_t c[4] = {uint32_t(gid), uint32_t(gid >> 32), step, 0x100u};
  philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
  act[i] = make_float4(float(c[0] >> 8) * 0x1p-23f - 1.0f, float(c[1] >> 8) * 0x1p-23f - 1.0f,
                       float(c[2] >> 8) * 0x1p-23f - 1.0f, float(c[3] >> 8) * 0x1p-23f - 1.0f);
}

// SB3 RolloutBuffer.compute_returns_and_advantage, time-major [T, N]
__global__ __launch_bounds__(BLOCK) void k_gae(const float* __restrict__ rew, const float* __restrict__ val,
                                               const float* __restrict__ starts,
                                               const float* __restrict__ last_val,
                                               const float* __restrict__ dones, int32_t T, int32_t n,
                                               float gamma, float lam, float* __restrict__ adv,
                                               float* __restrict__ ret) {
  const int i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  float last = 0.f;
  float next_v = last_val[i];
  float next_nt = 1.0f - dones[i];
  for (int t = T - 1; t >= 0; t--) {
    const size_t o = size_t(t) * n + i;
    const float v = val[o];
    const float delta = rew[o] + gamma * next_v * next_nt - v;
    last = delta + gamma * lam * next_nt * last;
    adv[o] = last;
    ret[o] = last + v;
    next_v = v;
    next_nt = 1.0f - starts[o];
  }
}

}  // namespace

struct QuadHandle {
  QuadCfg cfg;
  int lanes = 1;  // lanes per env in k_step_g (1, 2, 4); 0 = k_step. QUADENV_LANES overrides
  PhysConstsD pd;
  KParams kp;
  int device;
  int n;
  float* tiles = nullptr;     // env state (layout at the top of this file)
  size_t tile_bytes = 0;
  uint32_t* stage = nullptr;  // [NFT][n] staging for host-side get/set_state, allocated on first use
  KConsts<float> kh;                 // host copy of the constant block
  KConsts<float>* kdev = nullptr;    // device copy the kernels read (scalar loads, K$-resident)
  bool spec = false;                 // kh == a reference default block: k_step's SPEC form
  bool helper = true;                // one-thread form: k_step_h (helper waves draw the resets)
  int hblock = 0;                    // envs per k_step_h block: 0 = by size (h_wide: 256 between H_SMALL and 2M, else 64)
  int hd = -1;                       // k_step_hd for the 64-env nt launches: -1 = by size (hd_form), 0 / 1
  int nt = -1;                       // k_step_h's state cache policy: -1 = by size (nt_state), 0 / 1
};

namespace {

int grid_of(int n) { return (n + BLOCK - 1) / BLOCK; }

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// k_step_h's state cache policy for a launch of `count` envs (env_tiles.h): nt where it measured
// faster -- one step wave per SIMD (65,536 envs) and the DRAM-bound sizes from 2M envs -- and the
// default policy where the next step reads the state back from the Infinity Cache (4,096 and
// 262,144 .. 1M envs; 32,768 measured equal). QUADENV_NT=0 / 1 pins it (A/B and tests).
bool nt_state(const QuadHandle* h, int64_t count) {
  if (h->nt >= 0) return h->nt != 0;
  return (count > H_SMALL && count < (int64_t(1) << 17)) || count >= (int64_t(1) << 21);
}

// k_step_h's block size for a launch of `count` envs: 256-env blocks above H_SMALL (the comment at
// H_SMALL), back to 64 from 2M envs, where the state streams from DRAM with the nt policy: 4M
// 264.2-264.5 vs 269.8-270.1 us, 2M 95.6-96.1 vs 97.7-98.4, 8M 545.7-546.9 vs 551.7-552.1, while 1M
// keeps 256 (52.7 vs 55.5-55.8; profiles/r04/r4_step_hb_large.txt). QUADENV_HBLOCK pins it.
bool h_wide(const QuadHandle* h, int64_t count) {
  if (h->hblock) return h->hblock == 256;
  return count > H_SMALL && count < (int64_t(1) << 21);
}

// k_step_hd instead of k_step_h<.., 64, true> for a launch of `count` envs: from 4M envs, where the
// step streams from DRAM (the comment at k_step_hd). QUADENV_HD=0 / 1 pins it (A/B and tests).
// Only HoverEnv without the rate controller by size: the trajectory and CTBR kinds spill 15-130
// VGPRs under its 7-wave budget (HoverEnv: 5) and keep k_step_h.
bool hd_form(const QuadHandle* h, int64_t count) {
  if (h_wide(h, count) || !nt_state(h, count)) return false;
  if (h->hd >= 0) return h->hd != 0;
  return count >= (int64_t(1) << 22) && h->cfg.env_kind == QUAD_ENV_HOVER && h->cfg.wrapper == QUAD_WRAP_NONE;
}

}  // namespace

extern "C" {

int quad_abi_version(void) { return QUADENV_ABI_VERSION; }

const char* quad_last_error(void) { return g_err.c_str(); }

int quad_default_cfg(int32_t env_kind, int32_t wrapper, QuadCfg* c) {
  if (!c) return fail(QUAD_EINVAL, "cfg is NULL");
  if (env_kind < QUAD_ENV_HOVER || env_kind > QUAD_ENV_BRAX_TRAJ)
    return fail(QUAD_EINVAL, "unknown env_kind");
  if (wrapper < QUAD_WRAP_NONE || wrapper > QUAD_WRAP_CTBR_RELPOS) return fail(QUAD_EINVAL, "unknown wrapper");
  if (env_kind >= QUAD_ENV_BRAX_HOVER && wrapper != QUAD_WRAP_NONE)
    return fail(QUAD_EINVAL, "the brax env kinds take no wrapper");
  default_cfg_fill(env_kind, wrapper, c);
  return QUAD_OK;
}

int quad_create(const QuadCfg* cfg, int32_t device, uint64_t seed, uint64_t env_id_base,
                int32_t n_envs, QuadHandle** out) {
  if (!cfg || !out) return fail(QUAD_EINVAL, "cfg/out is NULL");
  *out = nullptr;
  if (n_envs <= 0) return fail(QUAD_EINVAL, "n_envs must be > 0");
  // the tiles are one buffer resource (32-bit byte range); row outputs use 32-bit byte offsets
  if ((int64_t(n_envs) + 63) / 64 * TILE_BYTES > int64_t(UINT32_MAX))
    return fail(QUAD_EINVAL, "n_envs too large (max 31,580,608)");
  if (cfg->env_kind < QUAD_ENV_HOVER || cfg->env_kind > QUAD_ENV_BRAX_TRAJ)
    return fail(QUAD_EINVAL, "unknown env_kind");
  if (cfg->wrapper < QUAD_WRAP_NONE || cfg->wrapper > QUAD_WRAP_CTBR_RELPOS)
    return fail(QUAD_EINVAL, "unknown wrapper");
  if (cfg->env_kind >= QUAD_ENV_BRAX_HOVER && cfg->wrapper != QUAD_WRAP_NONE)
    return fail(QUAD_EINVAL, "the brax env kinds take no wrapper");
  if (cfg->max_episode_steps <= 0) return fail(QUAD_EINVAL, "max_episode_steps must be > 0");
  if (!(cfg->max_motor_thrust >= 0.0 && cfg->max_motor_thrust <= 1e30))
    return fail(QUAD_EINVAL, "max_motor_thrust must be finite and >= 0");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(QUAD_EINVAL, "device out of range");
  QuadHandle* h = new (std::nothrow) QuadHandle();
  if (!h) return fail(QUAD_ENOMEM, "host allocation failed");
  h->cfg = *cfg;
  const char* why = "";
  if (!make_phys_consts(*cfg, h->pd, &why)) {
    delete h;
    return fail(QUAD_EMODEL, why);
  }
  make_kconsts<float>(*cfg, h->pd, h->kh);
  h->spec = is_default_block(h->kh, cfg->env_kind, cfg->wrapper == QUAD_WRAP_CTBR);
  if (const char* v = std::getenv("QUADENV_SPEC")) h->spec = h->spec && std::atoi(v) != 0;
  // measured: helper waves 6.54 -> 5.87 us at 65,536 envs, 5.74 -> 4.24 at 4,096;
  // QUADENV_HELPER=0 keeps the plain k_step (A/B and tests)
  if (const char* v = std::getenv("QUADENV_HELPER")) h->helper = std::atoi(v) != 0;
  // QUADENV_HBLOCK=64|256 pins the helper form's block size (tests run the 256-env blocks at small N)
  if (const char* v = std::getenv("QUADENV_NT")) h->nt = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("QUADENV_HD")) h->hd = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("QUADENV_HBLOCK")) {
    const int b = std::atoi(v);
    if (b == 64 || b == 256) h->hblock = b;
  }
  h->device = device;
  h->n = n_envs;
  DeviceGuard g(device);
  h->tile_bytes = size_t((n_envs + 63) / 64) * TILE_BYTES;
  hipError_t e = hipMalloc(&h->tiles, h->tile_bytes);
  if (e == hipSuccess) e = hipMemset(h->tiles, 0, h->tile_bytes);
  if (e == hipSuccess) e = hipMalloc(&h->kdev, sizeof(KConsts<float>));
  if (e == hipSuccess) e = hipMemcpy(h->kdev, &h->kh, sizeof(KConsts<float>), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    quad_destroy(h);
    return hip_fail(e, "quad_create allocation");
  }
  h->kp.kc = h->kdev;
  h->kp.tiles = h->tiles;
  h->kp.tile_bytes = uint32_t(h->tile_bytes);
  h->kp.n = n_envs;
  h->kp.first = 0;
  h->kp.count = n_envs;
  h->kp.auto_reset = cfg->auto_reset;
  h->kp.seed = seed;
  h->kp.gid_base = env_id_base;
  // measured on MI355X (round 4, tools/step_env_ab.py, profiles/r04/r4_step_forms_nt.txt and
  // r4_step_nt_sizes.txt): the helper-wave form k_step_h (256-env blocks above 32,768 envs) with
  // its size-chosen cache policy (nt_state) is the fastest form at every size -- 262,144 envs 14.4
  // vs 15.9 us for k_step_g<1>, 1M 51.1 vs 51.9, 2M 97 vs 117 for k_step_g<2> (both nt), 4M 268.6 vs
  // 268.3, 8M 546 vs 557; the lane-group forms k_step_g<G> stay selectable (QUADENV_LANES)
  h->lanes = 0;
  if (const char* v = std::getenv("QUADENV_LANES")) {
    const int g = std::atoi(v);
    if (g == 0 || g == 1 || g == 2 || g == 4) h->lanes = g;
  }
  *out = h;
  return QUAD_OK;
}

void quad_destroy(QuadHandle* h) {
  if (!h) return;
  DeviceGuard g(h->device);
  if (h->tiles) (void)hipFree(h->tiles);
  if (h->stage) (void)hipFree(h->stage);
  if (h->kdev) (void)hipFree(h->kdev);
  delete h;
}

int32_t quad_num_envs(const QuadHandle* h) { return h ? h->n : 0; }

int32_t quad_kernel_form(const QuadHandle* h) {
  if (!h) return -1;
  // RELPOS and the brax kinds have one kernel each (k_step_relpos / k_step_brax): no lanes, SPEC
  // or helper forms to report
  if (wrap_relpos(h->cfg.wrapper) || h->cfg.env_kind >= QUAD_ENV_BRAX_HOVER) return 64;
  const bool wide = h_wide(h, h->n);
  return h->lanes | (h->spec ? 16 : 0) | (h->lanes == 0 && h->helper ? 32 : 0) |
         (h->lanes == 0 && h->helper && wide ? 128 : 0) | (h->lanes == 0 && h->helper && nt_state(h, h->n) ? 256 : 0) |
         (h->lanes == 0 && h->helper && hd_form(h, h->n) ? 512 : 0);
}

int quad_seed(QuadHandle* h, uint64_t seed, void* stream) {
  if (!h) return fail(QUAD_EINVAL, "handle is NULL");
  DeviceGuard g(h->device);
  h->kp.seed = seed;
  hipLaunchKernelGGL(k_fill_field, dim3(grid_of(h->n)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                     h->kp, int32_t(F_EP), 0u);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_reset(QuadHandle* h, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail(QUAD_EINVAL, "handle is NULL");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (h->cfg.env_kind == QUAD_ENV_BRAX_HOVER)
    hipLaunchKernelGGL(k_reset_brax<QUAD_ENV_BRAX_HOVER>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else if (h->cfg.env_kind == QUAD_ENV_BRAX_TRAJ)
    hipLaunchKernelGGL(k_reset_brax<QUAD_ENV_BRAX_TRAJ>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else if (wrap_relpos(h->cfg.wrapper) && h->cfg.env_kind == QUAD_ENV_TRAJ)
    hipLaunchKernelGGL((k_reset<QUAD_ENV_TRAJ, true>), dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else if (wrap_relpos(h->cfg.wrapper))
    hipLaunchKernelGGL((k_reset<QUAD_ENV_HOVER, true>), dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else if (h->cfg.env_kind == QUAD_ENV_TRAJ)
    hipLaunchKernelGGL((k_reset<QUAD_ENV_TRAJ, false>), dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  else
    hipLaunchKernelGGL((k_reset<QUAD_ENV_HOVER, false>), dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, mask, obs);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_step(QuadHandle* h, const float* actions, const QuadStepOut* out, void* stream) {
  return quad_step_range(h, 0, h ? h->n : 0, actions, out, stream);
}

int quad_step_range(QuadHandle* h, int32_t first, int32_t count, const float* actions,
                    const QuadStepOut* out, void* stream) {
  if (!h || !actions || !out) return fail(QUAD_EINVAL, "handle/actions/out is NULL");
  if (first < 0 || count < 0 || int64_t(first) + count > h->n)
    return fail(QUAD_EINVAL, "env range out of bounds");
  if (count == 0) return QUAD_OK;
  if (!out->obs || !out->reward || !out->terminated || !out->truncated)
    return fail(QUAD_EINVAL, "obs, reward, terminated and truncated are required");
  if ((reinterpret_cast<uintptr_t>(actions) | reinterpret_cast<uintptr_t>(out->obs)) & 15u)
    return fail(QUAD_EINVAL, "actions and obs must be 16-byte aligned");
  if (out->motor_commands && (reinterpret_cast<uintptr_t>(out->motor_commands) & 15u))
    return fail(QUAD_EINVAL, "motor_commands must be 16-byte aligned");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float4* a = reinterpret_cast<const float4*>(actions);
  const bool traj = h->cfg.env_kind == QUAD_ENV_TRAJ, ctbr = h->cfg.wrapper == QUAD_WRAP_CTBR;
  const dim3 blk(BLOCK);
  const int G = h->lanes;
  KParams kp = h->kp;
  kp.first = first;
  kp.count = count;
  if (wrap_relpos(h->cfg.wrapper)) {
    const dim3 grid(grid_of(count));
    const bool rc = h->cfg.wrapper == QUAD_WRAP_CTBR_RELPOS;
    if (traj && rc)
      hipLaunchKernelGGL((k_step_relpos<QUAD_ENV_TRAJ, true>), grid, blk, 0, s, h->kdev, kp, a, *out);
    else if (traj)
      hipLaunchKernelGGL((k_step_relpos<QUAD_ENV_TRAJ, false>), grid, blk, 0, s, h->kdev, kp, a, *out);
    else if (rc)
      hipLaunchKernelGGL((k_step_relpos<QUAD_ENV_HOVER, true>), grid, blk, 0, s, h->kdev, kp, a, *out);
    else
      hipLaunchKernelGGL((k_step_relpos<QUAD_ENV_HOVER, false>), grid, blk, 0, s, h->kdev, kp, a, *out);
  } else if (h->cfg.env_kind >= QUAD_ENV_BRAX_HOVER) {
    const dim3 grid(grid_of(count));
    if (h->cfg.env_kind == QUAD_ENV_BRAX_TRAJ)
      hipLaunchKernelGGL((k_step_brax<QUAD_ENV_BRAX_TRAJ>), grid, blk, 0, s, h->kdev, kp, a, *out);
    else
      hipLaunchKernelGGL((k_step_brax<QUAD_ENV_BRAX_HOVER>), grid, blk, 0, s, h->kdev, kp, a, *out);
  } else if (G == 0) {  // one thread per env with the LDS obs transpose
    const dim3 grid(grid_of(count));
#define QD_KARGS kp.tiles, a, kp.tile_bytes, kp.first, kp.count, h->kdev, kp, *out
#define QD_LAUNCH_K(SP)                                                                            \
  if (traj && ctbr)                                                                             \
    hipLaunchKernelGGL((k_step<QUAD_ENV_TRAJ, true, SP>), grid, blk, 0, s, QD_KARGS);      \
  else if (traj)                                                                                \
    hipLaunchKernelGGL((k_step<QUAD_ENV_TRAJ, false, SP>), grid, blk, 0, s, QD_KARGS);     \
  else if (ctbr)                                                                                \
    hipLaunchKernelGGL((k_step<QUAD_ENV_HOVER, true, SP>), grid, blk, 0, s, QD_KARGS);     \
  else                                                                                          \
    hipLaunchKernelGGL((k_step<QUAD_ENV_HOVER, false, SP>), grid, blk, 0, s, QD_KARGS);
#define QD_LAUNCH_H2(SP, HB, NT)                                                                       \
  if (traj && ctbr)                                                                             \
    hipLaunchKernelGGL((k_step_h<QUAD_ENV_TRAJ, true, SP, HB, NT>), grid, blk2, 0, s, QD_KARGS);      \
  else if (traj)                                                                                \
    hipLaunchKernelGGL((k_step_h<QUAD_ENV_TRAJ, false, SP, HB, NT>), grid, blk2, 0, s, QD_KARGS);     \
  else if (ctbr)                                                                                \
    hipLaunchKernelGGL((k_step_h<QUAD_ENV_HOVER, true, SP, HB, NT>), grid, blk2, 0, s, QD_KARGS);     \
  else                                                                                          \
    hipLaunchKernelGGL((k_step_h<QUAD_ENV_HOVER, false, SP, HB, NT>), grid, blk2, 0, s, QD_KARGS);
#define QD_LAUNCH_H(SP, HB) \
  if (nt) { QD_LAUNCH_H2(SP, HB, true) } else { QD_LAUNCH_H2(SP, HB, false) }
#define QD_LAUNCH_HD(SP)                                                                        \
  if (traj && ctbr)                                                                             \
    hipLaunchKernelGGL((k_step_hd<QUAD_ENV_TRAJ, true, SP>), grid, blk2, 0, s, QD_KARGS);       \
  else if (traj)                                                                                \
    hipLaunchKernelGGL((k_step_hd<QUAD_ENV_TRAJ, false, SP>), grid, blk2, 0, s, QD_KARGS);      \
  else if (ctbr)                                                                                \
    hipLaunchKernelGGL((k_step_hd<QUAD_ENV_HOVER, true, SP>), grid, blk2, 0, s, QD_KARGS);      \
  else                                                                                          \
    hipLaunchKernelGGL((k_step_hd<QUAD_ENV_HOVER, false, SP>), grid, blk2, 0, s, QD_KARGS);
    const bool wide = h_wide(h, count);
    const bool nt = nt_state(h, count);
    if (h->helper && hd_form(h, count)) {
      const dim3 grid(unsigned((int64_t(count) + 63) / 64)), blk2(128);
      if (h->spec) { QD_LAUNCH_HD(true) } else { QD_LAUNCH_HD(false) }
    } else if (h->helper && !wide) {
      const dim3 grid(unsigned((int64_t(count) + 63) / 64)), blk2(128);
      if (h->spec) { QD_LAUNCH_H(true, 64) } else { QD_LAUNCH_H(false, 64) }
    } else if (h->helper) {
      const dim3 grid(unsigned((int64_t(count) + 255) / 256)), blk2(512);
      if (h->spec) { QD_LAUNCH_H(true, 256) } else { QD_LAUNCH_H(false, 256) }
    } else if (h->spec) { QD_LAUNCH_K(true) } else { QD_LAUNCH_K(false) }
#undef QD_LAUNCH_K
#undef QD_LAUNCH_H
#undef QD_LAUNCH_H2
#undef QD_LAUNCH_HD
#undef QD_KARGS
  } else {
    const dim3 grid(unsigned((int64_t(count) * G + BLOCK - 1) / BLOCK));
#define QD_GARGS kp.tiles, a, kp.tile_bytes, kp.first, kp.count, h->kdev, kp, *out
#define QD_LAUNCH(GG, SP)                                                                          \
  if (traj && ctbr)                                                                             \
    hipLaunchKernelGGL((k_step_g<QUAD_ENV_TRAJ, true, GG, SP>), grid, blk, 0, s, QD_GARGS);   \
  else if (traj)                                                                                \
    hipLaunchKernelGGL((k_step_g<QUAD_ENV_TRAJ, false, GG, SP>), grid, blk, 0, s, QD_GARGS);  \
  else if (ctbr)                                                                                \
    hipLaunchKernelGGL((k_step_g<QUAD_ENV_HOVER, true, GG, SP>), grid, blk, 0, s, QD_GARGS);  \
  else                                                                                          \
    hipLaunchKernelGGL((k_step_g<QUAD_ENV_HOVER, false, GG, SP>), grid, blk, 0, s, QD_GARGS);
    if (G == 1) {  // the batch-size default above 262,144 envs: SPEC form when the block is the default
      if (h->spec) { QD_LAUNCH(1, true) } else { QD_LAUNCH(1, false) }
    } else if (G == 2) {
      if (h->spec) { QD_LAUNCH(2, true) } else { QD_LAUNCH(2, false) }
    } else { QD_LAUNCH(4, false) }
#undef QD_LAUNCH
#undef QD_GARGS
  }
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_rollout(QuadHandle* h, const float* packed, const QuadRollout* r, void* stream) {
  if (!h || !packed || !r) return fail(QUAD_EINVAL, "handle/packed/rollout is NULL");
  if (!r->obs_copy || !r->actions || !r->log_prob || !r->value || !r->episode_starts || !r->rewards ||
      !r->last_obs || !r->last_start || !r->ep_ret || !r->ep_len || !r->stats)
    return fail(QUAD_EINVAL, "quad_rollout: NULL buffer");
  if (r->rows < 1 || r->steps < 1 || r->t0 < 0) return fail(QUAD_EINVAL, "quad_rollout: rows, steps >= 1, t0 >= 0");
  if ((reinterpret_cast<uintptr_t>(packed) | reinterpret_cast<uintptr_t>(r->actions) |
       reinterpret_cast<uintptr_t>(r->obs_copy) | reinterpret_cast<uintptr_t>(r->last_obs)) & 15u)
    return fail(QUAD_EINVAL, "quad_rollout: packed, actions, obs_copy and last_obs must be 16-byte aligned");
  if (h->cfg.env_kind != QUAD_ENV_HOVER && h->cfg.env_kind != QUAD_ENV_TRAJ)
    return fail(QUAD_EINVAL, "quad_rollout: env_kind must be HOVER or TRAJ");
  if (wrap_relpos(h->cfg.wrapper)) return fail(QUAD_EINVAL, "quad_rollout: the policy takes 12-D obs (no RELPOS)");
  if (!h->cfg.auto_reset) return fail(QUAD_EINVAL, "quad_rollout: the handle needs auto_reset = 1");
  DeviceGuard g(h->device);
  RollArgs a{r->obs_copy, r->actions, r->log_prob, r->value, r->episode_starts, r->rewards, r->last_obs,
             r->last_start, r->ep_ret, r->ep_len, r->stats, uint32_t(r->rows), uint32_t(r->t0), r->steps,
             r->deterministic, r->seed, r->gamma};
  HIP_TRY(launch_rollout(h->kdev, h->kp, h->cfg.env_kind, h->cfg.wrapper == QUAD_WRAP_CTBR, h->spec, packed, a,
                         static_cast<hipStream_t>(stream)));
  return QUAD_OK;
}

int quad_observe(QuadHandle* h, float* obs, float* state12, void* stream) {
  if (!h || !obs) return fail(QUAD_EINVAL, "handle/obs is NULL");
  DeviceGuard g(h->device);
  if (h->cfg.env_kind >= QUAD_ENV_BRAX_HOVER) {  // raw [qpos, qvel]; no QuadState
    if (state12) return fail(QUAD_EINVAL, "state12 is not defined for the brax env kinds");
    hipLaunchKernelGGL(k_observe_brax, dim3(grid_of(h->n)), dim3(BLOCK), 0,
                       static_cast<hipStream_t>(stream), h->kp, obs);
    HIP_TRY(hipGetLastError());
    return QUAD_OK;
  }
  if (wrap_relpos(h->cfg.wrapper))
    hipLaunchKernelGGL(k_observe<true>, dim3(grid_of(h->n)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                       h->kp, obs, state12);
  else
    hipLaunchKernelGGL(k_observe<false>, dim3(grid_of(h->n)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                       h->kp, obs, state12);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_step_random(QuadHandle* h, uint32_t step0, int32_t steps, const QuadStepOut* out, float* actions_out,
                     void* stream) {
  if (!h || !out) return fail(QUAD_EINVAL, "handle/out is NULL");
  if (steps < 0) return fail(QUAD_EINVAL, "steps must be >= 0");
  if (steps == 0) return QUAD_OK;
  if (h->cfg.env_kind != QUAD_ENV_HOVER && h->cfg.env_kind != QUAD_ENV_TRAJ)
    return fail(QUAD_EINVAL, "quad_step_random drives the hover / trajectory kinds");
  if (wrap_relpos(h->cfg.wrapper)) return fail(QUAD_EINVAL, "quad_step_random: wrapper NONE or CTBR");
  if (!out->obs || !out->reward || !out->terminated || !out->truncated)
    return fail(QUAD_EINVAL, "obs, reward, terminated and truncated are required");
  if (out->motor_commands || out->voltage_scale || out->state12 || out->target_info)
    return fail(QUAD_EINVAL, "quad_step_random writes obs, reward, flags and terminal_obs only");
  if ((reinterpret_cast<uintptr_t>(out->obs) | reinterpret_cast<uintptr_t>(actions_out)) & 15u)
    return fail(QUAD_EINVAL, "obs and actions_out must be 16-byte aligned");
  if (int64_t(steps) * h->n * 48 > int64_t(UINT32_MAX))
    return fail(QUAD_EINVAL, "steps * N too large for one launch (time-major rows use 32-bit byte offsets)");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(grid_of(h->n)), blk(BLOCK);
  float4* ao = reinterpret_cast<float4*>(actions_out);
  const bool traj = h->cfg.env_kind == QUAD_ENV_TRAJ, ctbr = h->cfg.wrapper == QUAD_WRAP_CTBR;
#define QD_LAUNCH_R(SP)                                                                                     \
  if (traj && ctbr)                                                                                      \
    hipLaunchKernelGGL((k_step_random<QUAD_ENV_TRAJ, true, SP>), grid, blk, 0, s, h->kdev, h->kp, *out, ao, step0, steps);   \
  else if (traj)                                                                                         \
    hipLaunchKernelGGL((k_step_random<QUAD_ENV_TRAJ, false, SP>), grid, blk, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else if (ctbr)                                                                                         \
    hipLaunchKernelGGL((k_step_random<QUAD_ENV_HOVER, true, SP>), grid, blk, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else                                                                                                   \
    hipLaunchKernelGGL((k_step_random<QUAD_ENV_HOVER, false, SP>), grid, blk, 0, s, h->kdev, h->kp, *out, ao, step0, steps);
#define QD_LAUNCH_RH(SP, RB)                                                                                     \
  if (traj && ctbr)                                                                                      \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_TRAJ, true, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);   \
  else if (traj)                                                                                         \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_TRAJ, false, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else if (ctbr)                                                                                         \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_HOVER, true, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else                                                                                                   \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_HOVER, false, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);
  // the block size of k_step_h's policy (h_wide: 64-env blocks up to H_SMALL and from 2M envs);
  // the K-step form reads and writes its state once per launch, so the nt policy does not apply
  const bool wide = h_wide(h, h->n);
  if (h->helper && !wide) {
    const dim3 grid(unsigned((int64_t(h->n) + 63) / 64)), blk2(128);
    if (h->spec) { QD_LAUNCH_RH(true, 64) } else { QD_LAUNCH_RH(false, 64) }
  } else if (h->helper) {
    const dim3 grid(unsigned((int64_t(h->n) + 255) / 256)), blk2(512);
    if (h->spec) { QD_LAUNCH_RH(true, 256) } else { QD_LAUNCH_RH(false, 256) }
  } else if (h->spec) { QD_LAUNCH_R(true) } else { QD_LAUNCH_R(false) }
#undef QD_LAUNCH_R
#undef QD_LAUNCH_RH
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_terminated(QuadHandle* h, const float* state12, int32_t n, uint8_t* terminated, void* stream) {
  if (!h || !state12 || !terminated) return fail(QUAD_EINVAL, "handle/state12/terminated is NULL");
  if (h->cfg.env_kind >= QUAD_ENV_BRAX_HOVER) return fail(QUAD_EINVAL, "the brax env kinds have no QuadState bounds");
  if (n < 0) return fail(QUAD_EINVAL, "n must be >= 0");
  if (n == 0) return QUAD_OK;
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(k_terminated, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                     h->kdev, state12, n, terminated);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_random_actions(QuadHandle* h, uint32_t step_index, float* actions, void* stream) {
  if (!h || !actions) return fail(QUAD_EINVAL, "handle/actions is NULL");
  if (reinterpret_cast<uintptr_t>(actions) & 15u) return fail(QUAD_EINVAL, "actions must be 16-byte aligned");
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(k_random_actions, dim3(grid_of(h->n)), dim3(BLOCK), 0,
                     static_cast<hipStream_t>(stream), h->n, h->kp.seed, h->kp.gid_base, step_index,
                     reinterpret_cast<float4*>(actions));
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

static int copy_state(QuadHandle* h, const QuadStateSoA* u, int on_host, void* stream, bool to_handle) {
  if (!h || !u) return fail(QUAD_EINVAL, "handle/state is NULL");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t n = size_t(h->n);
  struct Piece { void* user; int f0, cnt; };  // user: dense [cnt][n] 4-byte elements
  const Piece pieces[8] = {
      {u->qpos, F_QPOS, 11}, {u->qvel, F_QVEL, 10}, {u->voltage, F_VOLT, 1}, {u->target, F_TGT, 3},
      {u->rate_int, F_RINT, 3}, {u->step_count, F_STEP, 1}, {u->episode, F_EP, 1}, {u->prev_action, F_PREV, 4},
  };
  if (on_host && !h->stage) HIP_TRY(hipMalloc(&h->stage, sizeof(uint32_t) * size_t(NFT) * n));
  StateIO io;
  for (int k = 0; k < 8; k++) {
    const Piece& p = pieces[k];
    io.f0[k] = p.f0;
    io.cnt[k] = p.cnt;
    io.ptr[k] = !p.user ? nullptr : on_host ? h->stage + size_t(p.f0) * n : static_cast<uint32_t*>(p.user);
  }
  const size_t esz = sizeof(uint32_t);
  if (to_handle) {
    if (on_host)
      for (const Piece& p : pieces)
        if (p.user) HIP_TRY(hipMemcpyAsync(h->stage + size_t(p.f0) * n, p.user, esz * p.cnt * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_state_io<true>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, io);
    HIP_TRY(hipGetLastError());
  } else {
    hipLaunchKernelGGL(k_state_io<false>, dim3(grid_of(h->n)), dim3(BLOCK), 0, s, h->kp, io);
    HIP_TRY(hipGetLastError());
    if (on_host)
      for (const Piece& p : pieces)
        if (p.user) HIP_TRY(hipMemcpyAsync(p.user, h->stage + size_t(p.f0) * n, esz * p.cnt * n, hipMemcpyDeviceToHost, s));
  }
  if (on_host) HIP_TRY(hipStreamSynchronize(s));
  return QUAD_OK;
}

int quad_get_state(QuadHandle* h, const QuadStateSoA* dst, int32_t on_host, void* stream) {
  return copy_state(h, dst, on_host, stream, false);
}

int quad_set_state(QuadHandle* h, const QuadStateSoA* src, int32_t on_host, void* stream) {
  return copy_state(h, src, on_host, stream, true);
}

static int check_waypoints(QuadHandle* h, const QuadWaypoints* w, const QuadWaypointState* s) {
  if (!h || !w || !s) return fail(QUAD_EINVAL, "handle/waypoints/state is NULL");
  if (!w->points || !w->counts || w->max_points < 1) return fail(QUAD_EINVAL, "waypoint table is empty");
  if (!(w->reach_radius > 0.f)) return fail(QUAD_EINVAL, "reach_radius must be > 0");
  if (!s->wp_idx || !s->reached || !s->laps || !s->steps || !s->status || !s->total_reward)
    return fail(QUAD_EINVAL, "waypoint tracker arrays are required");
  if (h->cfg.env_kind >= QUAD_ENV_BRAX_HOVER) return fail(QUAD_EINVAL, "waypoint evaluation needs a HoverEnv kind");
  return QUAD_OK;
}

int quad_waypoints_begin(QuadHandle* h, const QuadWaypoints* w, const QuadWaypointState* s, float* obs,
                         void* stream) {
  if (int rc = check_waypoints(h, w, s)) return rc;
  if (!obs) return fail(QUAD_EINVAL, "obs is NULL");
  DeviceGuard g(h->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (wrap_relpos(h->cfg.wrapper))
    hipLaunchKernelGGL(k_waypoints_begin<true>, dim3(grid_of(h->n)), dim3(BLOCK), 0, st, h->kp, *w, *s, obs);
  else
    hipLaunchKernelGGL(k_waypoints_begin<false>, dim3(grid_of(h->n)), dim3(BLOCK), 0, st, h->kp, *w, *s, obs);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_waypoints_update(QuadHandle* h, const QuadWaypoints* w, const QuadWaypointState* s,
                          const float* state12, const float* reward, const uint8_t* terminated,
                          const uint8_t* truncated, void* stream) {
  if (int rc = check_waypoints(h, w, s)) return rc;
  if (!state12 || !reward || !terminated || !truncated) return fail(QUAD_EINVAL, "step outputs are required");
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(k_waypoints_update, dim3(grid_of(h->n)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream),
                     h->kp, *w, *s, state12, reward, terminated, truncated);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

int quad_gae(const float* rewards, const float* values, const float* episode_starts,
             const float* last_values, const float* dones, int32_t T, int32_t N, float gamma,
             float gae_lambda, float* advantages, float* returns, void* stream) {
  if (!rewards || !values || !episode_starts || !last_values || !dones || !advantages || !returns)
    return fail(QUAD_EINVAL, "NULL argument");
  if (T <= 0 || N <= 0) return fail(QUAD_EINVAL, "T and N must be > 0");
  hipLaunchKernelGGL(k_gae, dim3(grid_of(N)), dim3(BLOCK), 0, static_cast<hipStream_t>(stream), rewards,
                     values, episode_starts, last_values, dones, T, N, gamma, gae_lambda, advantages,
                     returns);
  HIP_TRY(hipGetLastError());
  return QUAD_OK;
}

}  // extern "C"
