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
//   k_step_h<KIND, CTBR> fused: (CTBR) -> mixer -> voltage -> mj_step -> obs -> reward ->
//   (k_step_hd)          termination/truncation -> SB3 auto-reset -> obs, with helper waves
//                        (control path, next-reset rows); k_step_hd: its >= 4M-env DRAM form
//   k_step_random_h      config 2: K random-action steps per launch
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
constexpr int H_PRE = 1;  // Philox blocks of the helper's reset draw issued before barrier (C): 1 measured best (below)
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
// (profiles/r05/step_rowmajor_image_ab.txt).
// H / CT layout: 16-byte env rows (H: 28 words, CT: CT_STRIDE) without CTBR; the CTBR kinds keep the
// field-major [f][HB] forms (config 5 at 65,536 envs measured 5.92 vs 5.78 us with row-major H)
template <bool CTBR>
constexpr bool ct_rows() { return !CTBR; }
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
    constexpr int PRE = H_PRE;
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
#if defined(QD_ABL_HDRAW0)  // cost ablation (tools only): the helper's reset row without its Philox words
#pragma unroll
    for (int j = 0; j < 16; j++) u16[j] = u01(uint32_t(i) * 0x9E3779B9u + ep * 0x85EBCA6Bu + uint32_t(j) * 0xC2B2AE35u);
#endif
    float init12[12], tgt[3], obs[12], s12[12];
    reset_affine_u(K.init_lo, K.init_span, K.tgt_lo, K.tgt_span, u16, init12, tgt);
    EnvRegs<float> e;
    env_reset_from<float, KIND>(K, e, init12, tgt, obs, s12);
#if defined(QD_ABL_HROW0)  // cost ablation (tools only): no reset row at all (zeros)
#pragma unroll
    for (int j = 0; j < 3; j++) { e.pos[j] = e.v[j] = e.w[j] = e.target[j] = 0.f; }
#pragma unroll
    for (int j = 0; j < 4; j++) e.q[j] = 0.f;
#pragma unroll
    for (int j = 0; j < 12; j++) obs[j] = 0.f;
#endif
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
#if !defined(QD_ABL_NOPHYSH)  // cost ablation (tools only): k_step_h without the rigid-body step
    forward_base(K.ph, qn, e.th, e.v, e.w, e.s, fa);
#endif
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
#if !defined(QD_ABL_NOPHYSH)
    physics_finish<float, true>(K.ph, e, qn, fa, m);
#else
    e.pos[0] += m.Fsum * 1e-9f;  // keeps the control hand-off live
#endif
    if (stamps) { QD_PIN_N(e.pos, 3); QD_PIN_N(e.q, 4); QD_PIN_N(e.v, 3); QD_PIN_N(e.w, 3); }
    QD_STAMP(stamps, 4);
    StepRes r;
    env_post(K, e, r);
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

// SPEC: the handle's constant block equals the reference default (quad_create checks the bytes), so
// the constants are compiled in -- no scalar loads of the block and no waits on them inside the step.
// Kernel-argument preload (csrc/Makefile: -amdgpu-kernarg-preload-count=16): the leading scalar
// arguments -- what the state loads need: tiles, their size, the env range, the actions -- arrive
// in SGPRs at wave launch, so the loads are issued without first waiting on a scalar load of the
// kernarg segment (the KParams / QuadStepOut aggregates behind them are not preloaded).
template <int KIND, bool CTBR, bool SPEC, int HB, bool NT>
__global__ __launch_bounds__(2 * HB) void k_step_h(float* tiles, const float4* __restrict__ act, uint32_t tile_bytes,
                                                      int32_t first, int32_t count,
                                                      const KConsts<float>* __restrict__ kc, KParams p, QuadStepOut out) {
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;  // preloaded (above)
  p.kc = kc;  // noalias: constant-block loads stay scalar after the stores (see KParams)
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
  p.tiles = tiles; p.tile_bytes = tile_bytes; p.first = first; p.count = count;  // preloaded (see k_step_h)
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

// quad_mem_floor: the step's loads and stores with no compute (bench.py's live DRAM floor). One env
// per lane, 256-env blocks, the state through the same buffer resource and cache policy (AUX) as
// k_step_h's tiles; obs rows as three dwordx4 per lane (a wave's rows are contiguous).
template <int AUX>
__global__ __launch_bounds__(256) void k_mem_floor(KParams p, const float4* __restrict__ act, QuadStepOut out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.n) return;
  const TilesA<AUX> S(p);
  const uint32_t o = env_off(uint32_t(i));
  uint32_t x[26];
#pragma unroll
  for (int f = 0; f < 25; f++) x[f] = S.ldu(f, o);
  x[25] = S.ldu(F_STEP, o);
  const float4 a = act[i];
  // the action feeds the flags (false for any finite action), so its load is not dead
  const bool big = !(fabsf(a.x + a.y + a.z + a.w) < 1e30f);
  const uint32_t q = fresh_off(o);
#pragma unroll
  for (int f = 0; f < 25; f++) S.stu(f, q, x[f]);
  S.stu(F_STEP, q, x[25]);
  float4* ob = reinterpret_cast<float4*>(out.obs) + size_t(i) * 3;
#pragma unroll
  for (int j = 0; j < 3; j++)
    ob[j] = make_float4(__uint_as_float(x[4 * j]), __uint_as_float(x[4 * j + 1]), __uint_as_float(x[4 * j + 2]),
                        __uint_as_float(x[4 * j + 3]));
  out.reward[i] = __uint_as_float(x[0]);
  out.terminated[i] = big;
  out.truncated[i] = big;
}

// Config 2 of the scope table -- debug_training.py:111's loop env.step(env.action_space.sample())
// -- as ONE launch: `steps` whole steps per env with the action of step s drawn in-kernel from
// quad_random_actions' map, Philox(seed; gid, step0 + s, 0x100), and the env state kept in registers
// between steps (read once, written once). Per step every output row goes to HBM as in k_step_h:
// obs [N,12], reward, flags, terminal obs of finishing envs, all time-major [steps][N, ...].
// RB = envs per k_step_random_h block: 64 up to H_SMALL envs (4,096 envs: 2.22 vs 2.40 us per
// step with 256), 256 above (65,536: 3.4 vs 4.5 us with 64); profiles/r02/ab_step_h_block.txt.
// The helper-wave form (see k_step_h): a 512-thread block owns 256 envs; waves 0-3 step them,
// waves 4-7 draw -- two steps ahead -- each env's actions (quad_random_actions' Philox map) into a
// double-buffered LDS slot, and keep each env's next-reset row (k_step_h's image) current: after
// every step they read which envs reset, advance those episode counters and redraw their rows.
// Per step: barrier A (flags known; the image is current) -> resets copied, obs rows staged ->
// barrier B -> obs rows stored by all 512 threads, helpers redraw. Same env_step code as k_step_h, so
// the same bits as K single steps.
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
  PhysConstsD pd;
  KParams kp;
  int device;
  int n;
  float* tiles = nullptr;     // env state (layout at the top of this file)
  size_t tile_bytes = 0;
  uint32_t* stage = nullptr;  // [NFT][n] staging for host-side get/set_state, allocated on first use
  KConsts<float> kh;                 // host copy of the constant block
  KConsts<float>* kdev = nullptr;    // device copy the kernels read (scalar loads, K$-resident)
  bool spec = false;                 // kh == a reference default block: k_step_h's SPEC form
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
  // The step forms: the helper-wave form k_step_h (256-env blocks above 32,768 envs) with
  // its size-chosen cache policy (nt_state) and k_step_hd from 4M envs measured fastest at every size
  // (round 2: helper waves 6.54 -> 5.87 us at 65,536 envs, 5.74 -> 4.24 at 4,096 against the one-wave
  // form; round 4, profiles/r04/r4_step_forms_nt.txt and r4_step_nt_sizes.txt: 262,144 envs 14.4 vs
  // 15.9 us for the lane-group form with one env per lane, 1M 51.1 vs 51.9, 2M 97 vs 117 for two lanes
  // per env). The one-wave and lane-group forms were A/B builds; round 6 removed them from the library.
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
  // bit 5: the helper-wave form (always; bits 0-2 were the removed lane-group forms)
  return (h->spec ? 16 : 0) | 32 | (h_wide(h, h->n) ? 128 : 0) | (nt_state(h, h->n) ? 256 : 0) |
         (hd_form(h, h->n) ? 512 : 0);
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
  } else {  // one thread per env, helper waves beside the step waves
#define QD_KARGS kp.tiles, a, kp.tile_bytes, kp.first, kp.count, h->kdev, kp, *out
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
    if (hd_form(h, count)) {
      const dim3 grid(unsigned((int64_t(count) + 63) / 64)), blk2(128);
      if (h->spec) { QD_LAUNCH_HD(true) } else { QD_LAUNCH_HD(false) }
    } else if (!wide) {
      const dim3 grid(unsigned((int64_t(count) + 63) / 64)), blk2(128);
      if (h->spec) { QD_LAUNCH_H(true, 64) } else { QD_LAUNCH_H(false, 64) }
    } else {
      const dim3 grid(unsigned((int64_t(count) + 255) / 256)), blk2(512);
      if (h->spec) { QD_LAUNCH_H(true, 256) } else { QD_LAUNCH_H(false, 256) }
    }
#undef QD_LAUNCH_H
#undef QD_LAUNCH_H2
#undef QD_LAUNCH_HD
#undef QD_KARGS
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

int quad_mem_floor(QuadHandle* h, const float* actions, const QuadStepOut* out, void* stream) {
  if (!h || !actions || !out) return fail(QUAD_EINVAL, "handle/actions/out is NULL");
  if (!out->obs || !out->reward || !out->terminated || !out->truncated)
    return fail(QUAD_EINVAL, "obs, reward, terminated and truncated are required");
  if ((reinterpret_cast<uintptr_t>(actions) | reinterpret_cast<uintptr_t>(out->obs)) & 15u)
    return fail(QUAD_EINVAL, "actions and obs must be 16-byte aligned");
  if (h->cfg.env_kind != QUAD_ENV_HOVER && h->cfg.env_kind != QUAD_ENV_TRAJ)
    return fail(QUAD_EINVAL, "quad_mem_floor: hover / trajectory kinds");
  if (wrap_relpos(h->cfg.wrapper)) return fail(QUAD_EINVAL, "quad_mem_floor: no RELPOS (7-D obs rows)");
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(unsigned((int64_t(h->n) + 255) / 256)), blk(256);
  const float4* a = reinterpret_cast<const float4*>(actions);
  if (nt_state(h, h->n))
    hipLaunchKernelGGL(k_mem_floor<2>, grid, blk, 0, s, h->kp, a, *out);
  else
    hipLaunchKernelGGL(k_mem_floor<0>, grid, blk, 0, s, h->kp, a, *out);
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
  float4* ao = reinterpret_cast<float4*>(actions_out);
  const bool traj = h->cfg.env_kind == QUAD_ENV_TRAJ, ctbr = h->cfg.wrapper == QUAD_WRAP_CTBR;
#define QD_LAUNCH_RH(SP, RB)                                                                                     \
  if (traj && ctbr)                                                                                      \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_TRAJ, true, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);   \
  else if (traj)                                                                                         \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_TRAJ, false, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else if (ctbr)                                                                                         \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_HOVER, true, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);  \
  else                                                                                                   \
    hipLaunchKernelGGL((k_step_random_h<QUAD_ENV_HOVER, false, SP, RB>), grid, blk2, 0, s, h->kdev, h->kp, *out, ao, step0, steps);
  // 64-env blocks up to H_SMALL envs, 256 above at every size: the K-step form reads and writes its
  // state once per launch, so k_step_h's reason for 64-env blocks from 2M envs (nt state streams)
  // does not apply -- 2M envs 93.6 vs 97.4 us per step, 4M 182.9 vs 195.7 with 64-env blocks
  // (profiles/r06/kstep_random_block_ab.txt). QUADENV_HBLOCK pins it.
  const bool wide = h->hblock ? h->hblock == 256 : h->n > H_SMALL;
  if (!wide) {
    const dim3 grid(unsigned((int64_t(h->n) + 63) / 64)), blk2(128);
    if (h->spec) { QD_LAUNCH_RH(true, 64) } else { QD_LAUNCH_RH(false, 64) }
  } else {
    const dim3 grid(unsigned((int64_t(h->n) + 255) / 256)), blk2(512);
    if (h->spec) { QD_LAUNCH_RH(true, 256) } else { QD_LAUNCH_RH(false, 256) }
  }
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
