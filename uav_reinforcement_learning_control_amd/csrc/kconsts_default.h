// kconsts_default.h -- the reference defaults' constant blocks (KConsts<float>, quad_physics.h) as
// compile-time objects, for the kernels' SPEC forms. The words are generated at build time by
// gen_kconsts.cpp from the same default_cfg_fill / make_phys_consts / make_kconsts that
// quad_create runs; a handle takes the SPEC kernels only when its block is byte-identical
// (is_default_block), so a SPEC kernel computes exactly what the generic one would, with every
// constant an immediate operand instead of a scalar load of the handle's block (-0.7 us of a
// 7.2 us step at 65,536 envs: the lone wave otherwise waits on those loads).
#pragma once

#include <cstring>

#include "quad_physics.h"

namespace quadenv {
#include "kconsts_default.inc"

template <int KIND, bool CTBR>
constexpr KConsts<float> kdef_block() {
  static_assert(sizeof(KWords) == sizeof(KConsts<float>), "stale kconsts_default.inc: rebuild");
  return __builtin_bit_cast(KConsts<float>, KIND == QUAD_ENV_TRAJ ? (CTBR ? kdef_traj_ctbr : kdef_traj)
                                                                  : (CTBR ? kdef_hover_ctbr : kdef_hover));
}

inline bool is_default_block(const KConsts<float>& k, int kind, bool ctbr) {
  if (kind != QUAD_ENV_HOVER && kind != QUAD_ENV_TRAJ) return false;
  const KWords& w = kind == QUAD_ENV_TRAJ ? (ctbr ? kdef_traj_ctbr : kdef_traj) : (ctbr ? kdef_hover_ctbr : kdef_hover);
  return std::memcmp(&k, &w, sizeof w) == 0;
}
}  // namespace quadenv
