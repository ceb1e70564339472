// rollout.h -- host-side entry of the fused rollout kernel (rollout.hip), called by quad_rollout.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "env_tiles.h"

namespace quadenv {

struct RollArgs {  // QuadRollout, flattened
  float* obs_copy;
  float* actions;
  float* log_prob;
  float* value;
  float* starts;
  float* rewards;
  float* last_obs;
  float* last_start;
  float* ep_ret;
  float* ep_len;
  double* stats;
  uint32_t rows;
  uint32_t t0;
  int32_t steps;
  int32_t deterministic;
  uint64_t seed;
  float gamma;
};

// k_rollout<env_kind, ctbr> over all envs of kp (one 256-env block per CU-resident slot)
hipError_t launch_rollout(const KConsts<float>* kc, const KParams& kp, int env_kind, bool ctbr, bool spec,
                          const float* packed, const RollArgs& a, hipStream_t s);

}  // namespace quadenv
