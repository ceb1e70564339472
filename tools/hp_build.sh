#!/bin/bash
# Profiling tool (not product; needs tools/patches/step_hp_persistent_prefetch.patch applied -- round 6
# A/B, not kept, profiles/r06/step_hp_ab.txt): libquadenv.so builds with k_step_hp's waves-per-SIMD floor
# (QD_HP_WAVES) = 4 / 5 / 6 -> tools/_build/hp<N>.so, the other objects from the in-tree build.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/uav_reinforcement_learning_control_amd/csrc
O=$ROOT/uav_reinforcement_learning_control_amd/_lib/obj
make -s -C $C
mkdir -p $ROOT/tools/_build/obj
for w in ${HP_WAVES:-4 5 6}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=on \
    -fno-slp-vectorize -I$O -mllvm -amdgpu-kernarg-preload-count=16 -DQD_HP_WAVES=$w \
    -c -o $ROOT/tools/_build/obj/quadenv_hp$w.o $C/quadenv.hip &
done
wait
for w in ${HP_WAVES:-4 5 6}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/_build/hp$w.so \
    $ROOT/tools/_build/obj/quadenv_hp$w.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o
  echo built tools/_build/hp$w.so
done
