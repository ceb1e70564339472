#!/bin/bash
# Profiling tool (not product): libquadenv.so with the learner's QD_LPROBE stamps (learner_x3.hip)
# -> tools/_build/lprobe.so
set -e
cd "$(dirname "$0")/../../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
O=../_lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -mllvm -amdgpu-mfma-vgpr-form -DQD_LPROBE \
  -c -o ../../tools/_build/obj/learner_x3_probe.o learner_x3.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/lprobe.so \
  $O/quadenv.o $O/policy.o $O/rollout.o $O/learner.o ../../tools/_build/obj/learner_x3_probe.o
