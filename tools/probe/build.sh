#!/bin/bash
# Profiling tool (not product): libquadenv.so built with -DQD_PROBE (k_step records per-wave
# s_memtime phase stamps into the target_info buffer) -> tools/_build/probe.so
set -e
cd "$(dirname "$0")/../../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=16"
O=../_lib/obj
/opt/rocm/bin/hipcc $F -I$O -DQD_PROBE ${EXTRA:-} -c -o ../../tools/_build/obj/quadenv_probe.o quadenv.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/probe.so \
  ../../tools/_build/obj/quadenv_probe.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o
