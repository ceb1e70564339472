#!/bin/bash
# Profiling tool (not product): k_step_h's helper reset-draw cost ablations -> tools/_build/hd_HDRAW0.so
# (the reset row from a cheap hash instead of the 4 Philox blocks) and hd_HROW0.so (no reset row);
# ("A+B" builds both ablations); A/B with tools/lib_ab.py N tools/_build/hd_HDRAW0.so tools/_build/hd_HROW0.so
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=16"
O=../_lib/obj
for v in ${VARIANTS:-HDRAW0 HROW0}; do
  ( D=$(echo $v | sed "s/+/ -DQD_ABL_/g"); /opt/rocm/bin/hipcc $F -I$O -DQD_ABL_$D -c -o ../../tools/_build/obj/quadenv_$v.o quadenv.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/hd_$v.so \
      ../../tools/_build/obj/quadenv_$v.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o ) &
done
wait
