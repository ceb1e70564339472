#!/bin/bash
# Profiling tool (not product): cost-ablation builds of libquadenv.so for tools/learner_bench.py --
# quad_ppo_grad without the L2 MFMAs, without the weight-gradient MFMAs (dW2, dW3), without
# dh1 + dW1. Output: tools/_build/lrn_*.so (run learner_bench.py with QUADENV_LIB=<so>)
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -c -o ../../tools/_build/obj/quadenv.o quadenv.hip &
/opt/rocm/bin/hipcc $F -c -o ../../tools/_build/obj/policy.o policy.hip &
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -c -o ../../tools/_build/obj/rollout.o rollout.hip &
for v in NOL2 NODW NODH1; do
  /opt/rocm/bin/hipcc $F -DQD_LRN_$v -c -o ../../tools/_build/obj/learner_$v.o learner.hip &
done
wait
for v in NOL2 NODW NODH1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/lrn_$v.so \
    ../../tools/_build/obj/quadenv.o ../../tools/_build/obj/policy.o ../../tools/_build/obj/rollout.o \
    ../../tools/_build/obj/learner_$v.o
done
