#!/bin/bash
# Profiling tool (not product): cost-ablation builds of libquadenv.so for tools/rollout_variants.py --
# k_rollout without the env step, without the MLPs, without the critic. Output: tools/_build/roll_*.so
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -c -o ../../tools/_build/obj/quadenv.o quadenv.hip &
/opt/rocm/bin/hipcc $F -c -o ../../tools/_build/obj/policy.o policy.hip &
for v in NOENV NOMLP NOCRITIC; do
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize -DQD_ROLL_$v -c -o ../../tools/_build/obj/rollout_$v.o rollout.hip &
done
wait
for v in NOENV NOMLP NOCRITIC; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/roll_$v.so \
    ../../tools/_build/obj/quadenv.o ../../tools/_build/obj/policy.o ../../tools/_build/obj/rollout_$v.o
done
