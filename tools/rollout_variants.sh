#!/bin/bash
# Profiling tool (not product): cost-ablation builds of libquadenv.so for tools/rollout_variants.py --
# k_rollout without the env step, without the MLPs, without the critic, without the obs-copy rows
# (NOOBSCOPY). (The round-4 alternatives PK0 / ALP0 were dropped from the product source in round 6.)
# Output: tools/_build/roll_*.so
# (the other objects from the in-tree build)
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
O=../_lib/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -I$O"
for v in NOENV NOMLP NOCRITIC NOOBSCOPY; do
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize -DQD_ROLL_$v -c -o ../../tools/_build/obj/rollout_$v.o rollout.hip &
done
wait
for v in NOENV NOMLP NOCRITIC NOOBSCOPY; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/roll_$v.so \
    $O/quadenv.o $O/policy.o ../../tools/_build/obj/rollout_$v.o $O/learner.o $O/learner_x3.o
done
