#!/bin/bash
# Profiling tool (not product): cost-ablation builds of libquadenv.so for tools/rollout_variants.py --
# k_rollout without the env step, without the MLPs, without the critic, without the obs-copy rows
# (NOOBSCOPY), single-FMA heads (PK0), L2-only W2 pieces (ALP0).
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
# PK0: the actor head on four v_fma_f32 per hidden value instead of two v_pk_fma_f32
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DQD_HEAD_PK=0 -c -o ../../tools/_build/obj/rollout_PK0.o rollout.hip &
# ALP0: both nets' W2 pieces from L2 (round 3) instead of the actor's from LDS
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DQD_ROLL_ALP=0 -c -o ../../tools/_build/obj/rollout_ALP0.o rollout.hip &
wait
for v in NOENV NOMLP NOCRITIC NOOBSCOPY PK0 ALP0; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/roll_$v.so \
    $O/quadenv.o $O/policy.o ../../tools/_build/obj/rollout_$v.o $O/learner.o $O/learner_x3.o
done
