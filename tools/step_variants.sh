#!/bin/bash
# Profiling tool (not product): build cost-ablation variants of libquadenv.so for
# tools/step_variants.py -- the physics run twice / skipped, the observation (scipy Euler) skipped,
# the auto-reset branch compiled out (k_step_h), the SLP vectorizer on. Output: tools/_build/abl_*.so
# (the rollout / learner objects are the product's, from csrc/Makefile's _lib/obj)
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -mllvm -amdgpu-kernarg-preload-count=16"
O=../_lib/obj
for v in PHYS2 NOPHYS NOOBS NORESET; do
  ( /opt/rocm/bin/hipcc $F -I$O -fno-slp-vectorize -DQD_ABL_$v -c -o ../../tools/_build/obj/quadenv_$v.o quadenv.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/abl_$v.so \
      ../../tools/_build/obj/quadenv_$v.o $O/policy.o $O/rollout.o $O/learner.o ) &
done
# the product source WITH the SLP vectorizer (v_pk_* f32 packing; csrc/Makefile turns it off)
( /opt/rocm/bin/hipcc $F -I$O -c -o ../../tools/_build/obj/quadenv_SLP.o quadenv.hip &&
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/abl_SLP.so \
    ../../tools/_build/obj/quadenv_SLP.o $O/policy.o $O/rollout.o $O/learner.o ) &
wait
