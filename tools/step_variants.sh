#!/bin/bash
# Profiling tool (not product): build cost-ablation variants of libquadenv.so for
# tools/step_variants.py -- the physics run twice / skipped, the observation (scipy Euler) skipped,
# the auto-reset branch compiled out (k_step, QUADENV_LANES=0), the SLP vectorizer on. Output: tools/_build/abl_*.so
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
mkdir -p ../../tools/_build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function -ffp-contract=on"
for v in PHYS2 NOPHYS NOOBS NORESET; do
  /opt/rocm/bin/hipcc $F -fno-slp-vectorize -DQD_ABL_$v -o ../../tools/_build/abl_$v.so quadenv.hip policy.hip &
done
# the product source WITH the SLP vectorizer (v_pk_* f32 packing; csrc/Makefile turns it off)
/opt/rocm/bin/hipcc $F -o ../../tools/_build/abl_SLP.so quadenv.hip policy.hip &
wait
