#!/bin/bash
# Profiling tool (not product): libquadenv.so whose env translation unit (quadenv.hip and its
# headers) comes from git ref $2 -> tools/_build/ref_<name>.so (the learner / policy / rollout
# objects from the in-tree build), for same-box A/B of the step kernels against an older tree.
# Usage: build_ref_env.sh name git-ref
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
O=$ROOT/uav_reinforcement_learning_control_amd/_lib/obj
T=$(mktemp -d)
git -C "$ROOT" archive "$2" uav_reinforcement_learning_control_amd/csrc include | tar -x -C "$T"
make -s -C $ROOT/uav_reinforcement_learning_control_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -fno-slp-vectorize \
  -mllvm -amdgpu-kernarg-preload-count=16 -I$O -c -o $T/quadenv.o $T/uav_reinforcement_learning_control_amd/csrc/quadenv.hip
mkdir -p $ROOT/tools/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/_build/ref_$1.so \
  $T/quadenv.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o
rm -rf "$T"
echo built tools/_build/ref_$1.so
