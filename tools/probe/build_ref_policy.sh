#!/bin/bash
# Profiling tool (not product): libquadenv.so whose policy and rollout translation units
# (policy.hip, rollout.hip and their headers) come from git ref $2 -> tools/_build/ref_<name>.so
# (the env / learner objects from the in-tree build), for same-box A/B of the policy MLP.
# Usage: build_ref_policy.sh name git-ref
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
O=$ROOT/uav_reinforcement_learning_control_amd/_lib/obj
T=$(mktemp -d)
git -C "$ROOT" archive "$2" uav_reinforcement_learning_control_amd/csrc include | tar -x -C "$T"
make -s -C $ROOT/uav_reinforcement_learning_control_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on"
/opt/rocm/bin/hipcc $F -c -o $T/policy.o $T/uav_reinforcement_learning_control_amd/csrc/policy.hip
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -I$O -c -o $T/rollout.o $T/uav_reinforcement_learning_control_amd/csrc/rollout.hip
mkdir -p $ROOT/tools/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/_build/ref_$1.so \
  $O/quadenv.o $T/policy.o $T/rollout.o $O/learner.o $O/learner_x3.o
rm -rf "$T"
echo built tools/_build/ref_$1.so
