#!/bin/bash
# Profiling tool (not product): the whole libquadenv.so (every translation unit) from git ref $2 ->
# tools/_build/ref_<name>.so, for digest A/Bs (tools/env_digest.py) of a refactor that touches
# headers shared by the step and rollout kernels. Usage: build_ref_full.sh name git-ref
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$2" uav_reinforcement_learning_control_amd/csrc include | tar -x -C "$T"
make -s -j4 -C $T/uav_reinforcement_learning_control_amd/csrc OUT=$T/lib/libquadenv.so
mkdir -p $ROOT/tools/_build
cp $T/lib/libquadenv.so $ROOT/tools/_build/ref_$1.so
rm -rf "$T"
echo built tools/_build/ref_$1.so
