#!/bin/bash
# Profiling tool (not product): libquadenv.so with a given learner_x3.hip source (and extra -D
# flags) -> tools/_build/x3_<name>.so, the other objects from the in-tree build.
# Usage: x3_build.sh name path/to/learner_x3.hip ["-DFOO"]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/uav_reinforcement_learning_control_amd/csrc
O=$ROOT/uav_reinforcement_learning_control_amd/_lib/obj
make -s -C $C
mkdir -p $ROOT/tools/_build/obj
src=$(realpath "$2")
cp "$src" $C/.x3_variant.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=on ${3:-} \
  -c -o $ROOT/tools/_build/obj/x3_$1.o $C/.x3_variant.hip
rm -f $C/.x3_variant.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/_build/x3_$1.so \
  $O/quadenv.o $O/policy.o $O/rollout.o $O/learner.o $ROOT/tools/_build/obj/x3_$1.o
echo built tools/_build/x3_$1.so
