#!/bin/bash
# Profiling tool (not product): libquadenv.so with extra -D flags -> tools/_build/var_<name>.so.
# Usage: build_variant.sh name "-DFOO=1 -DBAR" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../../uav_reinforcement_learning_control_amd/csrc"
make -s
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=16"
O=../_lib/obj
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc $F -I$O $flags -c -o ../../tools/_build/obj/quadenv_var_$name.o quadenv.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/var_$name.so \
      ../../tools/_build/obj/quadenv_var_$name.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o ) &
done
wait
