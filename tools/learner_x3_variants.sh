#!/bin/bash
# Profiling tool (not product): variant builds of k_ppo_grad_x3 (learner_x3.hip) linked with the
# in-tree objects of the other translation units. Usage: learner_x3_variants.sh NAME "-DFLAG ..." ...
# Output: tools/_build/x3_NAME.so (run tools/learner_bench.py with QUADENV_LIB=<so>)
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
make -s -j4 >/dev/null
O=../_lib/obj
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc $F $flags -c -o ../../tools/_build/obj/x3_$name.o learner_x3.hip &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/x3_$name.so \
     $O/quadenv.o $O/policy.o $O/rollout.o $O/learner.o ../../tools/_build/obj/x3_$name.o) &
done
wait
