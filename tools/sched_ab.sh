#!/bin/bash
# Profiling tool (not product): libquadenv.so variants whose env-kernel translation unit is built
# with other LLVM AMDGPU scheduler settings. Usage: sched_ab.sh NAME "flags" ... -> tools/_build/sch_NAME.so
set -e
cd "$(dirname "$0")/../uav_reinforcement_learning_control_amd/csrc"
make -s -j4 >/dev/null
O=../_lib/obj
mkdir -p ../../tools/_build/obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -ffp-contract=on -fno-slp-vectorize -I$O -mllvm -amdgpu-kernarg-preload-count=16"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc $F $flags -c -o ../../tools/_build/obj/sch_$name.o quadenv.hip &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_build/sch_$name.so \
     ../../tools/_build/obj/sch_$name.o $O/policy.o $O/rollout.o $O/learner.o $O/learner_x3.o) &
done
wait
