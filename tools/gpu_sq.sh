#!/bin/bash
# SQ counter passes (wave-cycle accounting) for the step-kernel forms at 65,536 envs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
for lanes in 0 1 2; do
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
    tag=$(echo $set | cut -d' ' -f1)
    echo "=== lanes=$lanes $tag"
    QUADENV_LANES=$lanes timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/l${lanes}_$tag -o sq -- python tools/lanes_sweep.py $lanes 65536 100 > $O/l${lanes}_$tag.log 2>&1
    rc=$?; echo "rc=$rc"; tail -2 $O/l${lanes}_$tag.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
