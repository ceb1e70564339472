#!/bin/bash
# Profiling tool (not product): rocprofv3 PMC passes (one counter group per run) over
# tools/rollout_once.py (quad_rollout, 65,536 hover envs, 64 steps per launch) and a kernel-trace
# pass. Output: gpurun_out/ro_pmc/<pass>/ (summarize with tools/pmc/rollout_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ro_pmc
mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex k_rollout --output-format csv -d $O/p$i -o pmc -- python3 tools/rollout_once.py 65536 64 4 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -1 $O/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --kernel-include-regex k_rollout --output-format csv -d $O/trace -o t -- python3 tools/rollout_once.py 65536 64 4 > $O/trace.log 2>&1 || exit $?
echo done
