#!/bin/bash
# Profiling tool (not product): rocprofv3 PMC passes (one counter group per run) over
# tools/learner_bench.py at the SB3-schedule minibatch (524,288 rows); QUADENV_LEARNER selects the
# kernel form. Output: gpurun_out/lrn_pmc_<form>/<pass>/ (summarize with tools/pmc/summarize.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
form=${QUADENV_LEARNER:-x3}
O=gpurun_out/lrn_pmc_$form
mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o pmc -- python tools/learner_bench.py 524288 8388608 5 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -1 $O/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
