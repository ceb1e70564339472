#!/bin/bash
# Profiling tool (not product): the step kernel's counted issue roofline. rocprofv3 PMC passes
# (one counter group per run, SQ <= 8 and GRBM <= 2 per pass) over tools/step_once.py -- eager
# quad_step launches, random actions -- at the sizes in $SIZES (default 65,536 envs: k_step_h, one
# step wave per SIMD; 1,048,576: k_step_h, 256-env blocks; 4,194,304: k_step_hd); then tools/pmc/issue_roofline.py writes
# profiles/<round>/pmc_issue.json and profiles/pmc_issue.json (read by bench.py, keyed by kernel
# symbol and env count). Every pass runs under its own time limit; a failing pass ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/issue
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for N in ${SIZES:-65536 1048576 4194304}; do
  K=$([ "$N" -ge 4194304 ] && echo 30 || echo 60)
  for set in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "k_step" --output-format csv -d $O/n$N/p$i -o sq \
      -- python3 tools/step_once.py $N $K > $O/n${N}_p$i.log 2>&1
    rc=$?; echo "N=$N pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $O/n${N}_p$i.log; exit $rc; fi
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_step" --output-format csv -d $O/trace_$N -o st \
    -- python3 tools/step_once.py $N $K > $O/trace_$N.log 2>&1 || exit $?
done
echo done
