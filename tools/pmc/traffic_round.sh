#!/bin/bash
# Profiling tool (not product): HBM-side traffic of the step kernels the bench times, per kernel.
# rocprofv3 PMC passes, one counter group per run (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2, so
# they never share a pass), over tools/step_once.py (eager quad_step launches, random actions,
# auto-reset on) at 65,536 envs (k_step_h, the bench's N=1 kernel), 1,048,576 and 4,194,304 envs
# (k_step_h, 256-env blocks; k_step_hd), plus the dword-per-lane calibration copy (tools/pmc/pmc_calib.hip) whose byte count
# is known. EXTRA="<counter> ..." adds one pass per listed counter (e.g. DRAM-side TCC counters).
# tools/pmc/traffic_summary.py turns the CSVs into profiles/<round>/pmc_traffic.json.
# Every pass runs under its own time limit; a failing pass ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/traffic
mkdir -p $O
make -s -C tools/pmc _build/pmc_calib || exit 1
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
pass() {  # name counters... -- cmd
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -s KILL 90 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d $O/$name -o p -- "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi
}
for N in ${SIZES:-65536 1048576 4194304}; do
  K=$([ "$N" -ge 4194304 ] && echo 20 || echo 60)
  pass fetch_$N FETCH_SIZE -- python3 tools/step_once.py $N $K
  pass write_$N WRITE_SIZE -- python3 tools/step_once.py $N $K
  for c in ${EXTRA:-}; do pass ${c}_$N $c -- python3 tools/step_once.py $N $K; done
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --kernel-include-regex k_step --output-format csv -d $O/trace_$N -o t \
    -- python3 tools/step_once.py $N $K > $O/trace_$N.log 2>&1 || { echo "trace_$N failed"; exit 1; }
done
pass cal_fetch FETCH_SIZE -- tools/pmc/_build/pmc_calib
pass cal_write WRITE_SIZE -- tools/pmc/_build/pmc_calib
for c in ${EXTRA:-}; do pass cal_$c $c -- tools/pmc/_build/pmc_calib; done
echo done
