#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of bench.py, then separate --pmc passes
# (FETCH_SIZE, WRITE_SIZE) on bench.py and on the dword-copy calibration kernel.
# Any step that faults / aborts / times out ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
B="python bench.py --no-cpu-baseline --steps 400 --warmup 100"
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- $B
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o bench -- $B
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o bench -- $B
run pmc_cal_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_cal_fetch -o cal -- tools/pmc/_build/pmc_calib
run pmc_cal_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_cal_write -o cal -- tools/pmc/_build/pmc_calib
echo "=== done"
