#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; any exit status other than 0 (ok) or 1 (test
# failures) -- i.e. a fault, abort, segfault or timeout -- ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -x -q
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
[[ $STEPS == *sweep* ]] && run sweep 600 python tools/lanes_sweep.py
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --no-cpu-baseline --e2e-iters 0 --no-configs
echo "=== done"
