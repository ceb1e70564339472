#!/bin/bash
# One gpurun call for the round's evidence: GPU tests, smoke, the driver's bench command, a
# rocprofv3 kernel trace of the same bench command, and the PMC issue-roofline passes. Each GPU
# step has its own time limit; a fault / abort / timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
STEPS=${STEPS:-pytest,smoke,bench,prof,pmc,lrnpmc}
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0
[[ $STEPS == *,pmc* ]] && run pmc 900 bash tools/pmc/issue_roofline.sh
[[ $STEPS == *lrnpmc* ]] && run lrnpmc 300 bash tools/pmc/learner_pmc.sh
echo "=== done"
