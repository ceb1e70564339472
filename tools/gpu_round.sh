#!/bin/bash
# One gpurun call for a round checkpoint: GPU tests, smoke, the driver's bench command, the 2-rank
# rehearsal of `bench.py --gpus 2` (gloo, both ranks on the one GPU), and a rocprofv3 kernel trace
# of the driver's bench command. STEPS selects a subset (comma list). Every GPU step has its own
# time limit; a fault / abort / segfault / timeout ends the script there (no retries).
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
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest,smoke,bench,rehearsal,prof}
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
[[ $STEPS == *rehearsal* ]] && QUAD_BENCH_REHEARSAL=1 run rehearsal 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --rollout-steps 0 --large-envs 0 --e2e-iters 1 --e2e-steps 64 --e2e-epochs 2
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0 --no-configs
echo "=== done"
