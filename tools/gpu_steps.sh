#!/bin/bash
# One gpurun call as a list of steps: gpu_steps.sh NAME TIMEOUT 'CMD' [NAME TIMEOUT 'CMD' ...]
# Each step runs under its own `timeout -k 10`, writes gpurun_out/NAME.log and prints its tail.
# Exit status 0 (ok) or 1 (test failures) continues; anything else -- a fault, abort, segfault or
# time limit -- ends the call there (no GPU step after a failed one). Replaces the round-4 one-off
# tools/r4_*.sh scripts, e.g. the driver's round-end sequence:
#   gpu_steps.sh tests 900 'python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread' \
#                smoke 300 'python -u -c "import __graft_entry__ as g; g.smoke()"' \
#                bench 600 'python -u bench.py --gpus 1 --steps 20 --warmup 5'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -ge 3 ]; do
  name=$1 to=$2 cmd=$3
  shift 3
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 8 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
done
echo "=== done"
