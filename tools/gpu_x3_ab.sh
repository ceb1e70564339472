#!/bin/bash
# One gpurun call for a learner change (tools/_build/x3_old.so vs x3_new.so): gradient bits A/B,
# alternating timing A/B, then the learner GPU tests on the in-tree build. Each GPU step has its own
# time limit; anything but a plain failure ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step x3_bits 300 python -u tools/x3_bits_ab.py tools/_build/x3_old.so tools/_build/x3_new.so
step x3_time 500 bash tools/x3_ab_time.sh
[ -n "${X3_TESTS:-1}" ] && step learner_tests 600 python -u -m pytest tests/test_gpu_learner.py -q -rf --timeout 300 --timeout-method thread
[ -f tools/_build/lprobe.so ] && step lprobe 300 python -u tools/probe/probe_learner.py
echo "=== done"
