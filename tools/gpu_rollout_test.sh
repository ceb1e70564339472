#!/bin/bash
# GPU check of the fused rollout + the ragged auto-reset regression (one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rollout.py \
  "tests/test_gpu_parity.py::test_ragged_mass_auto_reset_draws" > gpurun_out/rollout_test.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/rollout_test.log | tail -30; echo "rc=$rc"
exit $rc
