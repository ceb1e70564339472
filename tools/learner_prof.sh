#!/bin/bash
# Profiling tool (not product): rocprofv3 kernel trace + stats of tools/learner_bench.py (quad_ppo_grad
# at 524,288 rows, the library given as $1, default the in-tree build) -> gpurun_out/lprof/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lprof
lib=${1:-}
if [ -n "$lib" ]; then export QUADENV_LIB=$lib; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof -o run -- \
  python tools/learner_bench.py 524288 8388608 30 > gpurun_out/lprof/bench.txt 2>&1
rc=$?
f=$(find gpurun_out/lprof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit $rc
