#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of bench.py, then separate --pmc passes
# (FETCH_SIZE, WRITE_SIZE) per step kernel via tools/pmc/traffic_round.sh.
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
# kernel trace of the bench (no end-to-end PPO iteration: its ~250k torch launches would make a
# >64 MiB trace); PMC passes on a minimal driver (tools/step_once.py: eager quad_step launches)
B="python bench.py --no-cpu-baseline --e2e-iters 0 --steps 400 --warmup 100"
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- $B
# HBM-side traffic per kernel: tools/pmc/traffic_round.sh (then tools/pmc/traffic_summary.py here)
run traffic 900 bash tools/pmc/traffic_round.sh
echo "=== done"
