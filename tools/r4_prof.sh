# round-4 GPU call: PMC / trace evidence of the kernels the bench times (rollout, step at 65,536 /
# 1M / 4M envs: issue roofline and HBM traffic, learner). Each pass under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4_ro_pmc 400 bash tools/pmc/rollout_pmc.sh
step r4_issue 600 env SIZES="65536 1048576 4194304" bash tools/pmc/issue_roofline.sh
step r4_traffic 600 bash tools/pmc/traffic_round.sh
step r4_lrn_pmc 300 bash tools/pmc/learner_pmc.sh
echo "=== done"
