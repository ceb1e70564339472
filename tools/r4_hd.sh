# round-4 GPU call: k_step_hd from 4M envs -- the GPU suite, then the 4M kernel's
# PMC issue and traffic passes (its symbol changed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4_hd_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_hd_tests.log; [ $rc -eq 0 ] || exit $rc
SIZES=4194304 bash tools/pmc/issue_roofline.sh > gpurun_out/r4_hd_issue.log 2>&1 || { tail -5 gpurun_out/r4_hd_issue.log; exit 1; }
SIZES=4194304 bash tools/pmc/traffic_round.sh > gpurun_out/r4_hd_traffic.log 2>&1 || { tail -5 gpurun_out/r4_hd_traffic.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_hd_bench.log 2>&1 || { tail -5 gpurun_out/r4_hd_bench.log; exit 1; }
echo all-ok
