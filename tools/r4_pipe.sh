# round-4 GPU call: two pipelined half-batch streams vs one launch per step; bench's launch-floor fields
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/step_pipe2.py 65536 100 > gpurun_out/r4_pipe2.txt 2>&1
echo "pipe rc=$?"; cat gpurun_out/r4_pipe2.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --e2e-iters 0 --rollout-steps 0 > gpurun_out/r4_bench_quick.txt 2>&1
echo "bench rc=$?"; tail -c 1500 gpurun_out/r4_bench_quick.txt
