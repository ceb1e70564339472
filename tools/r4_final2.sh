# round-4 GPU call after the nt state policy: GPU tests, smoke(), the driver's bench command and its
# rocprofv3 trace, the counted issue roofline and PMC traffic of the timed step kernels, then the
# nt-vs-default size sweep. Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4g_tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider
step r4g_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step r4g_bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step r4g_rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
step r4g_issue 500 env SIZES="65536 1048576 4194304" bash tools/pmc/issue_roofline.sh
step r4g_traffic 500 bash tools/pmc/traffic_round.sh
echo "=== done"
