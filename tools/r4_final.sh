# round-4 GPU call: the driver's round-end sequence -- GPU test suite, smoke(), the bench command
# the driver runs, and the rocprofv3 kernel trace of that bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4f_tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider
step r4f_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r4f_bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
step r4f_rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo "=== done"
