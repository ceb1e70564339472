# round-4 GPU call: the driver's bench command and its rocprofv3 trace on the final code (with the
# PMC records of the timed kernels in profiles/), then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step r4h_bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step r4h_rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
step r4h_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
echo "=== done"
