timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/pt_all.log 2>&1
r=$?; echo pytest rc=$r; grep -E "passed|failed|FAILED" gpurun_out/pt_all.log | tail -12; grep -E "^\[x3 seed" gpurun_out/pt_all.log | cut -c1-200
if [ $r -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke rc=$?; tail -2 gpurun_out/smoke.log
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo bench rc=$?; tail -c 3000 gpurun_out/bench.json
fi
