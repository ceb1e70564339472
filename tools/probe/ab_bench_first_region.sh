#!/bin/bash
# Profiling tool (not product): the driver-shaped bench line, bench.py vs a previous bench_prev.py, 3 fresh processes each
set -u
for r in 1 2 3; do
  for b in bench.py bench_prev.py; do  # bench_prev.py: git show 45e13bc:bench.py > bench_prev.py
    timeout -k 10 200 python $b --gpus 1 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --rollout-steps 0 --e2e-iters 0 --large-envs 0 > gpurun_out/ab_b.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_b.json'));print('$b', round(d['value']/1e9,3),'e9', round(d['ms_per_step']*1e3,3),'us wall', round(d['device_us_per_step'],3),'us dev', round(d['roofline']['kernel_us'],3),'us kernel')"
  done
done
