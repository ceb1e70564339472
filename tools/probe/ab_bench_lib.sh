#!/bin/bash
# Profiling tool (not product): the driver-shaped bench line (step part only) with the in-tree
# library vs another build (QUADENV_LIB=$1), interleaved, 4 fresh processes each
set -u
for r in 1 2 3 4; do
  for lib in base "$1"; do
    if [ "$lib" = base ]; then L=""; else L="$lib"; fi
    QUADENV_LIB=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --rollout-steps 0 --e2e-iters 0 --large-envs 0 > gpurun_out/ab_l.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_l.json'));print('$(basename $lib)', round(d['value']/1e9,3),'e9', round(d['ms_per_step']*1e3,3),'us wall', round(d['device_us_per_step'],3),'us dev', round(d['roofline']['kernel_us'],3),'us kernel')"
  done
done
