#!/bin/bash
# Round 6's evidence run (one gpurun call): GPU tests, smoke, the driver's bench command, a rocprofv3
# kernel trace of the same command, the step kernel's PMC issue and traffic passes, the learner's PMC
# passes. Each step under its own limit (tools/gpu_steps.sh); a fault / timeout ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
exec_steps=(
  tests 400 "python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread"
  smoke 200 "python -u -c 'import __graft_entry__ as g; g.smoke()'"
  bench 400 "python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final.json"
  rocprof 400 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
  issue 400 "SIZES='65536 4194304' bash tools/pmc/issue_roofline.sh"
  traffic 400 "SIZES='65536 1048576 4194304' bash tools/pmc/traffic_round.sh"
  lrnpmc 300 "bash tools/pmc/learner_pmc.sh"
)
bash tools/gpu_steps.sh "${exec_steps[@]}"
