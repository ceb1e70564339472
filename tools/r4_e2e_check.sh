# round-4 GPU call: train.py's PPO iteration and bench.py's end-to-end iteration on the same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/e2e
timeout -k 10 300 python -u -m uav_reinforcement_learning_control_amd.train --num-envs 65536 --total-timesteps 402653184 \
  --log-dir gpurun_out/e2e/logs --model-dir gpurun_out/e2e/models > gpurun_out/e2e/train.log 2>&1
echo "train rc=$?"; grep -h "^[0-9]" gpurun_out/e2e/logs/*/progress.csv | cut -d, -f1,6,7
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --rollout-steps 0 > gpurun_out/e2e/bench.txt 2>&1
echo "bench rc=$?"; python3 -c "
import json; l=[x for x in open('gpurun_out/e2e/bench.txt') if x.startswith('{')][-1]; d=json.loads(l)['end_to_end']; print({k: d[k] for k in ('rollout_s','train_s','ms_per_optimizer_step')}, d['learner_kernel']['us_per_minibatch'])"
