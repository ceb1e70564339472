#!/bin/bash
# Demonstration run (not product): train.py's defaults (HoverEnv + RateControlWrapper, SB3 PPO
# hyperparameters) at 65,536 envs on one MI355X for ~20 PPO iterations, then the batched
# deterministic evaluation of the exported SB3 archive (1,024 episodes of up to 512 steps,
# the reference's evaluate.py episode protocol). Output: gpurun_out/train_demo/
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/train_demo
mkdir -p $O
TS=${TS:-1.4e9}
timeout -k 10 400 python -u -m uav_reinforcement_learning_control_amd.train --num-envs 65536 \
  --total-timesteps $TS --log-dir $O/logs --model-dir $O/models > $O/train.log 2>&1
M=$(ls -d $O/models/*/ | tail -1)
timeout -k 10 200 python -u -m uav_reinforcement_learning_control_amd.evaluate --model ${M}hover_policy_final.zip \
  --mode episodes --num-episodes 1024 > $O/eval.log 2>&1
tail -3 $O/train.log; tail -5 $O/eval.log
