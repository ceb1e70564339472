#!/usr/bin/env python3
"""Profiling target (not product): train.py's PPO iteration on the GPU path at its own scale (16
HoverEnv + RateControlWrapper envs x 1,024 steps, 20 epochs x 128 minibatches of 128 rows), one
warm iteration then `iters` more -- run under rocprofv3 --kernel-trace --stats to see which
launches the 2,560 graph-replayed optimizer steps of an iteration spend their time in.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/profile_small_update.py [iters]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uav_reinforcement_learning_control_amd.envs import QuadVecEnv  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
env = QuadVecEnv(envs, env="hover", wrapper="RateControlWrapper", device="cuda:0", seed=0)
m = PPO(env, PPOConfig(batch_size=128), seed=0)
m.collect_rollouts()
m.train()
torch.cuda.synchronize()
for _ in range(iters):
    t0 = time.perf_counter()
    m.collect_rollouts()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m.train()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    opt = m.cfg.n_epochs * m.n_minibatches_per_epoch()
    print(f"rollout {1e3 * (t1 - t0):.1f} ms, update {1e3 * (t2 - t1):.1f} ms = {1e6 * (t2 - t1) / opt:.1f} us "
          f"per optimizer step ({opt} steps, graph {m._epoch_graph is not None})", flush=True)
env.close()
