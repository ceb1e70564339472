#!/usr/bin/env python3
"""Rollout-phase profiling target: PPO.collect_rollouts at N envs (graph-replayed steps)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uav_reinforcement_learning_control_amd.envs import QuadVecEnv  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 32
env = QuadVecEnv(n, wrapper="RateControlWrapper", device="cuda:0")
m = PPO(env, PPOConfig(n_steps=T), seed=0)
m.collect_rollouts()
for _ in range(2):
    rs = m.collect_rollouts()
print(f"n={n} T={T}: {rs.seconds / T * 1e3:.3f} ms/step, {rs.env_steps / rs.seconds:.3e} env-steps/s")
