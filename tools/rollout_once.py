#!/usr/bin/env python3
"""Profiling target (not product): quad_rollout at N hover envs, T steps per launch, `reps` launches
after one warm launch (the PPO default form, k_rollout<HOVER, noCTBR, 2, SPEC>). Usage:
rollout_once.py [N] [T] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uav_reinforcement_learning_control_amd import _native as N  # noqa: E402
from uav_reinforcement_learning_control_amd.envs import QuadVecEnv  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
torch.manual_seed(0)
env = QuadVecEnv(n, env="hover", device="cuda:0", seed=1)
fp = FusedPolicy(ActorCritic().cuda())
fp.pack()
f = dict(dtype=torch.float32, device="cuda")
b = dict(obs_copy=torch.zeros(T, n, 12, **f), actions=torch.zeros(T, n, 4, **f), log_prob=torch.zeros(T, n, **f),
         value=torch.zeros(T, n, **f), episode_starts=torch.zeros(T, n, **f), rewards=torch.zeros(T, n, **f),
         last_obs=torch.zeros(n, 12, **f), last_start=torch.ones(n, **f), ep_ret=torch.zeros(n, **f),
         ep_len=torch.zeros(n, **f), stats=torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device="cuda"))
b["last_obs"].copy_(env.reset())
for r in range(reps + 1):
    fp.rollout(env, t0=T * r, steps=T, seed=1, gamma=0.99, **b)
torch.cuda.synchronize()
print("done", n, T, reps)
