#!/usr/bin/env python3
"""Minimal profiling target: K eager quad_step launches at N hover envs with random actions
(auto-reset on). Usage: step_once.py N K [ctbr]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import _quad_step_fn  # noqa: E402
from uav_reinforcement_learning_control_amd.envs import QuadVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
env = QuadVecEnv(n, env="hover", wrapper="RateControlWrapper" if "ctbr" in sys.argv else None,
                 device="cuda:0", seed=1)
env.reset()
acts = [env.random_actions(i) for i in range(16)]
st = _quad_step_fn(env)
for i in range(k):
    st(acts[i % 16].data_ptr())
torch.cuda.synchronize()
print("done", n, k)
