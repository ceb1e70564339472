#!/usr/bin/env python3
"""Diagnostic: first step / env where quad_rollout and the two-launch path disagree."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_rollout as R  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy  # noqa: E402

kind, wrapper, max_steps, n, T = "hover", None, int(sys.argv[1]) if len(sys.argv) > 1 else 6, 1000, 20
seed, gamma = 0x1234_5678_9ABC, 0.97
fp = FusedPolicy(R._policy())
fp.pack()
ea, eb = R._env(n, kind, wrapper, max_steps, base=3 * n), R._env(n, kind, wrapper, max_steps, base=3 * n)
A, B = R._bufs(T, n), R._bufs(T, n)
A["last_obs"].copy_(ea.reset())
B["last_obs"].copy_(eb.reset())
R._two_launch(fp, ea, A, T, seed, gamma)
R._one_launch(fp, eb, B, T, seed, gamma, (T,))
a = {k: v.cpu().numpy() for k, v in A.items()}
b = {k: v.cpu().numpy() for k, v in B.items()}
for t in range(T):
    for k in ("obs_copy", "episode_starts", "value", "actions", "log_prob", "rewards"):
        x, y = a[k][t], b[k][t]
        d = x.view(np.uint32) != y.view(np.uint32)
        if d.any():
            envs = np.nonzero(d.reshape(n, -1).any(1))[0]
            print(f"t={t} {k}: {d.sum()} words, envs {envs[:20].tolist()} (of {len(envs)})")
            e = envs[0]
            print("   A", x[e].tolist(), "\n   B", y[e].tolist())
            if k != "obs_copy" and t > 0:
                print("   obs A", a["obs_copy"][t][e].tolist(), "\n   start", a["episode_starts"][t][e], b["episode_starts"][t][e])
            sys.exit(0)
print("identical")
