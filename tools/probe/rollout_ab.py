#!/usr/bin/env python3
"""Profiling tool (not product): same-box A/B of whole-library builds on the rollout policy -- per
library (one process each, interleaved: base, the others, base) one quad_rollout launch of T steps
at N hover envs (k_rollout, NT = 2) and the two-launch policy kernel (k_policy_act at N envs),
HIP-event timed, best of 3. Usage: rollout_ab.py N T lib1.so [lib2.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(lib, n, T):
    sys.path.insert(0, ROOT)
    from uav_reinforcement_learning_control_amd import _native as N
    if lib != "base":
        N.LIB_PATH = lib
    import torch
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
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
    fp.rollout(env, t0=0, steps=T, seed=1, gamma=0.99, **b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    us = []
    for r in range(3):
        e0.record()
        fp.rollout(env, t0=T * (r + 1), steps=T, seed=1, gamma=0.99, **b)
        e1.record()
        torch.cuda.synchronize()
        us.append(e0.elapsed_time(e1) * 1e3 / T)
    obs = torch.rand(n, 12, **f) * 2 - 1
    act_env = torch.empty(n, 4, **f)
    pa = []
    for r in range(4):
        e0.record()
        for _ in range(20):
            fp.act(obs, act_env, deterministic=False)
        e1.record()
        torch.cuda.synchronize()
        pa.append(e0.elapsed_time(e1) * 1e3 / 20)
    print(f"{os.path.basename(lib):18s} n={n} T={T}: k_rollout {min(us):.2f} us/step   k_policy_act {min(pa[1:]):.2f} us",
          flush=True)


def main():
    if sys.argv[1] == "child":
        return child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    n, T = sys.argv[1], sys.argv[2]
    for lib in ["base"] + sys.argv[3:] + ["base"]:
        r = subprocess.run([sys.executable, __file__, "child", lib, n, T], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-600:], flush=True)


if __name__ == "__main__":
    main()
