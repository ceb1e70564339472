#!/usr/bin/env python3
"""Profiling tool (not product): k_rollout's cost by part -- the in-tree library against the
ablation builds of tools/rollout_variants.sh (no env step / no MLPs / no critic), and the 1- vs
2-tile-per-wave forms (QUADENV_ROLLOUT_NT). One quad_rollout launch of T steps at N hover envs,
HIP-event timed. Usage: rollout_variants.py [N] [T]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = [("base", "2"), ("NOENV", "2"), ("base", "2"), ("NOMLP", "2"), ("base", "2"), ("NOCRITIC", "2")]
if os.environ.get("ROLL_VARIANTS"):  # e.g. "base,NTBUF,base,NTBUF" (tools/_build/roll_<name>.so)
    VARIANTS = [tuple((v + ":2").split(":")[:2]) for v in os.environ["ROLL_VARIANTS"].split(",")]  # name[:NT]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    if len(sys.argv) > 3 and sys.argv[3] == "child":
        return child(n, T, *VARIANTS[int(sys.argv[4])])
    for k in range(len(VARIANTS)):  # one process per variant: the library is loaded once per process
        r = subprocess.run([sys.executable, __file__, str(n), str(T), "child", str(k)], capture_output=True,
                           text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-600:], flush=True)


def child(n, T, v, nt):
    os.environ["QUADENV_ROLLOUT_NT"] = nt
    from uav_reinforcement_learning_control_amd import _native as N
    if v != "base":
        N.LIB_PATH = os.path.join(ROOT, "tools", "_build", f"roll_{v}.so")
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
    print(f"{v:8s} NT={nt} n={n} T={T}: {min(us):.2f} us/step (runs {', '.join(f'{u:.2f}' for u in us)})")


if __name__ == "__main__":
    main()
