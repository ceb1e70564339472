#!/usr/bin/env python3
"""A/B tool (not product): SHA-256 digests of every output of the env kernels under each given
library build -- so a refactor or a schedule change can be shown to give identical bits. One
process per library: 40 quad_step launches (each step form, pinned: k_step_h in 64/256-env blocks,
the 64-env nt form, k_step_hd; hover, hover + CTBR, trajectory + CTBR) with random actions and auto-resets, every
obs / reward / flag / terminal obs and the final state; and a 32-step quad_rollout (one launch).
Usage: env_digest.py lib1.so [lib2.so ...]"""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = lib
    import torch
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    out = {}
    forms = [("h64", dict(QUADENV_HBLOCK="64", QUADENV_NT="0")),
             ("h256", dict(QUADENV_HBLOCK="256", QUADENV_NT="0")),
             ("h64nt", dict(QUADENV_HBLOCK="64", QUADENV_NT="1")),
             ("hd", dict(QUADENV_HBLOCK="64", QUADENV_NT="1", QUADENV_HD="1"))]
    for fname, envs in forms:
        for k in ("QUADENV_HBLOCK", "QUADENV_NT", "QUADENV_HD"):
            os.environ.pop(k, None)
        os.environ.update(envs)
        for kind, wrapper in (("hover", None), ("hover", "RateControlWrapper"), ("trajectory", "RateControlWrapper")):
            h = hashlib.sha256()
            e = QuadVecEnv(5000, env=kind, wrapper=wrapper, device="cuda:0", seed=3)
            h.update(e.reset().cpu().numpy().tobytes())
            for t in range(40):
                a = e.random_actions(t)
                obs, rew, te, tr, inf = e.step(a, info="full")
                for x in (obs, rew, te, tr, inf["terminal_observation"], inf["state"], inf["motor_commands"]):
                    h.update(x.cpu().numpy().tobytes())
            for k, v in sorted(e.get_state().items()):
                h.update(v.tobytes())
            e.close()
            out[f"step {fname} {kind} {wrapper}"] = h.hexdigest()[:16]
    for k in ("QUADENV_HBLOCK", "QUADENV_NT", "QUADENV_HD"):
        os.environ.pop(k, None)
    from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    torch.manual_seed(0)
    fp = FusedPolicy(ActorCritic().cuda())
    fp.pack()
    for kind, wrapper in (("hover", None), ("trajectory", "RateControlWrapper")):
        n, T = 4096, 32
        e = QuadVecEnv(n, env=kind, wrapper=wrapper, device="cuda:0", seed=5, max_episode_steps=12)
        f = dict(dtype=torch.float32, device="cuda")
        b = dict(obs_copy=torch.zeros(T, n, 12, **f), actions=torch.zeros(T, n, 4, **f),
                 log_prob=torch.zeros(T, n, **f), value=torch.zeros(T, n, **f),
                 episode_starts=torch.zeros(T, n, **f), rewards=torch.zeros(T, n, **f),
                 last_obs=torch.zeros(n, 12, **f), last_start=torch.ones(n, **f), ep_ret=torch.zeros(n, **f),
                 ep_len=torch.zeros(n, **f),
                 stats=torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device="cuda"))
        b["last_obs"].copy_(e.reset())
        fp.rollout(e, t0=0, steps=T, seed=7, gamma=0.99, **b)
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for k in sorted(b):
            if k != "stats":
                h.update(b[k].cpu().numpy().tobytes())
        for k, v in sorted(e.get_state().items()):
            h.update(v.tobytes())
        out[f"rollout {kind} {wrapper}"] = h.hexdigest()[:16]
        e.close()
    for k, v in out.items():
        print(f"{k:45s} {v}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
        sys.exit(0)
    res = {}
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, __file__, "child", lib], capture_output=True, text=True, timeout=600)
        print(f"== {lib}\n{r.stdout.strip() or r.stderr.strip()[-800:]}", flush=True)
        res[lib] = r.stdout
    vals = list(res.values())
    print("IDENTICAL" if all(v == vals[0] and v for v in vals) else "DIFFERENT")
