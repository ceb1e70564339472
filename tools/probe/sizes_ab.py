#!/usr/bin/env python3
"""Profiling tool (not product): the step kernel at N envs under several library / form settings,
one process each (env overrides as KEY=VAL, a library path as LIB=path). Graph-replayed launches,
HIP events (tools/step_time.run), best of 3. Usage: sizes_ab.py N "KEY=VAL ..." ["..."]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "child":
        sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
        from uav_reinforcement_learning_control_amd import _native as N
        if os.environ.get("LIB"):
            N.LIB_PATH = os.environ["LIB"]
        from step_time import run

        n = int(sys.argv[2])
        t = min(run(n, steps=400) for _ in range(3))
        dg = ""
        if os.environ.get("DIGEST"):  # every output of 40 stepped steps: forms must agree bit for bit
            import hashlib
            import torch
            from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
            e = QuadVecEnv(n, device="cuda:0", seed=3)
            e.reset()
            h = hashlib.sha256()
            for k in range(40):
                obs, rew, term, trunc, inf = e.step(e.random_actions(k))
                for x in (obs, rew, term, trunc, inf["terminal_observation"]):
                    h.update(x.cpu().numpy().tobytes())
            for v in e.get_state().values():
                h.update(v.tobytes())
            dg = " digest " + h.hexdigest()[:16]
        print(f"{sys.argv[3]:40s} n={n}: {t:.2f} us = {278 * n / t / 1e3:.0f} GB/s{dg}", flush=True)
        return
    n = sys.argv[1]
    for spec in sys.argv[2:]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "child", n, spec], capture_output=True, text=True, timeout=300, env=env)
        print(r.stdout.strip() or r.stderr.strip()[-400:], flush=True)


if __name__ == "__main__":
    main()
