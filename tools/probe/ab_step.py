#!/usr/bin/env python3
"""Profiling tool (not product): A/B k_step builds. For each library (one process each; "base" =
the in-tree build): 60 steps at N envs with random actions, a digest of every step's outputs
(obs, reward, flags, terminal obs) and the final state -- which must equal base's for an exact
variant -- then graph-replayed timing (HIP events, 1,000 steps). Usage: ab_step.py N lib.so ..."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(n, lib, lanes):
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    if lib != "base":
        N.LIB_PATH = lib
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from bench import _quad_step_fn
    e = QuadVecEnv(n, device="cuda:0", seed=11)
    e.reset()
    acts = [e.random_actions(k) for k in range(16)]
    st = _quad_step_fn(e)
    h = hashlib.sha256()
    for k in range(60):
        st(acts[k % 16].data_ptr())
        done = (e.terminated | e.truncated)
        for t in (e.obs, e.reward, e.terminated, e.truncated, e.terminal_obs[done]):
            h.update(t.cpu().numpy().tobytes())
    g = e.get_state()
    for k in sorted(g):
        h.update(g[k].tobytes())
    from step_time import run
    us = sorted(run(n, steps=1000) for _ in range(3))
    print(f"{os.path.basename(lib):14s} n={n} lanes={lanes}: {us[0]:.2f} us/step (runs "
          f"{', '.join(f'{u:.2f}' for u in us)}) digest {h.hexdigest()[:16]}", flush=True)


def main():
    if sys.argv[1] == "child":
        return child(int(sys.argv[2]), sys.argv[3], sys.argv[4])
    n = sys.argv[1]
    lanes = os.environ.get("QUADENV_LANES", "0")
    for lib in ["base"] + sys.argv[2:] + ["base"]:
        r = subprocess.run([sys.executable, __file__, "child", n, lib, lanes], capture_output=True, text=True,
                           timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-400:], flush=True)


if __name__ == "__main__":
    main()
