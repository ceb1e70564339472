#!/usr/bin/env python3
"""A/B tool (not product): step-kernel variants -- library builds and/or QUADENV_* settings (round 4:
the prop-wave k_step_h, profiles/r04/r4_step_propwave_ab.txt). One process per (variant, size): 60 steps with random
actions and auto-resets hashed (obs, reward, flags, terminal obs, the final state -- an exact variant
gives base's digest), then bench.py's gated HIP-event timing of graph-replayed launches.
Variant = name=lib.so|in-tree[@VAR=VAL,...]. Usage: step_env_ab.py 4096,65536 reps variant ..."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n, spec):
    name, rest = spec.split("=", 1)
    lib, _, envs = rest.partition("@")
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v
    sys.path.insert(0, ROOT)
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    if lib != "in-tree":
        N.LIB_PATH = os.path.join(ROOT, lib)
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from bench import _gated_kernel_us, _kernel_symbol, _quad_step_fn
    # QUAD_AB_ENV / QUAD_AB_WRAPPER (a variant's @VAR=VAL settings): another env kind / wrapper
    e = QuadVecEnv(n, env=os.environ.get("QUAD_AB_ENV", "hover"), wrapper=os.environ.get("QUAD_AB_WRAPPER") or None,
                   device="cuda:0", seed=11)
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
    torch.cuda.synchronize()
    us = _gated_kernel_us(st, acts, 400)
    print(json.dumps({"variant": name, "envs": n, "kernel": _kernel_symbol(e),
                      "form": int(N.lib().quad_kernel_form(e._h)), "kernel_us": round(us, 3),
                      "digest": h.hexdigest()[:16]}), flush=True)


def main():
    if sys.argv[1] == "child":
        return child(int(sys.argv[2]), sys.argv[3])
    sizes = [int(x) for x in sys.argv[1].split(",")]
    reps = int(sys.argv[2])
    for n in sizes:
        for r in range(reps):
            for spec in sys.argv[3:]:
                p = subprocess.run([sys.executable, __file__, "child", str(n), spec], capture_output=True, text=True,
                                   timeout=300)
                print(p.stdout.strip() or p.stderr.strip()[-600:], flush=True)


if __name__ == "__main__":
    main()
