#!/usr/bin/env python3
"""Diagnostic (not product): does the GPU's clock state before bench.py's short timed region move
the headline? The 20-launch step region (65,536 envs) timed (wall + HIP events, bench.py's region)
after (a) 50 ms idle, (b) a 20 ms busy spin kernel, (c) a 200 ms busy spin, (d) 200 launches of
the step itself; 6 rounds round-robin, medians.

    python tools/diag/clock_state.py
"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def region(g):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6, e0.elapsed_time(e1) * 1e3


def spin_ms(ms):
    # torch.cuda._sleep spins for a cycle count; calibrate once
    torch.cuda._sleep(int(ms * 2.0e6))
    torch.cuda.synchronize()


def main():
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = QuadVecEnv(65536, env="hover", device=dev, seed=0)
    env.reset()
    actions = [env.random_actions(k) for k in range(25)]
    step = bench._quad_step_fn(env)
    g = bench._graph_of(step, actions, 5, 20)
    g200 = bench._graph_of(step, actions, 0, 200)
    g.replay(); g200.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); torch.cuda._sleep(int(2.0e7)); e1.record(); torch.cuda.synchronize()
    print(f"_sleep(2e7 cycles) = {e0.elapsed_time(e1):.2f} ms", flush=True)
    pre = {"idle_50ms": lambda: time.sleep(0.05), "spin_20ms": lambda: spin_ms(20), "spin_200ms": lambda: spin_ms(200),
           "steps_200": lambda: (g200.replay(), torch.cuda.synchronize())}
    res = {k: [] for k in pre}
    for _ in range(6):
        for k, f in pre.items():
            f()
            res[k].append(region(g))
    for k, v in res.items():
        print(f"{k:11s} wall median {statistics.median(x[0] for x in v):.1f} us, events median "
              f"{statistics.median(x[1] for x in v):.1f} us per 20-launch region (wall {', '.join(f'{x[0]:.0f}' for x in v)})")
    env.close()


if __name__ == "__main__":
    main()
