#!/usr/bin/env python3
"""Diagnostic (not product): does the FIRST replay of an uploaded step graph cost more than later
ones? bench.py times K steps as the first replay of a graph captured and uploaded (hipGraphUpload)
before the warmup; the warmup steps replay a different, W-launch graph through the same region.
Here: 8 rounds of {capture + upload a fresh 20-launch graph; warm region with a 5-launch graph;
time replay #1 of the fresh graph; time replay #2; time replay #3}, bench.py's region each time.

    python tools/diag/first_replay.py
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


def main():
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = QuadVecEnv(65536, env="hover", device=dev, seed=0)
    env.reset()
    actions = [env.random_actions(k) for k in range(25)]
    step = bench._quad_step_fn(env)
    res = {1: [], 2: [], 3: []}
    for _ in range(8):
        g = bench._graph_of(step, actions, 5, 20)
        gw = bench._graph_of(step, actions, 0, 5)
        region(gw)
        for k in (1, 2, 3):
            res[k].append(region(g))
    for k, v in res.items():
        print(f"replay #{k}: wall median {statistics.median(x[0] for x in v):.1f} us, events median "
              f"{statistics.median(x[1] for x in v):.1f} us per 20-launch region "
              f"(wall runs {', '.join(f'{x[0]:.0f}' for x in v)})")
    env.close()


if __name__ == "__main__":
    main()
