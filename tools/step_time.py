#!/usr/bin/env python3
"""Profiling tool (not product): graph-replayed quad_step time at one batch size (the size's default
kernel form; QUADENV_HBLOCK / QUADENV_NT / QUADENV_HD pin it), HIP events -- the same method as
bench.py. Imported by the A/B tools (lib_ab, lib_digest_ab, sched_ab, step_sizes, probe/*)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(n, wrapper=None, env="hover", steps=200, hover_actions=False):
    """Microseconds per step launch at n envs, averaged over `steps` graph-replayed launches."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from bench import _quad_step_fn
    e = QuadVecEnv(n, env=env, wrapper=wrapper, device="cuda:0", seed=0)
    e.reset()
    acts = [e.random_actions(k) for k in range(8)]
    if hover_actions:  # thrust ~ hover, tiny torques: (almost) no terminations -> no resets
        acts = [(a * 0.002 + torch.tensor([-0.9164, 0, 0, 0], device=a.device)).contiguous() for a in acts]
    st = _quad_step_fn(e)
    for k in range(20):
        st(acts[k % 8].data_ptr())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(50):
            st(acts[k % 8].data_ptr())
    g.replay()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(max(1, steps // 50)):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (max(1, steps // 50) * 50)
    e.close()
    return us
