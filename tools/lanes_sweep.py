#!/usr/bin/env python3
"""A/B the step-kernel forms (QUADENV_LANES = 0 legacy, 1, 2, 4) at 65,536 and 1,048,576 envs:
graph-replayed launches, HIP-event timing (same method as bench.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(lanes, n, wrapper=None, env="hover", steps=200, hover_actions=False):
    os.environ["QUADENV_LANES"] = str(lanes)
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
    g.replay(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps // 50):
        g.replay()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    e.close()
    return us


def run_split(lanes, n, splits, steps=200):
    """Step the batch as `splits` contiguous sub-ranges on `splits` streams (fork/join per step)."""
    import ctypes as C
    os.environ["QUADENV_LANES"] = str(lanes)
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    e = QuadVecEnv(n, device="cuda:0", seed=0)
    e.reset()
    acts = [e.random_actions(k) for k in range(8)]
    out = N.QuadStepOut(obs=e.obs.data_ptr(), reward=e.reward.data_ptr(),
                        terminated=e.terminated.data_ptr(), truncated=e.truncated.data_ptr(),
                        terminal_obs=e.terminal_obs.data_ptr())
    L = N.lib()
    streams = [torch.cuda.Stream() for _ in range(splits)]
    chunk = (n + splits - 1) // splits

    def step(k):
        main = torch.cuda.current_stream()
        for j, s in enumerate(streams):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                first = j * chunk
                cnt = min(chunk, n - first)
                N.check(L.quad_step_range(e._h, first, cnt, C.c_void_p(acts[k % 8].data_ptr()),
                                          C.byref(out), C.c_void_p(s.cuda_stream)), "range")
        for s in streams:
            main.wait_stream(s)
    for k in range(10):
        step(k)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(50):
            step(k)
    g.replay(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps // 50):
        g.replay()
    e1.record(); torch.cuda.synchronize()
    e.close()
    return e0.elapsed_time(e1) * 1e3 / steps


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "split":
        for lanes in (1, 0):
            for n in (65536, 1 << 20):
                for sp in (1, 2, 4):
                    us = run_split(lanes, n, sp)
                    print(f"split={sp} lanes={lanes} n={n}: {us:.2f} us/step {n / us * 1e6:.3e} env-steps/s", flush=True)
        sys.exit(0)
    if len(sys.argv) > 1:  # single config for counter runs: lanes n [steps]
        lanes, n = int(sys.argv[1]), int(sys.argv[2])
        us = run(lanes, n, steps=int(sys.argv[3]) if len(sys.argv) > 3 else 200,
                 hover_actions=len(sys.argv) > 4 and sys.argv[4] == "hover")
        print(f"lanes={lanes} n={n}: {us:.2f} us/step")
        sys.exit(0)
    res = {}
    for env, wrapper in (("hover", None), ("hover", "RateControlWrapper")):
        for n in (65536, 1 << 20):
            for lanes in (0, 1, 2, 4):
                us = run(lanes, n, wrapper, env)
                key = f"{env}{'+ctbr' if wrapper else ''} n={n} lanes={lanes}"
                res[key] = us
                print(f"{key}: {us:.2f} us/step  {n / us * 1e6:.3e} env-steps/s", flush=True)
    for lanes in (0, 1, 2):
        for n in (65536, 1 << 20):
            us = run(lanes, n, hover_actions=True)
            print(f"hover-actions (no resets) n={n} lanes={lanes}: {us:.2f} us/step", flush=True)
    json.dump(res, open("gpurun_out/lanes_sweep.json", "w"), indent=1)
