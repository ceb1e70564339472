#!/usr/bin/env python3
"""Profiling tool (not product): where the driver bench's wall clock goes beyond the device time.

Replays bench.py's timed region (synchronize, replay a K-step hipGraph, synchronize) many times
and reports the host-side split: replay() submission, the wait in synchronize, and the device
time from HIP events, under the default device schedule and under hipDeviceScheduleSpin /
hipDeviceScheduleYield / hipDeviceScheduleBlockingSync (argv[1]: auto|spin|yield|block).
Usage: python tools/probe/wall_overhead.py MODE [envs] [steps] [trials]
"""
import ctypes as C
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

MODES = {"auto": 0, "spin": 1, "yield": 2, "block": 4}


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    trials = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    if MODES[mode]:
        hip = C.CDLL("libamdhip64.so.7")
        rc = hip.hipSetDeviceFlags(C.c_uint(MODES[mode]))
        print(f"hipSetDeviceFlags({MODES[mode]}) -> {rc}")
    import bench
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = QuadVecEnv(n, env="hover", device=dev, seed=0)
    env.reset()
    acts = [env.random_actions(i) for i in range(k + 5)]
    step = bench._quad_step_fn(env)
    chunk = int(os.environ.get("CHUNK", k))  # CHUNK=5: the warmup replays the timed graph itself
    g = bench._graph_of(step, acts, 5, chunk)
    if chunk == k:
        gw = bench._graph_of(step, acts, 0, 5)
        gw.replay()
    else:
        g.replay()
    torch.cuda.synchronize()
    if os.environ.get("WARM_G") == "1":  # replay the timed graph once more before the first trial
        g.replay()
        torch.cuda.synchronize()
    spin = int(os.environ.get("SPIN_CYCLES", "0"))  # a spin kernel (no step) right before trial 0
    if spin:
        torch.cuda._sleep(spin)
        torch.cuda.synchronize()
    if os.environ.get("DRY") == "1":  # the timed region's host path once with no launches in it
        torch.cuda.synchronize()
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record()
        d1.record()
        torch.cuda.synchronize()
    if os.environ.get("EAGER") == "1":  # warm-up through the same host path (5 eager launches)
        torch.cuda.synchronize()
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record()
        for j in range(5):
            step(acts[j].data_ptr())
        d1.record()
        torch.cuda.synchronize()
    if os.environ.get("DRYG") == "1":  # ... and with the warm-up graph's steps (bench: warm-up then region)
        torch.cuda.synchronize()
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record()
        gw.replay()
        d1.record()
        torch.cuda.synchronize()
    sub, wait, wall, dev_us = [], [], [], []
    for _ in range(trials):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        if os.environ.get("EAGER") == "1":  # the K launches straight from the host, no graph
            for j in range(k):
                step(acts[(5 + j) % len(acts)].data_ptr())
        else:
            for _ in range(k // chunk):
                g.replay()
        e1.record()
        t1 = time.perf_counter()
        if os.environ.get("POLL") == "1":  # host polls the end event, then synchronizes
            while not e1.query():
                pass
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        sub.append((t1 - t0) * 1e6)
        wait.append((t2 - t1) * 1e6)
        wall.append((t2 - t0) * 1e6 / k)
        dev_us.append(e0.elapsed_time(e1) * 1e3 / k)
    med = statistics.median
    print("first trials wall/step:", " ".join(f"{w:.2f}" for w in wall[:4]),
          "| device/step:", " ".join(f"{d:.2f}" for d in dev_us[:4]))
    print(f"{mode:6s} chunk={chunk} n={n} K={k}: wall/step median {med(wall):.2f} us (min {min(wall):.2f}, max {max(wall):.2f}); "
          f"device/step {med(dev_us):.2f}; submit {med(sub):.1f} us, sync wait {med(wait):.1f} us per region")


if __name__ == "__main__":
    main()
