#!/usr/bin/env python3
"""Diagnostic (not product): where the fixed host/device overhead of bench.py's timed region goes.
The region replays one hipGraph of K step launches (65,536 envs) between two synchronizes; its wall
per step exceeds the gated kernel time by ~1 us (~20 us per 20-step region). Variants, each 60
times round-robin after warm-up, median wall per region:

  A  sync; t0; e0.record; replay; e1.record; sync; t1        (bench.py's region)
  B  sync; t0; replay; sync; t1                               (no events)
  C  sync; e0.record; t0; replay; e1.record; sync; t1         (first event outside the clock)
  D  sync; t0; hipGraphLaunch (ctypes); hipStreamSynchronize; t1
  E  sync; t0; replay; stream.synchronize(); t1

    python tools/diag/region_overhead.py [--steps 20]
"""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=60)
    a = ap.parse_args()
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = QuadVecEnv(65536, env="hover", device=dev, seed=0)
    env.reset()
    actions = [env.random_actions(k) for k in range(a.steps)]
    step = bench._quad_step_fn(env)
    g = bench._graph_of(step, actions, 0, a.steps)
    hip = C.CDLL("libamdhip64.so.7")
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    gexec = C.c_void_p(g.raw_cuda_graph_exec())
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()

    def va():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def vb():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def vc():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def vd():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hip.hipGraphLaunch(gexec, sp)
        hip.hipStreamSynchronize(sp)
        return time.perf_counter() - t0

    def ve():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        stream.synchronize()
        return time.perf_counter() - t0

    hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]

    def hev(flags):
        e = C.c_void_p()
        assert hip.hipEventCreateWithFlags(C.byref(e), flags) == 0
        return e

    fev = {0x20000000: (hev(0x20000000), hev(0x20000000)), 0x40000000: (hev(0x40000000), hev(0x40000000))}

    def vf(flags):
        def f():
            a, b = fev[flags]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hip.hipEventRecord(a, sp)
            g.replay()
            hip.hipEventRecord(b, sp)
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        return f

    vs = {"A_bench_region": va, "B_no_events": vb, "C_e0_outside": vc, "D_ctypes_launch": vd, "E_stream_sync": ve,
          "F_ev_nosysfence": vf(0x20000000), "G_ev_releasedev": vf(0x40000000)}
    res = {k: [] for k in vs}
    for _ in range(a.reps):
        for k, f in vs.items():
            res[k].append(f() * 1e6)
    kus = bench._gated_kernel_us(step, actions, 200)
    print(f"steps {a.steps}; gated kernel {kus:.3f} us -> {kus * a.steps:.1f} us of kernels per region")
    for k, v in res.items():
        m = statistics.median(v)
        print(f"{k:16s} median {m:7.1f} us/region = {m / a.steps:.3f} us/step; p10 {sorted(v)[len(v) // 10]:.1f} "
              f"p90 {sorted(v)[9 * len(v) // 10]:.1f}; overhead {m - kus * a.steps:.1f} us")
    env.close()


if __name__ == "__main__":
    main()
