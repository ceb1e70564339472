#!/usr/bin/env python3
"""A/B tool (not product): the 65,536-env step as ONE launch per step (bench.py's form) vs two
independent half-batches on two streams, each half's steps chained on its own stream (no per-step
join: half A's step t + 1 may run beside half B's step t -- the envs are independent), both chains
captured into one graph (fork at the start, join at the end). Per-step device time over K steps,
HIP events, and a digest of the final state and last outputs (the two forms must agree).
Usage: step_pipe2.py [N] [K] [QUADENV_HBLOCK for the halves]"""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, K, mode, hblock):
    if hblock:
        os.environ["QUADENV_HBLOCK"] = hblock
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from bench import _graph_upload
    L = N.lib()
    e = QuadVecEnv(n, device="cuda:0", seed=11)
    e.reset()
    acts = [e.random_actions(k) for k in range(16)]
    out = N.QuadStepOut(obs=e.obs.data_ptr(), reward=e.reward.data_ptr(), terminated=e.terminated.data_ptr(),
                        truncated=e.truncated.data_ptr(), terminal_obs=e.terminal_obs.data_ptr())
    h = e._h
    half = n // 2
    s_main = torch.cuda.Stream()
    s_b = torch.cuda.Stream()

    def capture():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s_main):
            with torch.cuda.graph(g, stream=s_main):
                cur = torch.cuda.current_stream()
                if mode == "one":
                    for k in range(K):
                        N.check(L.quad_step(h, C.c_void_p(acts[k % 16].data_ptr()), C.byref(out),
                                            C.c_void_p(cur.cuda_stream)), "quad_step")
                else:
                    s_b.wait_stream(cur)
                    for k in range(K):
                        N.check(L.quad_step_range(h, 0, half, C.c_void_p(acts[k % 16].data_ptr()), C.byref(out),
                                                  C.c_void_p(cur.cuda_stream)), "range A")
                    with torch.cuda.stream(s_b):
                        for k in range(K):
                            N.check(L.quad_step_range(h, half, n - half, C.c_void_p(acts[k % 16].data_ptr()),
                                                      C.byref(out), C.c_void_p(s_b.cuda_stream)), "range B")
                    cur.wait_stream(s_b)
        _graph_upload(g)
        return g

    g = capture()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    with torch.cuda.stream(s_main):
        torch.cuda._sleep(200_000)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * K)
    hh = hashlib.sha256()
    for t in (e.obs, e.reward, e.terminated, e.truncated):
        hh.update(t.cpu().numpy().tobytes())
    for k, v in sorted(e.get_state().items()):
        hh.update(v.tobytes())
    return us, hh.hexdigest()[:16]


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        us, d = run(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else "")
        print(json.dumps({"envs": int(sys.argv[2]), "K": int(sys.argv[3]), "mode": sys.argv[4],
                          "hblock": sys.argv[5] if len(sys.argv) > 5 else "", "us_per_step": round(us, 3), "digest": d}),
              flush=True)
        sys.exit(0)
    import subprocess
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    for rep in range(2):
        for mode, hb in (("one", ""), ("two", ""), ("two", "256"), ("two", "64")):
            r = subprocess.run([sys.executable, __file__, "child", str(n), str(K), mode, hb], capture_output=True,
                               text=True, timeout=300)
            print(r.stdout.strip() or r.stderr.strip()[-600:], flush=True)
