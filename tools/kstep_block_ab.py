#!/usr/bin/env python3
"""Profiling tool (not product): k_step_random_h (quad_step_random, config 2 as one launch) with 64-
vs 256-env blocks at large batches (it inherited k_step_h's h_wide policy, which goes back
to 64-env blocks from 2M envs for the nt reason that does not apply to a K-step launch).
QUADENV_HBLOCK pins the block size at handle creation; alternating, best of 3 per (size, block).
Usage: kstep_block_ab.py [N ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def rate(n, steps, block):
    os.environ["QUADENV_HBLOCK"] = str(block)
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    e = QuadVecEnv(n, env="hover", device="cuda:0", seed=0)
    e.reset()
    r = e.step_random(4, step0=0)  # warm-up (not timed)
    del r
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = e.step_random(steps, step0=4)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    del r
    e.close()
    torch.cuda.empty_cache()
    return us


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1 << 21, 1 << 22]
    for n in sizes:
        steps = max(4, min(64, (1 << 32) // (n * 48) - 1))  # time-major rows: steps * N * 48 < 2^32
        res = {64: [], 256: []}
        for _ in range(3):
            for b in (64, 256):
                res[b].append(rate(n, steps, b))
        print(json.dumps({"envs": n, "steps_per_launch": steps,
                          "us_per_step_64": sorted(res[64]), "us_per_step_256": sorted(res[256]),
                          "best_64": min(res[64]), "best_256": min(res[256])}), flush=True)


if __name__ == "__main__":
    main()
