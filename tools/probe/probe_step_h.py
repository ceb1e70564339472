#!/usr/bin/env python3
"""Profiling tool (not product): where the time goes in k_step_h (one step wave + one helper wave
per SIMD), from the QD_PROBE build (tools/probe/build.sh): per-wave s_memtime stamps
  step wave:   0 entry | 1 loads landed | 2 forward_base done | 3 past barrier C | 4 mj_step done |
               5 obs / reward / flags done | 6 at barrier 1 | 7 past it | 8 reset copy + state stores
               issued, obs rows staged | 9 past barrier 2 | 10 obs rows stored
  helper wave: 0 entry | 1 loads landed | 2 control path done | 3 past barrier C | 4 reset row
               drawn | 5 past barrier 1 | 6 past barrier 2 | 10 obs rows stored
plus s_memrealtime (100 MHz) at entry / exit. Usage: probe_step_h.py N [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import ctypes as C
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = os.path.join(ROOT, "tools", "_build", "probe.so")
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    env = QuadVecEnv(n, device="cuda:0", seed=3)
    env.reset()
    acts = [env.random_actions(k) for k in range(8)]
    L = N.lib()
    hb = 64 if n <= 32768 else 256
    waves = (n + hb - 1) // hb * (2 * hb // 64)
    stamp = torch.zeros(waves * 16 + 16, dtype=torch.int64, device="cuda:0")
    plain = N.QuadStepOut(obs=env.obs.data_ptr(), reward=env.reward.data_ptr(), terminated=env.terminated.data_ptr(),
                          truncated=env.truncated.data_ptr(), terminal_obs=env.terminal_obs.data_ptr())
    probe = N.QuadStepOut(obs=env.obs.data_ptr(), reward=env.reward.data_ptr(), terminated=env.terminated.data_ptr(),
                          truncated=env.truncated.data_ptr(), terminal_obs=env.terminal_obs.data_ptr(),
                          target_info=stamp.data_ptr())
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rows = []
    for k in range(steps):
        for j in range(3):  # back-to-back like the bench: the probed launch follows plain ones
            N.check(L.quad_step(env._h, C.c_void_p(acts[(k + j) % 8].data_ptr()), C.byref(plain), s))
        N.check(L.quad_step(env._h, C.c_void_p(acts[k % 8].data_ptr()), C.byref(probe), s))
        torch.cuda.synchronize()
        rows.append(stamp.view(-1, 16)[:waves].cpu().numpy().copy())
    a = np.concatenate(rows).astype(np.float64)
    helper = a[:, 15] > 0

    def show(mask, names, idx):
        sub = a[mask]
        tot = sub[:, 10] - sub[:, 0]
        print(f"  lifetime median {np.median(tot):.0f} cycles (p10 {np.percentile(tot, 10):.0f}, p90 {np.percentile(tot, 90):.0f})")
        for nm, (i0, i1) in zip(names, idx):
            d = sub[:, i1] - sub[:, i0]
            print(f"    {nm:30s} median {np.median(d):7.0f}  p10 {np.percentile(d, 10):7.0f}  p90 {np.percentile(d, 90):7.0f}")

    print(f"n={n}: {len(a)} wave samples ({helper.sum()} helper)")
    print(" step wave:")
    show(~helper, ["loads", "forward_base", "wait at barrier C", "wrench + mj_step finish", "obs / reward / flags",
                   "to barrier 1", "wait at barrier 1", "reset copy + stores + staging", "wait at barrier 2",
                   "obs row stores"], [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, 10)])
    print(" helper wave:")
    show(helper, ["loads", "control path", "to / at barrier C", "reset draw", "wait at barrier 1",
                  "wait at barrier 2", "obs row stores"], [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 10)])
    per = a.reshape(steps, -1, 16)
    for k in range(min(3, steps)):
        rt0, rt1 = per[k, :, 12], per[k, :, 13]
        print(f"  launch {k}: wave start spread {(rt0.max() - rt0.min()) * 10:.0f} ns, end spread "
              f"{(rt1.max() - rt1.min()) * 10:.0f} ns, first start -> last end {(rt1.max() - rt0.min()) * 10:.0f} ns")


if __name__ == "__main__":
    main()
