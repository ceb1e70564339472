#!/usr/bin/env python3
"""Profiling tool (not product): where a wave's time goes in k_step (QUADENV_LANES=0), from the
QD_PROBE build (tools/probe/build.sh): per-wave s_memtime stamps at
  0 entry | 1 all loads landed | 2 control path done (CTBR, mixer, voltage) | 3 physics done |
  4 observation done | 5 reward / flags done | 6 auto-reset branch done | 7 state + obs stores issued
plus s_memrealtime (100 MHz) at entry / exit for the kernel-wide spread of wave start and end.
Usage: probe_step.py N [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    os.environ["QUADENV_LANES"] = "0"
    import ctypes as C
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = os.path.join(ROOT, "tools", "_build", "probe.so")
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    env = QuadVecEnv(n, device="cuda:0", seed=3)
    env.reset()
    acts = [env.random_actions(k) for k in range(8)]
    L = N.lib()
    stamp = torch.zeros((n + 63) // 64 * 16 + 16, dtype=torch.int64, device="cuda:0")
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
        rows.append(stamp.view(-1, 16)[: (n + 63) // 64].cpu().numpy().copy())
    a = np.concatenate(rows)
    ph = np.diff(a[:, 0:8].astype(np.float64), axis=1)
    has = a[:, 8] > 0
    words = (a[:, 8] - a[:, 5]).astype(np.float64)
    tobs = (a[:, 9] - a[:, 8]).astype(np.float64)
    rstate = (a[:, 10] - a[:, 9]).astype(np.float64)
    tail = (a[:, 6] - a[:, 10]).astype(np.float64)
    names = ["loads", "control", "physics", "observe", "reward/flags", "reset branch", "stores"]
    tot = (a[:, 7] - a[:, 0]).astype(np.float64)
    print(f"n={n}: {len(a)} wave samples; wave lifetime (s_memtime cycles) median {np.median(tot):.0f}, "
          f"p10 {np.percentile(tot, 10):.0f}, p90 {np.percentile(tot, 90):.0f}")
    for j, nm in enumerate(names):
        print(f"  {nm:14s} median {np.median(ph[:, j]):8.0f}  p10 {np.percentile(ph[:, j], 10):8.0f}  "
              f"p90 {np.percentile(ph[:, j], 90):8.0f}  mean {ph[:, j].mean():8.0f}")
    m = has & (a[:, 9] > 0)
    print(f"  reset branch detail ({m.sum()} waves with a reset; resetting lanes per wave median "
          f"{np.median(a[:, 15]):.0f}, waves with none {(a[:, 15] == 0).mean() * 100:.1f} %):")
    for nm, v in (("flags->words", words[m]), ("terminal obs", tobs[m]), ("reset state+obs", rstate[m]),
                  ("branch tail", tail[m])):
        print(f"    {nm:16s} median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    per = a.reshape(steps, -1, 16)
    for k in range(min(3, steps)):
        rt0, rt1 = per[k, :, 12].astype(np.float64), per[k, :, 13].astype(np.float64)
        print(f"  launch {k}: wave start spread {(rt0.max() - rt0.min()) * 10:.0f} ns, end spread "
              f"{(rt1.max() - rt1.min()) * 10:.0f} ns, first start -> last end {(rt1.max() - rt0.min()) * 10:.0f} ns")
    xcc = per[0, :, 14] & 0xF
    print("  waves per XCC id:", np.bincount(xcc.astype(np.int64), minlength=8).tolist())


if __name__ == "__main__":
    main()
