#!/usr/bin/env python3
"""Profiling tool (not product): where a k_ppo_grad_x3 round's time goes, from the QD_LPROBE build
(tools/probe/build_learner_probe.sh -> tools/_build/lprobe.so): per-wave s_memtime stamps of round 2
of every block, recorded through the dump build's buffer (quad_ppo_hidden). Phases:
  0-1 obs image + B1 | 1-2 L1 + H1 image | 2-3 wait at B2 | 3-4 L2 MFMAs | 4-5 head partials |
  5-6 wait at B3 | 6-7 loss terms | 7-8 dh2 + images | 8-9 wait at B4 | 9-10 dW2 (+ db2) |
  10-11 dh1 MFMAs | 11-12 relu' + dW1 (to the next round's start)
Usage: probe_learner.py [B]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = os.path.join(ROOT, "tools", "_build", "lprobe.so")
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    torch.manual_seed(0)
    pol = ActorCritic(12, 4, (128, 128)).cuda()
    M = 4 * B
    obs = torch.rand(M, 12, device="cuda") * 2 - 1
    act = torch.randn(M, 4, device="cuda") * 0.5
    lp = torch.randn(M, device="cuda") * 0.1 - 3.0
    adv = torch.randn(M, device="cuda")
    ret = torch.randn(M, device="cuda")
    idx = torch.randperm(M, device="cuda")[:B].contiguous()
    L = FusedLearner(pol, 0.2, 0.0, 0.5)
    hidden = torch.zeros(2, B, 256, device="cuda")
    names = ["obs image + B1", "L1 + H1 image", "wait at B2", "L2 MFMAs", "head partials", "wait at B3",
             "loss terms", "dh2 + images", "wait at B4", "dW2 (+ db2)", "dh1 MFMAs", "relu' + dW1"]
    for rep in range(3):
        L.grads(obs, act, lp, adv, ret, idx, hidden=hidden)
        torch.cuda.synchronize()
    st = hidden.view(-1).view(torch.int64)[: 16 * 8 * 4096].view(-1, 16).cpu().numpy()
    st = st[st[:, 0] != 0]
    for nout, nm in ((4, "actor"), (1, "critic")):
        a = st[st[:, 15] == nout].astype(np.float64)
        if len(a) == 0:
            continue
        tot = a[:, 12] - a[:, 0]
        print(f"{nm}: {len(a)} waves; round 2 median {np.median(tot):.0f} cycles (p10 {np.percentile(tot, 10):.0f}, "
              f"p90 {np.percentile(tot, 90):.0f})")
        for k, n in enumerate(names):
            d = a[:, k + 1] - a[:, k]
            print(f"    {n:24s} median {np.median(d):7.0f}  ({np.median(d) / np.median(tot) * 100:4.1f} %)")


if __name__ == "__main__":
    main()
