#!/usr/bin/env python3
"""A/B tool (not product; round 4, profiles/r04/r4_adv_epoch_nt_ab.txt): quad_ppo_adv_stats_epoch at config 3's epoch (67,108,864 advantages, 128
minibatches of 524,288 through one quad_permutation) under each given library: device time per
launch (HIP events, 10 launches after 2 warm-up) and a digest of the sums.
Usage: adv_epoch_ab.py lib.so|in-tree ..."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    if lib != "in-tree":
        N.LIB_PATH = os.path.join(ROOT, lib)
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    cfg = PPOConfig()
    M, B, nmb = 65536 * 1024, 524288, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    adv = torch.randn(M, device="cuda", generator=g)
    perm = torch.empty(M, dtype=torch.int64, device="cuda")
    N.check(N.lib().quad_permutation(M, 7, __import__("ctypes").c_void_p(perm.data_ptr()), None), "perm")
    fl = FusedLearner(ActorCritic().cuda(), cfg.clip_range, cfg.ent_coef, cfg.vf_coef)
    out = None
    for _ in range(2):
        out = fl.adv_stats_epoch(adv, perm, B, nmb, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        out = fl.adv_stats_epoch(adv, perm, B, nmb, out)
    e1.record()
    torch.cuda.synchronize()
    d = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{os.path.basename(lib):14s} {e0.elapsed_time(e1) * 1e3 / 10:9.1f} us per epoch launch  sums {d}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "child":
        child(sys.argv[2])
        sys.exit(0)
    for rep in range(2):
        for lib in sys.argv[1:]:
            r = subprocess.run([sys.executable, __file__, "child", lib], capture_output=True, text=True, timeout=300)
            print(r.stdout.strip() or r.stderr.strip()[-500:], flush=True)
