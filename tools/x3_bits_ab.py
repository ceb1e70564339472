#!/usr/bin/env python3
"""A/B tool (not product): the bits of quad_ppo_grad's gradients under each given library build --
one process per library computes every parameter's .grad on the same seeded 524,288-row minibatch
(config 3's shape, three minibatches of one permutation) and prints a SHA-256 of the gradient bytes
and the stats, so a rebuilt learner can be shown to give identical results; X3_BITS_B=128 (say)
takes minibatches of that many rows instead (the small-batch launch form). Usage:
x3_bits_ab.py lib1.so [lib2.so ...]"""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = lib
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    torch.manual_seed(0)
    cfg = PPOConfig()
    B = int(os.environ.get("X3_BITS_B", 524288))
    M = max(65536 * 32 if B == 524288 else 8 * B, 3 * B)
    pol = ActorCritic().cuda()
    g = torch.Generator(device="cuda").manual_seed(1)
    obs = torch.rand(M, 12, device="cuda", generator=g) * 2 - 1
    act = torch.randn(M, 4, device="cuda", generator=g)
    logp = torch.randn(M, device="cuda", generator=g) * 0.1 - 5.0
    adv = torch.randn(M, device="cuda", generator=g)
    ret = torch.randn(M, device="cuda", generator=g)
    perm = torch.randperm(M, device="cuda", generator=g)
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef)
    stats = torch.zeros(4, device="cuda")
    h = hashlib.sha256()
    for mb in range(3):
        fl.grads(obs, act, logp, adv, ret, perm[mb * B:(mb + 1) * B].contiguous(), stats)
        torch.cuda.synchronize()
        for p in pol.parameters():
            h.update(p.grad.detach().cpu().numpy().tobytes())
        h.update(stats.cpu().numpy().tobytes())
    print(f"{os.path.basename(lib)} (B = {B}): {h.hexdigest()[:32]}", flush=True)


def main():
    if sys.argv[1] == "child":
        child(sys.argv[2])
        return
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, __file__, "child", lib], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-400:], flush=True)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
