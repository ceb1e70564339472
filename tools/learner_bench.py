#!/usr/bin/env python3
"""Profiling tool (not product): one PPO minibatch optimizer step at the SB3 schedule's size
(524,288 rows of a 65,536 x 1,024 buffer) -- quad_ppo_grad alone, the fused optimizer step
(quad_ppo_grad + quad_clip_adam), and the torch autograd step (ppo_loss + backward + clip +
Adam), HIP-event timed. Usage: learner_bench.py [B] [M] [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 8 * 1024 * 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from uav_reinforcement_learning_control_amd import _native as N
    if os.environ.get("QUADENV_LIB"):  # an ablation build (tools/learner_variants.sh)
        N.LIB_PATH = os.environ["QUADENV_LIB"]
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedAdam, FusedLearner
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig, ppo_loss
    torch.manual_seed(0)
    cfg = PPOConfig()
    pol = ActorCritic().cuda()
    obs = torch.rand(M, 12, device="cuda") * 2 - 1
    act = torch.randn(M, 4, device="cuda")
    with torch.no_grad():
        mean, v = pol.forward_heads(obs[:B])
    logp = torch.randn(M, device="cuda") * 0.1 - 5.0
    adv = torch.randn(M, device="cuda")
    ret = torch.randn(M, device="cuda")
    params = list(pol.parameters())
    opt = torch.optim.Adam(params, lr=cfg.learning_rate, eps=cfg.adam_eps, fused=True)
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef)
    fadam = FusedAdam(opt, cfg.max_grad_norm)
    stats = torch.zeros(4, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    flop = 2 * B * (2 * (12 * 128 + 128 * 128) + 5 * 128) * 3  # fwd + 2x bwd, both nets

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def fused_grad():
        idx = torch.randint(0, M, (B,), device="cuda")
        fl.grads(obs, act, logp, adv, ret, idx, stats)

    def fused_step():
        fused_grad()
        fadam.step()  # quad_clip_adam

    def torch_step():
        idx = torch.randint(0, M, (B,), device="cuda")
        loss, *_ = ppo_loss(pol, obs[idx], act[idx], logp[idx], adv[idx], ret[idx], cfg)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, cfg.max_grad_norm)
        opt.step()

    t = timed(fused_grad, iters)
    print(f"B={B} M={M}: quad_ppo_grad {t * 1e3:.1f} us  ({flop / t / 1e9:.1f} TF/s nominal)", flush=True)
    if os.environ.get("QUADENV_LIB"):
        return
    print(f"fused optimizer step {timed(fused_step, iters) * 1e3:.1f} us", flush=True)
    print(f"torch optimizer step {timed(torch_step, max(3, iters // 4)) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
