"""Fused PPO minibatch gradient (csrc/learner.hip, quad_ppo_grad) against torch autograd of the
SB3 loss (ppo/ppo.py `ppo_loss`) evaluated in float64 on a float64 copy of the same policy.

Tolerance: the kernel sums B per-row terms in fp32 (MFMA k-chains, then a block-order sum of the
per-block partials), so every gradient tensor must agree with the float64 gradient to
|d| <= 1e-4 * max|g_ref| + 4 * err_torch32 and to |d| <= 4 * err_torch32 + 1e-6 * max|g_ref|, where
err_torch32 is the error of torch's own fp32 autograd on the same inputs (a strongly cancelling sum
over 262,144 rows has max|g| far below the sum of |terms|, so torch's error sets the scale there).
Ratios are placed at least 1e-3 away from the clip bounds so that no implementation's rounding can
flip a clipping decision; the exact in-range tie of min(A r, A clip(r)) follows torch (half the
gradient to each side). Likewise the minibatch rows are drawn from those whose float64 hidden
pre-activations (both nets, both layers) are all at least 1e-5 away from zero: a ReLU decision on a
pre-activation within f32 rounding of zero flips between any two f32 implementations (torch fp32
included: measured 1e-4..2e-2 relative gradient differences on unfiltered 65,536 / 262,144-row
minibatches, tools/x3_diag.py), which is a discontinuity of the loss, not an accuracy statement.
Loss statistics to 1e-4 relative. test_config3_minibatch_unfiltered covers config 3's own unfiltered
524,288-row minibatch, separating the decision flips (counted from the kernel's own pre-activations)
from the arithmetic error.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _policy(seed):
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    torch.manual_seed(seed)
    pol = ActorCritic(12, 4, (128, 128)).cuda()
    with torch.no_grad():  # non-trivial biases / heads / log_std (orthogonal init leaves zeros)
        for n, p in pol.named_parameters():
            if n.endswith("bias"):
                p.copy_(torch.randn_like(p) * 0.1)
        pol.action_net.weight.mul_(30.0)
        pol.log_std.copy_(torch.tensor([-0.4, 0.1, 0.3, -1.0]))
    return pol


def _buffers(pol, M, seed, clip):
    g = torch.Generator(device="cpu").manual_seed(seed)
    obs = (torch.rand(M, 12, generator=g) * 2 - 1).cuda()
    obs[::7] *= 0.01  # rows near the origin
    with torch.no_grad():
        mean, v = pol.forward_heads(obs)
        act = mean + pol.log_std.exp() * torch.randn(M, 4, generator=g).cuda()
        lp = pol.log_prob(mean, act).double()
    # target ratios in [0.55, 1.45], at least 1e-3 away from 1 +- clip
    r = torch.rand(M, generator=g, dtype=torch.float64) * 0.9 + 0.55
    for edge in (1 - clip, 1 + clip):
        near = (r - edge).abs() < 1e-3
        r[near] = edge + torch.where(r[near] >= edge, 2e-3, -2e-3).double()
    logp_old = (lp - torch.log(r.cuda())).float()
    adv = (torch.randn(M, generator=g) * 2.0 + 0.3).cuda()
    ret = (v + torch.randn(M, generator=g).cuda()).float()
    return obs, act.contiguous(), logp_old, adv, ret


RELU_MARGIN = 1e-5


def _relu_margin(pol, x):
    """Per row: the smallest |pre-activation| of the hidden layers of both nets, in float64."""
    x = x.double()
    ex = pol.mlp_extractor
    m = torch.full((x.shape[0],), float("inf"), dtype=torch.float64, device=x.device)
    with torch.no_grad():
        for net in (ex.policy_net, ex.value_net):
            h1 = x @ net[0].weight.double().T + net[0].bias.double()
            h2 = torch.relu(h1) @ net[2].weight.double().T + net[2].bias.double()
            m = torch.minimum(m, torch.minimum(h1.abs().min(1).values, h2.abs().min(1).values))
    return m


def _index(pol, obs, M, B, seed):
    """B rows of a seeded permutation of [0, M), skipping rows with an ambiguous ReLU decision."""
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(seed)).cuda()
    perm = perm[_relu_margin(pol, obs[perm]) >= RELU_MARGIN]
    assert perm.numel() >= B
    return perm[:B].contiguous()


def _torch_grads(pol, dtype, obs, act, logp_old, adv, ret, idx, cfg):
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import ppo_loss
    from uav_reinforcement_learning_control_amd.ppo.learner import _ordered
    ref = ActorCritic(12, 4, (128, 128)).to(device=obs.device, dtype=dtype)
    ref.load_state_dict({k: v.to(dtype) for k, v in pol.state_dict().items()})
    sel = [t[idx].to(dtype) for t in (obs, act, logp_old, adv, ret)]
    loss, pg, vf, ent, cf = ppo_loss(ref, *sel, cfg)
    loss.backward()
    return [p.grad.double() for p in _ordered(ref)], torch.stack([pg, vf, ent, cf]).detach().double()


LEARNER_FORMS = {"x3": 1, "f32": 0}


@pytest.fixture(params=["x3", "f32"])
def learner_form(request, monkeypatch):
    """Both forms of quad_ppo_grad: k_ppo_grad_x3 (bf16 MFMA on three-piece splits, the default)
    and k_ppo_grad (f32-input MFMA), selected per call by QUADENV_LEARNER."""
    from uav_reinforcement_learning_control_amd import _native as N
    if request.param == "x3":
        monkeypatch.delenv("QUADENV_LEARNER", raising=False)
    else:
        monkeypatch.setenv("QUADENV_LEARNER", request.param)
    assert N.lib().quad_ppo_grad_form() == LEARNER_FORMS[request.param]
    return request.param


@pytest.mark.parametrize("M,B,norm,seed", [
    (6400, 6000, True, 0),       # most of the buffer, several blocks with ragged last rounds
    (20000, 4096 + 17, True, 1),
    (3000, 64, True, 2),         # exactly one round
    (3000, 37, False, 3),        # one partial round, no advantage normalization
    (500, 1, True, 4),           # batch 1: normalization skipped (SB3 len(adv) > 1)
    (300000, 262144, True, 5),   # many rounds per block, the 128-block cap
])
def test_fused_grad_matches_autograd(M, B, norm, seed, learner_form):
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    cfg = PPOConfig(normalize_advantage=norm)
    pol = _policy(seed)
    obs, act, logp_old, adv, ret = _buffers(pol, M, seed, cfg.clip_range)
    idx = _index(pol, obs, M, B, seed + 9)
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, norm)
    for p in pol.parameters():  # garbage in .grad: the kernel must overwrite, not accumulate
        p.grad = torch.full_like(p, 7.0)
    stats = torch.zeros(4, device="cuda")
    fl.grads(obs, act, logp_old, adv, ret, idx, stats)
    torch.cuda.synchronize()
    got = [p.grad.double() for p in _ordered(pol)]
    ref64, st64 = _torch_grads(pol, torch.float64, obs, act, logp_old, adv, ret, idx, cfg)
    ref32, _ = _torch_grads(pol, torch.float32, obs, act, logp_old, adv, ret, idx, cfg)
    names = ["pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b", "vf_w0", "vf_b0", "vf_w1", "vf_b1",
             "val_w", "val_b", "log_std"]
    bad = []
    for n, g, r64, r32 in zip(names, got, ref64, ref32):
        scale = r64.abs().max().item()
        err = (g - r64).abs().max().item()
        err32 = (r32 - r64).abs().max().item()
        tol = 1e-4 * scale + 4 * err32 + 1e-9  # (long cancelling sums: torch fp32's own error sets the bar)
        if not (err <= tol and err <= 4 * err32 + 1e-6 * scale + 1e-9):
            bad.append(f"{n}: max err {err:.3e} (scale {scale:.3e}, torch fp32 err {err32:.3e})")
    assert not bad, "; ".join(bad)
    np.testing.assert_allclose(stats.double().cpu().numpy(), st64.cpu().numpy(), rtol=1e-4, atol=1e-7)


def _pre_acts(pol, dtype, x):
    """Hidden pre-activations [2 nets][B][h1 | h2] of a copy of `pol` in `dtype` (the modules'
    own forward: for float32 the same addmm calls torch's fp32 autograd makes)."""
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    ref = ActorCritic(12, 4, (128, 128)).to(device=x.device, dtype=dtype)
    ref.load_state_dict({k: v.to(dtype) for k, v in pol.state_dict().items()})
    out = []
    with torch.no_grad():
        for net in (ref.mlp_extractor.policy_net, ref.mlp_extractor.value_net):
            h1 = net[0](x.to(dtype))
            h2 = net[2](torch.relu(h1))
            out.append(torch.cat([h1, h2], 1))
    return torch.stack(out)


class _FixedMask(torch.nn.Module):
    """ReLU with its decisions taken from another implementation: forward h * m, backward g * m
    (torch's ReLU passes the gradient where its input is > 0; here where that implementation's was)."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, h):
        return h * self.m


def _masked_grads(pol, obs, act, logp_old, adv, ret, idx, cfg, pre):
    """float64 autograd of ppo_loss with every ReLU decision taken from `pre` ([2][B][256]
    pre-activations of some implementation, minibatch order): the float64 gradient of the loss
    that implementation evaluates once its activation pattern is fixed."""
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import ppo_loss
    from uav_reinforcement_learning_control_amd.ppo.learner import _ordered
    ref = ActorCritic(12, 4, (128, 128)).to(device=obs.device, dtype=torch.float64)
    ref.load_state_dict({k: v.double() for k, v in pol.state_dict().items()})
    m = (pre > 0).double()
    for k, net in enumerate((ref.mlp_extractor.policy_net, ref.mlp_extractor.value_net)):
        net[1] = _FixedMask(m[k, :, :128])
        net[3] = _FixedMask(m[k, :, 128:])
    sel = [t[idx].double() for t in (obs, act, logp_old, adv, ret)]
    loss = ppo_loss(ref, *sel, cfg)[0]
    loss.backward()
    return [p.grad.double() for p in _ordered(ref)]


CONFIG3_MINIBATCH = 524288  # 65,536 envs x 1,024 steps / 128 minibatches


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_config3_minibatch_unfiltered(seed, learner_form):
    """quad_ppo_grad on config 3's own minibatch: 524,288 rows of a seeded permutation, NO ReLU-margin
    filter, torch fp32 autograd on the same rows as the yardstick (SB3 PPO.train as train.py:50-68
    configures it; ppo/ppo.py ppo_loss).

    Every f32 implementation puts some ReLU decisions within f32 rounding of zero on the other side
    of float64's, and ONE such flip on an influential row moves a first-layer gradient by ~1e-3 of
    max|g| (measured: the kernel and torch fp32 flip 3-5 of 268 M decisions each, with equal
    pre-activation error, yet one of the kernel's flips moved pi_w0 by 1.5e-3 while torch's moved it
    by 2e-5). So the bar separates the two error sources:
      * decisions: the kernel's own ReLU decisions (its hidden pre-activations, from the dump build
        of the same kernel body, quad_ppo_hidden) flip against float64's at most 2x as often as
        torch fp32's (+ 8 for small counts), and its pre-activation error is at most 4x torch's;
      * arithmetic: per gradient tensor, |g_kernel - G64(kernel's decisions)| <= 2 |g_torch32 -
        G64(torch32's decisions)| + 1e-6 max|g|, where G64(D) is float64 autograd of the same loss
        with the ReLU decisions D (what each implementation evaluates once its activation pattern is
        fixed). The plain errors against float64 (decisions included) are printed.
    Both forms meet that bar on every tensor. For the bf16x3 form that takes care with the hardware's
    accumulation: v_mfma_f32_32x32x16_bf16 does not round to nearest -- tails of terms far below the
    largest addend are truncated with a negative bias (profiles/r03/mfma_bf16_accumulation.txt,
    tools/diag/mfma_rounding.hip: C = 1 plus eight +2^-27 and eight -2^-27 gives 1 - 2^-24), ~1 ulp
    per MFMA. The kernel therefore keeps each product's five small-term MFMAs in their own
    accumulator (mma3s) and sums dW1 per round in fresh accumulators added with round-to-nearest
    adds; with one chain per output (round 3's first form) the forward pre-activations carried
    5.4e-7 relative error (torch fp32: 5.3e-7), vf_b1 2.6e-6 (torch 7.7e-7) and the first layer's
    gradients up to 5.6e-6 of max|g|, against 2.0e-7 and <= 2e-6 now (profiles/r03/learner_config3_unfiltered.txt).
    """
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    cfg = PPOConfig()
    pol = _policy(100 + seed)
    M, B = 600000, CONFIG3_MINIBATCH
    obs, act, logp_old, adv, ret = _buffers(pol, M, 100 + seed, cfg.clip_range)
    idx = torch.randperm(M, generator=torch.Generator().manual_seed(200 + seed))[:B].cuda().contiguous()
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, True)
    stats = torch.zeros(4, device="cuda")
    fl.grads(obs, act, logp_old, adv, ret, idx, stats)
    got = [p.grad.double().clone() for p in _ordered(pol)]
    hid = torch.empty(2, B, 256, device="cuda")
    fl.grads(obs, act, logp_old, adv, ret, idx, hidden=hid)  # the dump build: same gradients, + pre-activations
    torch.cuda.synchronize()
    for a, p in zip(got, _ordered(pol)):
        assert torch.equal(a, p.grad.double()), "the dump build must compute the production kernel's bits"
    ref64, st64 = _torch_grads(pol, torch.float64, obs, act, logp_old, adv, ret, idx, cfg)
    ref32, _ = _torch_grads(pol, torch.float32, obs, act, logp_old, adv, ret, idx, cfg)
    x = obs[idx]
    h64, h32 = _pre_acts(pol, torch.float64, x), _pre_acts(pol, torch.float32, x)
    g64_k = _masked_grads(pol, obs, act, logp_old, adv, ret, idx, cfg, hid)
    g64_t = _masked_grads(pol, obs, act, logp_old, adv, ret, idx, cfg, h32)
    names = ["pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b", "vf_w0", "vf_b0", "vf_w1", "vf_b1",
             "val_w", "val_b", "log_std"]
    rep, bad = [], []
    for n, g, r64, r32, rk, rt in zip(names, got, ref64, ref32, g64_k, g64_t):
        scale = r64.abs().max().item()
        err, err32 = (g - rk).abs().max().item(), (r32 - rt).abs().max().item()
        raw, raw32 = (g - r64).abs().max().item(), (r32 - r64).abs().max().item()
        rep.append(f"{n} {err / scale:.1e}/{err32 / scale:.1e} (raw {raw / scale:.1e}/{raw32 / scale:.1e})")
        floor = 1e-6
        if not err <= 2 * err32 + floor * scale + 1e-12:
            bad.append(f"{n}: err {err:.3e} > 2 x torch32 {err32:.3e} + {floor:g} x {scale:.3e}")
    pos64 = h64 > 0
    flips_k = int(((hid > 0) != pos64).sum())
    flips_32 = int(((h32 > 0) != pos64).sum())
    perr_k = ((hid.double() - h64).abs().max() / h64.abs().max()).item()
    perr_32 = ((h32.double() - h64).abs().max() / h64.abs().max()).item()
    print(f"\n[{learner_form} seed {seed}] ReLU flips vs float64: kernel {flips_k}, torch32 {flips_32} of "
          f"{hid.numel()}; pre-activation rel err {perr_k:.2e} / {perr_32:.2e}; gradient rel err at fixed "
          f"decisions kernel/torch32 (raw vs float64): {'; '.join(rep)}")
    assert not bad, "; ".join(bad)
    assert flips_k <= 2 * flips_32 + 8, (flips_k, flips_32)
    assert perr_k <= 4 * perr_32 + 1e-7, (perr_k, perr_32)
    np.testing.assert_allclose(stats.double().cpu().numpy(), st64.cpu().numpy(), rtol=1e-4, atol=1e-7)


def test_fused_grad_rejects_bad_arguments():
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner
    pol = _policy(0)
    obs, act, logp_old, adv, ret = _buffers(pol, 100, 0, 0.2)
    fl = FusedLearner(pol, 0.2, 0.0, 0.5)
    with pytest.raises(ValueError):
        fl.grads(obs, act, logp_old, adv, ret, torch.arange(10, device="cuda", dtype=torch.int32))
    with pytest.raises(ValueError):
        fl.grads(obs, act, logp_old, adv, ret, torch.arange(0, device="cuda"))
    with pytest.raises(ValueError):
        fl.grads(obs[:, :6].contiguous(), act, logp_old, adv, ret, torch.arange(10, device="cuda"))
    L = N.lib()
    assert L.quad_ppo_workspace_bytes(0) == 0
    assert L.quad_ppo_grad(None, None, None, None, 0, None) == N.QUAD_EINVAL


@pytest.mark.parametrize("batch_size", [None, 5000, 16384 + 5])
def test_ppo_train_fused_matches_torch_update(learner_form, batch_size):
    """One PPO.train pass with the fused gradient vs the torch loss: 2 equal minibatches; SB3's
    ragged partition (batch_size 5000 over 16,384 rows: three full minibatches and a short fourth,
    RolloutBuffer.get); and batch_size > the buffer (one minibatch of every row; the epoch
    statistics launch cannot serve it, so the gradient's own pre-pass does). Adam's first steps move
    each parameter by ~lr * sign(g), so a gradient element within fp32 noise of zero can move either
    way: allow that (<= 2 lr per step) on a small fraction of the elements, and fp32 noise elsewhere."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
    outs = []
    for fused in (True, False):
        env = QuadVecEnv(1024, env="hover", device="cuda:0", seed=3)
        cfg = PPOConfig(n_steps=16, n_minibatches=2, n_epochs=1, fused_update=fused, batch_size=batch_size)
        algo = PPO(env, cfg, seed=11)
        assert (algo._learner is not None) == fused
        algo.collect_rollouts()
        torch.manual_seed(5)  # same epoch permutation
        st = algo.train()
        outs.append(([p.detach().clone() for p in algo.policy.parameters()], st))
        env.close()
    (pa, sa), (pb, sb) = outs
    steps = {None: 2, 5000: 4, 16384 + 5: 1}[batch_size]
    assert sa["n"] == sb["n"] == steps
    lr = PPOConfig().learning_rate
    d = torch.cat([(a - b).abs().reshape(-1) for a, b in zip(pa, pb)])
    assert d.max().item() <= 2 * lr * steps + 1e-6
    assert (d > 1e-6).float().mean().item() < 0.01, f"{(d > 1e-6).sum().item()} of {d.numel()} differ"
    for k in ("pg_loss", "vf_loss", "entropy", "clip_fraction"):
        assert math.isclose(sa[k], sb[k], rel_tol=1e-3, abs_tol=1e-6), (k, sa[k], sb[k])


def test_epoch_stats_fallback_is_bit_identical(monkeypatch):
    """Past EPOCH_STATS_MAX_MINIBATCHES full minibatches per epoch the fused update skips the
    one-launch epoch statistics and every minibatch runs its own statistics pre-pass (ADVICE r04:
    the epoch launch's grid and its [nmb, 512] buffer). Both give the same statistics, so the update
    is the same bits either way (here: 3 full + 1 short minibatch, the cap lowered to 1)."""
    import uav_reinforcement_learning_control_amd.ppo.ppo as ppo_mod
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    outs = []
    for cap in (ppo_mod.EPOCH_STATS_MAX_MINIBATCHES, 1):
        monkeypatch.setattr(ppo_mod, "EPOCH_STATS_MAX_MINIBATCHES", cap)
        env = QuadVecEnv(1024, env="hover", device="cuda:0", seed=3)
        cfg = ppo_mod.PPOConfig(n_steps=16, n_epochs=2, fused_update=True, batch_size=5000)
        algo = ppo_mod.PPO(env, cfg, seed=11)
        algo.collect_rollouts()
        torch.manual_seed(5)
        st = algo.train()
        assert st["n"] == 8
        outs.append([p.detach().clone() for p in algo.policy.parameters()])
        env.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("normalize", [True, False])
def test_graph_replayed_update_is_bit_identical(normalize):
    """PPOConfig.graph_update (one GPU, minibatches tiling the buffer): each epoch's launches --
    advantage statistics + per minibatch quad_ppo_grad + quad_clip_adam -- captured once as a
    hipGraph and replayed per epoch on the epoch's permutation. The same kernels on the same data in
    the same order as the eager loop: the parameters, Adam moments and loss statistics after two
    updates (the second all replays) are the same bits. train.py's scale: 8 envs, minibatches of 128."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
    outs = []
    for graph in (True, False):
        env = QuadVecEnv(8, env="hover", wrapper="RateControlWrapper", device="cuda:0", seed=3)
        cfg = PPOConfig(n_steps=256, batch_size=128, n_epochs=3, graph_update=graph, normalize_advantage=normalize)
        algo = PPO(env, cfg, seed=11)
        torch.manual_seed(5)
        sts = []
        for _ in range(2):
            algo.collect_rollouts()
            sts.append(algo.train())
        assert (algo._epoch_graph is not None) == graph
        st = algo.opt.state
        outs.append(([p.detach().clone() for p in algo.policy.parameters()],
                     [st[p]["exp_avg_sq"].clone() for p in algo.policy.parameters()], sts))
        env.close()
    (pa, va, sa), (pb, vb, sb) = outs
    for a, b in zip(pa + va, pb + vb):
        assert torch.equal(a, b)
    assert sa == sb and sa[0]["n"] == 3 * 16


def test_graph_update_recaptures_on_resumed_state_and_new_lr():
    """The captured epoch graph holds the Adam state tensors' pointers and the learning rate as
    kernel arguments. After PPO.load_state_dict (which replaces the optimizer's state tensors) and a
    changed lr, the graph path must recapture and stay bit-identical to the eager loop: iteration 1,
    snapshot, iteration 2, load the snapshot, lr x 2, iteration 3."""
    import copy
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
    outs = []
    for graph in (True, False):
        env = QuadVecEnv(8, env="hover", wrapper="RateControlWrapper", device="cuda:0", seed=3)
        cfg = PPOConfig(n_steps=256, batch_size=128, n_epochs=2, graph_update=graph)
        algo = PPO(env, cfg, seed=11)
        torch.manual_seed(5)
        algo.collect_rollouts()
        algo.train()
        snap = copy.deepcopy(algo.state_dict())
        algo.collect_rollouts()
        algo.train()
        algo.load_state_dict(snap)
        algo.opt.param_groups[0]["lr"] *= 2.0
        algo.collect_rollouts()
        algo.train()
        assert (algo._epoch_graph is not None) == graph
        st = algo.opt.state
        outs.append([p.detach().clone() for p in algo.policy.parameters()] +
                    [st[p][k].clone() for p in algo.policy.parameters() for k in ("exp_avg", "exp_avg_sq", "step")])
        env.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("max_norm", [0.5, 1e9, 0.0])
def test_fused_clip_adam_matches_torch(max_norm):
    """quad_clip_adam (clip_grad_norm_ + Adam.step) vs torch's on identical gradients, 4 steps, on
    the optimizer's own state (step counters, moments): fp32 rounding-level agreement."""
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedAdam
    pa, pb = _policy(7), _policy(7)
    oa = torch.optim.Adam(pa.parameters(), lr=3e-3, eps=1e-5, fused=True)
    ob = torch.optim.Adam(pb.parameters(), lr=3e-3, eps=1e-5, fused=True)
    fa = FusedAdam(oa, max_norm)
    g = torch.Generator(device="cpu").manual_seed(1)
    for it in range(4):
        for p, q in zip(pa.parameters(), pb.parameters()):
            gr = (torch.randn(p.shape, generator=g) * (3.0 if it % 2 else 0.01)).cuda()
            p.grad = gr.clone()
            q.grad = gr.clone()
        fa.step()
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(list(pb.parameters()), max_norm)
        ob.step()
    torch.cuda.synchronize()
    for (n, p), q in zip(pa.named_parameters(), pb.parameters()):
        d = (p - q).abs().max().item()
        assert d <= 1e-6 * max(1.0, q.abs().max().item()), (n, d)
        assert torch.allclose(p.grad, q.grad, rtol=1e-5, atol=1e-8), n  # clipped in place as torch does
        sa, sb = oa.state[p], ob.state[q]
        assert float(sa["step"]) == float(sb["step"]) == 4.0
        assert torch.allclose(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-9), n
        assert torch.allclose(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-12), n
    # the optimizer state stays torch's: a plain torch step continues from it
    oa.step()


DP_ENVS, DP_STEPS = 2048, 64
DP_BUFFERS = ("buf_obs", "buf_act", "buf_logp", "buf_val", "buf_rew", "buf_start", "buf_adv", "buf_ret",
              "last_obs", "last_start")


def _dp_worker(rank, world, port, q):
    try:
        import os
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)  # both ranks share cuda:0 here
        from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
        from uav_reinforcement_learning_control_amd.ppo import ppo as PP
        from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
        perms, draw = [], PP.epoch_permutation

        def recorded(total, device):  # the minibatch order this rank's update used
            p = draw(total, device)
            perms.append(p.cpu().numpy())
            return p
        PP.epoch_permutation = recorded
        n = DP_ENVS
        env = QuadVecEnv(n, env="hover", device="cuda:0", seed=5, env_id_base=rank * n)
        algo = PPO(env, PPOConfig(n_steps=DP_STEPS, n_minibatches=4, n_epochs=1), seed=3)
        assert algo._learner is not None and algo.world == world
        p0 = torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()]).cpu()
        algo.collect_rollouts()
        bufs = {k: getattr(algo, k).cpu().numpy() for k in DP_BUFFERS}
        st = algo.train()
        p1 = torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()]).cpu()
        bufs["perms"] = perms
        q.put((rank, p0.numpy(), p1.numpy(), st["n"], bufs))
        env.close()
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e), None, None, None))


def test_fused_update_two_ranks_stay_in_sync():
    """Data-parallel PPO with the fused update: 2 ranks (gloo, one GPU), different env shards,
    one all-reduce per optimizer step -> identical parameters on both ranks after the update, equal
    bit for bit to one process replaying both shards' minibatches with the averaged gradient."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (a, b, n, bufs) for r, a, b, n, bufs in (q.get(timeout=240) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    assert all(b is not None for _, b, _, _ in res.values()), res
    (a0, b0, n0, _), (a1, b1, n1, _) = res[0], res[1]
    assert n0 == n1 == 4
    assert np.array_equal(a0, a1)                  # same init
    assert np.abs(b0 - a0).max() > 1e-5            # the update moved the policy
    np.testing.assert_array_equal(b0, b1)          # ... identically on both ranks
    # SURVEY 8(e) / DESIGN 5: rank r's shard is bit-identical to the same global env ids run in
    # one process -- the rollout (policy noise, auto-resets, timeout bootstraps, GAE) of the two
    # ranks concatenated equals one process stepping all 2 x DP_ENVS envs
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
    env = QuadVecEnv(2 * DP_ENVS, env="hover", device="cuda:0", seed=5, env_id_base=0)
    one = PPO(env, PPOConfig(n_steps=DP_STEPS, n_minibatches=4, n_epochs=1), seed=3)
    one.collect_rollouts()
    resets = 0
    for k in DP_BUFFERS:
        full = getattr(one, k).cpu().numpy()
        axis = 0 if k.startswith("last") else 1
        for r in range(2):
            shard = np.take(full, range(r * DP_ENVS, (r + 1) * DP_ENVS), axis=axis)
            np.testing.assert_array_equal(res[r][3][k], shard, err_msg=f"{k} rank {r}")
        if k == "buf_start":
            resets = int(full[1:].sum())
    assert resets > 0  # the window covers auto-resets
    env.close()
    # ... and the update is the mean of the shards' minibatch gradients: one process replays both
    # ranks' minibatches (their buffers, their recorded permutations) through the same learner,
    # averages the two gradients as the all-reduce does (SUM, then / world) and takes the same
    # clip + Adam step -- the parameters after the 4 optimizer steps are the ranks' bit for bit
    env = QuadVecEnv(DP_ENVS, env="hover", device="cuda:0", seed=5)
    emu = PPO(env, PPOConfig(n_steps=DP_STEPS, n_minibatches=4, n_epochs=1), seed=3)
    assert emu.world == 1 and emu._learner is not None
    dev = torch.device("cuda:0")
    shard = []
    for r in range(2):
        b = res[r][3]
        assert len(b["perms"]) == 1
        total = DP_STEPS * DP_ENVS
        shard.append(dict(obs=torch.from_numpy(b["buf_obs"]).to(dev).reshape(total, 12),
                          act=torch.from_numpy(b["buf_act"]).to(dev).reshape(total, 4),
                          logp=torch.from_numpy(b["buf_logp"]).to(dev).reshape(total),
                          adv=torch.from_numpy(b["buf_adv"]).to(dev).reshape(total),
                          ret=torch.from_numpy(b["buf_ret"]).to(dev).reshape(total),
                          perm=torch.from_numpy(b["perms"][0]).to(dev)))
    assert not torch.equal(shard[0]["perm"], shard[1]["perm"])  # each rank draws its own order
    B = emu.batch
    for m in range(4):
        g = []
        for s in shard:
            idx = s["perm"][m * B:(m + 1) * B].contiguous()
            emu._learner.grads(s["obs"], s["act"], s["logp"], s["adv"], s["ret"], idx)
            g.append(emu._flat.clone())
        emu._flat.copy_(g[0] + g[1]).div_(2)
        emu._adam.step()
    torch.cuda.synchronize()
    pe = torch.cat([p.detach().reshape(-1) for p in emu.policy.parameters()]).cpu().numpy()
    np.testing.assert_array_equal(pe, b0)
    env.close()


def test_split_kernels_match_combined(monkeypatch):
    """QUADENV_LEARNER_SPLIT=1 (one kernel per net, two streams) computes the same bits as the
    combined k_ppo_grad_x3 launch: same block slices, same arithmetic."""
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    monkeypatch.delenv("QUADENV_LEARNER", raising=False)
    cfg = PPOConfig()
    pol = _policy(11)
    obs, act, logp_old, adv, ret = _buffers(pol, 40000, 11, cfg.clip_range)
    idx = _index(pol, obs, 40000, 32768, 12)
    out = []
    for split in ("0", "1"):
        monkeypatch.setenv("QUADENV_LEARNER_SPLIT", split)
        fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, True)
        stats = torch.zeros(4, device="cuda")
        fl.grads(obs, act, logp_old, adv, ret, idx, stats)
        torch.cuda.synchronize()
        out.append(([p.grad.clone() for p in _ordered(pol)], stats.clone()))
    for a, b in zip(out[0][0], out[1][0]):
        assert torch.equal(a, b)
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("norm", [True, False])
def test_precomputed_adv_stats_are_bit_identical(norm, learner_form):
    """The data-parallel overlap (ppo/ppo.py _train_fused): quad_ppo_adv_stats for minibatch k+1 is
    enqueued while minibatch k's all-reduce is in flight, and grads(..., adv_ready=True) then skips
    its own statistics pre-pass (QUAD_ADV_PRECOMPUTED). That must give the same bits as the normal
    launch sequence -- every gradient tensor and the loss statistics -- for both learner forms; and
    the precomputed path must really read what adv_stats wrote (stats of another minibatch give a
    different gradient)."""
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig
    cfg = PPOConfig(normalize_advantage=norm)
    pol = _policy(21)
    M, B = 50000, 32768 + 77
    obs, act, logp_old, adv, ret = _buffers(pol, M, 21, cfg.clip_range)
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(3)).cuda()
    idx, other = perm[:B].contiguous(), perm[M - B:].contiguous()
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, norm)

    def run(pre, ready):
        for p in pol.parameters():
            p.grad = torch.full_like(p, 7.0)
        st = torch.zeros(4, device="cuda")
        if pre is not None:
            fl.adv_stats(adv, pre)
        fl.grads(obs, act, logp_old, adv, ret, idx, st, adv_ready=ready)
        torch.cuda.synchronize()
        return [p.grad.clone() for p in _ordered(pol)], st.clone()

    g0, s0 = run(None, False)
    g1, s1 = run(idx, True)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    assert torch.equal(s0, s1)
    g2, _ = run(other, True)  # another minibatch's mean / std
    if norm:
        assert any(not torch.equal(a, b) for a, b in zip(g0, g2))
    else:  # without normalization there are no statistics to use: the flag changes nothing
        assert all(torch.equal(a, b) for a, b in zip(g0, g2))


@pytest.mark.parametrize("norm", [True, False])
def test_epoch_adv_stats_are_bit_identical(norm, learner_form):
    """PPO.train's fused update forms every minibatch's advantage statistics of an epoch in one
    launch (quad_ppo_adv_stats_epoch) and hands minibatch m its row (QUAD_ADV_GIVEN): every gradient
    tensor and the loss statistics must equal the per-minibatch pre-pass's bits, for several
    minibatches of one permutation (including the last)."""
    from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig, epoch_permutation
    cfg = PPOConfig(normalize_advantage=norm)
    pol = _policy(23)
    M, nmb = 40000, 5
    B = M // nmb
    obs, act, logp_old, adv, ret = _buffers(pol, M, 23, cfg.clip_range)
    torch.manual_seed(4)
    perm = epoch_permutation(M, obs.device)
    fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, norm)
    sums = fl.adv_stats_epoch(adv, perm, B, nmb)
    assert (sums is None) == (not norm)
    for m in (0, 2, nmb - 1):
        idx = perm[m * B:(m + 1) * B]
        out = []
        for row in (None, None if sums is None else sums[m]):
            for p in pol.parameters():
                p.grad = torch.full_like(p, 7.0)
            st = torch.zeros(4, device="cuda")
            fl.grads(obs, act, logp_old, adv, ret, idx, st, adv_sums=row)
            torch.cuda.synchronize()
            out.append(([p.grad.clone() for p in _ordered(pol)], st.clone()))
        (g0, s0), (g1, s1) = out
        assert all(torch.equal(a, b) for a, b in zip(g0, g1)), m
        assert torch.equal(s0, s1), m
        if m == 0:
            ref0 = g0
    if norm:  # the rows differ between minibatches, and a wrong row gives a different gradient
        assert not torch.equal(sums[0], sums[1])
        fl.grads(obs, act, logp_old, adv, ret, perm[:B], None, adv_sums=sums[1])
        torch.cuda.synchronize()
        assert any(not torch.equal(p.grad, q) for p, q in zip(_ordered(pol), ref0))
