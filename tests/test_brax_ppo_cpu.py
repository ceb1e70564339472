"""Brax-profile PPO pieces (ppo/brax_ppo.py) against NumPy restatements of brax's published
algorithms (brax is absent: learner parity unpinned), plus the params file round trip."""
import math

import numpy as np
import pytest
import torch

from uav_reinforcement_learning_control_amd.ppo import brax_ppo as B


def test_tanh_normal_log_prob_and_entropy():
    torch.manual_seed(0)
    d = B.NormalTanh(4)
    logits = torch.randn(64, 8, dtype=torch.float64)
    raw = torch.randn(64, 4, dtype=torch.float64) * 1.5
    loc, sraw = logits[:, :4].numpy(), logits[:, 4:].numpy()
    scale = np.log1p(np.exp(sraw)) + 0.001
    r = raw.numpy()
    ref = (-0.5 * ((r - loc) / scale) ** 2 - 0.5 * math.log(2 * math.pi) - np.log(scale)
           - np.log(1 - np.tanh(r) ** 2)).sum(-1)   # change of variables through tanh
    np.testing.assert_allclose(d.log_prob(logits, raw).numpy(), ref, rtol=1e-9, atol=1e-9)
    g = torch.Generator().manual_seed(1)
    ent = d.entropy(logits, g)
    g = torch.Generator().manual_seed(1)
    x = torch.from_numpy(loc) + torch.from_numpy(scale) * torch.randn(64, 4, dtype=torch.float64, generator=g)
    ref_e = (0.5 + 0.5 * math.log(2 * math.pi) + np.log(scale) + np.log(1 - np.tanh(x.numpy()) ** 2)).sum(-1)
    np.testing.assert_allclose(ent.numpy(), ref_e, rtol=1e-9, atol=1e-9)
    assert torch.equal(d.mode(logits), torch.tanh(logits[:, :4]))


def test_running_statistics_match_batch_moments():
    rs = B.RunningStats(5, "cpu")
    rng = np.random.default_rng(0)
    xs = [rng.normal(3.0, 2.0, (n, 5)).astype(np.float32) for n in (100, 37, 1000)]
    for x in xs:
        rs.update(torch.from_numpy(x))
    allx = np.concatenate(xs).astype(np.float64)
    assert rs.count.item() == allx.shape[0]
    np.testing.assert_allclose(rs.mean.numpy(), allx.mean(0), rtol=1e-5)
    np.testing.assert_allclose(rs.std.numpy(), allx.std(0), rtol=1e-4)
    z = rs.normalize(torch.from_numpy(xs[0]))
    np.testing.assert_allclose(z.numpy(), (xs[0] - rs.mean.numpy()) / rs.std.numpy(), rtol=1e-6)


def _np_gae(trunc, term, r, v, boot, lam, g):
    T = r.shape[0]
    tm = 1 - trunc
    vt1 = np.concatenate([v[1:], boot[None]])
    delta = (r + g * (1 - term) * vt1 - v) * tm
    acc = np.zeros_like(boot)
    out = np.zeros_like(v)
    for t in reversed(range(T)):
        acc = delta[t] + g * (1 - term[t]) * tm[t] * lam * acc
        out[t] = acc
    vs = out + v
    vs1 = np.concatenate([vs[1:], boot[None]])
    return vs, (r + g * (1 - term) * vs1 - v) * tm


def test_brax_gae_with_truncation_and_termination():
    rng = np.random.default_rng(3)
    T, Bn = 10, 64
    r = rng.normal(size=(T, Bn)); v = rng.normal(size=(T, Bn)); boot = rng.normal(size=Bn)
    done = rng.random((T, Bn)) < 0.15
    trunc = (done & (rng.random((T, Bn)) < 0.5)).astype(np.float64)
    term = (done & (trunc == 0)).astype(np.float64)
    vs, adv = B.brax_gae(*(torch.from_numpy(x) for x in (trunc, term, r, v, boot)), 0.95, 0.99)
    vs_r, adv_r = _np_gae(trunc, term, r, v, boot, 0.95, 0.99)
    np.testing.assert_allclose(vs.numpy(), vs_r, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(adv.numpy(), adv_r, rtol=1e-12, atol=1e-12)
    assert np.all(adv.numpy()[trunc == 1] == 0)  # truncated steps carry no advantage


def test_loss_terms():
    torch.manual_seed(1)
    cfg = B.BraxPPOConfig()
    net = B.BraxActorCritic(21, 4, cfg).double()
    L, Bn = 10, 32
    obs = torch.randn(L, Bn, 21, dtype=torch.float64)
    nxt = torch.randn(Bn, 21, dtype=torch.float64)
    raw = torch.randn(L, Bn, 4, dtype=torch.float64)
    with torch.no_grad():
        blp = net.dist.log_prob(net.policy(obs), raw)
    rew = torch.rand(L, Bn, dtype=torch.float64)
    disc = torch.ones(L, Bn, dtype=torch.float64)
    trunc = torch.zeros(L, Bn, dtype=torch.float64)
    total, pl, vl, el = B.brax_ppo_loss(net, obs, nxt, raw, blp, rew, disc, trunc, cfg,
                                        torch.Generator().manual_seed(0))
    # on-policy (behaviour == target): ratio 1, so the policy loss is -mean(normalized adv) = 0
    assert abs(pl.item()) < 1e-12
    with torch.no_grad():
        v = net.value(obs).squeeze(-1); bv = net.value(nxt).squeeze(-1)
    vs, _ = B.brax_gae(trunc, 1 - disc, rew, v, bv, cfg.gae_lambda, cfg.discounting)
    assert abs(vl.item() - 0.25 * ((vs - v) ** 2).mean().item()) < 1e-12
    assert abs(total.item() - (pl + vl + el).item()) < 1e-12
    total.backward()
    assert all(p.grad is not None for p in net.parameters())


def test_brax_params_file_round_trip(tmp_path):
    import pickletools
    from uav_reinforcement_learning_control_amd import export as X
    net = B.BraxActorCritic(21, 4)
    rs = B.RunningStats(21, "cpu")
    rs.update(torch.randn(50, 21))
    params = (dict(count=rs.count.numpy(), mean=rs.mean.numpy(), summed_variance=rs.summed_variance.numpy(),
                   std=rs.std.numpy()), net.policy.flax_params(), net.value.flax_params())
    path = X.save_brax_params(str(tmp_path / "ppo_params.msgpack"), params)
    raw = open(path, "rb").read()
    names = {a for op, a, _ in pickletools.genops(raw) if op.name in ("SHORT_BINUNICODE", "BINUNICODE")}
    assert {"brax.training.acme.running_statistics", "RunningStatisticsState", "hidden_0", "kernel"} <= names
    norm, pol, val = X.load_brax_params(path)
    assert norm["count"] == 50.0 and np.allclose(norm["mean"], rs.mean.numpy())
    k = pol["params"]["hidden_2"]["kernel"]
    assert k.shape == (128, 8) and k.dtype == np.float32  # flax Dense kernel is [in, out]
    net2 = B.BraxActorCritic(21, 4)
    net2.policy.load_flax_params(pol)
    net2.value.load_flax_params(val)
    x = torch.randn(7, 21)
    assert torch.equal(net.policy(x), net2.policy(x)) and torch.equal(net.value(x), net2.value(x))
