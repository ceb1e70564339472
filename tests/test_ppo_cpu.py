"""PPO learner pieces on CPU: SB3 policy layout/init, the loss against a NumPy restatement of
SB3 PPO.train, and the RCCL-path gradient averaging with a world-size-2 gloo group.
(SB3 is absent; learner parity is unpinned -- these pin our restatement of its semantics.)"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from uav_reinforcement_learning_control_amd.ppo import ActorCritic, PPOConfig, allreduce_mean_, ppo_loss


def test_policy_matches_sb3_layout():
    p = ActorCritic()
    names = {k: tuple(v.shape) for k, v in p.state_dict().items()}
    assert names == {
        "log_std": (4,),
        "mlp_extractor.policy_net.0.weight": (128, 12), "mlp_extractor.policy_net.0.bias": (128,),
        "mlp_extractor.policy_net.2.weight": (128, 128), "mlp_extractor.policy_net.2.bias": (128,),
        "mlp_extractor.value_net.0.weight": (128, 12), "mlp_extractor.value_net.0.bias": (128,),
        "mlp_extractor.value_net.2.weight": (128, 128), "mlp_extractor.value_net.2.bias": (128,),
        "action_net.weight": (4, 128), "action_net.bias": (4,),
        "value_net.weight": (1, 128), "value_net.bias": (1,)}
    assert sum(v.numel() for v in p.parameters()) == 37001  # actor 18,696 + critic 18,305
    # orthogonal init with SB3 gains: W W^T = gain^2 I for the wide layers
    w = p.mlp_extractor.policy_net[2].weight.detach()
    np.testing.assert_allclose((w @ w.T).numpy(), 2 * np.eye(128), atol=1e-4)
    a = p.action_net.weight.detach()
    np.testing.assert_allclose((a @ a.T).numpy(), 1e-4 * np.eye(4), atol=1e-8)
    assert torch.all(p.log_std == 0)


def test_log_prob_and_entropy_match_gaussian():
    p = ActorCritic()
    with torch.no_grad():
        p.log_std.copy_(torch.tensor([-0.5, 0.1, 0.0, 0.3]))
    mean = torch.randn(64, 4)
    a = torch.randn(64, 4)
    d = torch.distributions.Normal(mean, p.log_std.detach().exp())
    np.testing.assert_allclose(p.log_prob(mean, a).detach().numpy(), d.log_prob(a).sum(-1).numpy(),
                               rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(float(p.entropy()), float(d.entropy().sum(-1).mean()), rtol=1e-6)


def test_loss_matches_numpy_restatement_of_sb3():
    torch.manual_seed(0)
    cfg = PPOConfig()
    p = ActorCritic()
    B = 256
    obs = torch.randn(B, 12); act = torch.randn(B, 4)
    logp_old = torch.randn(B) * 0.1 - 5.7
    adv = torch.randn(B) * 3 + 1; ret = torch.randn(B)
    loss, pg, vf, ent, cf = ppo_loss(p, obs, act, logp_old, adv, ret, cfg)
    with torch.no_grad():
        mean, v = p.forward_heads(obs)
        std = p.log_std.exp().numpy()
    m = mean.detach().numpy().astype(np.float64); vv = v.detach().numpy().astype(np.float64)
    an = act.numpy().astype(np.float64)
    logp = (-0.5 * ((an - m) / std) ** 2 - np.log(std) - 0.5 * math.log(2 * math.pi)).sum(-1)
    A = adv.numpy().astype(np.float64)
    A = (A - A.mean()) / (A.std(ddof=1) + 1e-8)  # torch .std() is unbiased, as in SB3
    r = np.exp(logp - logp_old.numpy())
    c = cfg.clip_range
    pg_ref = -np.minimum(A * r, A * np.clip(r, 1 - c, 1 + c)).mean()
    vf_ref = ((ret.numpy() - vv) ** 2).mean()
    ent_ref = (0.5 + 0.5 * math.log(2 * math.pi) + np.log(std)).sum()
    np.testing.assert_allclose(float(pg), pg_ref, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(float(vf), vf_ref, rtol=1e-5)
    np.testing.assert_allclose(float(ent), ent_ref, rtol=1e-6)
    np.testing.assert_allclose(float(loss), pg_ref - cfg.ent_coef * ent_ref + 0.5 * vf_ref, rtol=1e-4)
    loss.backward()
    assert all(q.grad is not None for q in p.parameters())


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    return port


def _worker(rank, world, port, q):
    try:
        _worker_body(rank, world, port, q)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e), None))


def _worker_body(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    p = ActorCritic()  # identical init on every rank
    torch.manual_seed(100 + rank)
    obs = torch.randn(32, 12)
    mean, v = p.forward_heads(obs)
    loss = v.pow(2).mean() + mean.pow(2).mean() + (rank + 1.0) * p.log_std.pow(2).sum() + p.entropy()
    loss.backward()
    local = torch.cat([x.grad.reshape(-1) for x in p.parameters()]).clone()
    flat = torch.zeros_like(local)
    allreduce_mean_(list(p.parameters()), flat, world)
    avg = torch.cat([x.grad.reshape(-1) for x in p.parameters()])
    # the same gradient with the .grad tensors bound to the bucket: autograd accumulates into the
    # views, the all-reduce runs in place, and the result is the same average
    from uav_reinforcement_learning_control_amd.ppo.ppo import _bucket_bound, bind_grad_bucket
    params = list(p.parameters())
    bucket = torch.zeros_like(local)
    bind_grad_bucket(params, bucket)
    for x in params:
        x.grad.zero_()
    mean, v = p.forward_heads(obs)
    loss = v.pow(2).mean() + mean.pow(2).mean() + (rank + 1.0) * p.log_std.pow(2).sum() + p.entropy()
    loss.backward()
    assert _bucket_bound(params, bucket)
    assert torch.equal(bucket, local)
    allreduce_mean_(params, bucket, world)
    assert _bucket_bound(params, bucket) and torch.equal(bucket, avg)
    # broadcast_parameters_: a rank-dependent initialization ends equal to rank 0's
    from uav_reinforcement_learning_control_amd.ppo.ppo import broadcast_parameters_
    torch.manual_seed(7 + rank)
    r = ActorCritic()
    broadcast_parameters_(list(r.parameters()), 0)
    torch.manual_seed(7)
    r0 = ActorCritic()
    assert all(torch.equal(a, b) for a, b in zip(r.parameters(), r0.parameters()))
    q.put((rank, local.numpy(), avg.numpy()))
    dist.destroy_process_group()


def test_gradient_allreduce_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (l, a)) for r, l, a in (q.get(timeout=240) for _ in range(world)))
    assert all(a is not None for _, a in res.values()), res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mean = (res[0][0] + res[1][0]) / 2
    np.testing.assert_allclose(res[0][1], mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(res[1][1], mean, rtol=1e-6, atol=1e-7)


def test_split_k_linear_gradients_match_plain():
    """The split-K weight gradient (tall PPO minibatches) equals the plain one to fp32 rounding."""
    import torch.nn as nn
    from uav_reinforcement_learning_control_amd.ppo import policy as P
    torch.manual_seed(0)
    lin = nn.Linear(12, 128)
    x = torch.randn(65536 * 2, 12, requires_grad=True)
    y = P._linear(x, lin)
    assert P._chunks(x.shape[0]) == 32
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, lin.weight, lin.bias), g)
    y2 = torch.nn.functional.linear(x, lin.weight, lin.bias)
    gx2, gw2, gb2 = torch.autograd.grad(y2, (x, lin.weight, lin.bias), g)
    assert torch.equal(y, y2) and torch.allclose(gx, gx2, atol=1e-5)
    assert torch.allclose(gw, gw2, rtol=1e-4, atol=1e-3) and torch.allclose(gb, gb2, rtol=1e-4, atol=1e-3)
    assert P._chunks(100_000) == 16 and P._chunks(3) == 1


def test_cpu_ppo_baseline_runs_the_reference_loop_shape():
    """bench.py's cpu_baseline_ppo (SURVEY config 1): 16 oracle envs + CTBR through a full rollout,
    GAE and a (time-bounded, extrapolated) SB3 update on the host, one thread."""
    import bench
    r = bench._cpu_baseline_ppo(2.0)
    assert r["cores"] == 1 and r["kind"] == "port" and r["value"] > 0
    assert "16 oracle envs" in r["sample"] and "2560 Adam steps" in r["sample"]
    assert torch.get_num_threads() >= 1  # the thread count is restored


def test_minibatch_partition_is_sb3s():
    """SB3 RolloutBuffer.get(batch_size) slices indices[start:start + batch_size] for start < total:
    ceil(total / batch) minibatches, the last one short, one minibatch when batch_size >= total."""
    from uav_reinforcement_learning_control_amd.ppo.ppo import n_minibatches
    for total, batch in ((16384, 8192), (16384, 5000), (16384, 16389), (1, 128), (16 * 1024, 128), (10, 3)):
        starts = list(range(0, total, batch))
        assert n_minibatches(total, batch) == len(starts), (total, batch)
        sizes = [min(total, s + batch) - s for s in starts]
        assert sum(sizes) == total
