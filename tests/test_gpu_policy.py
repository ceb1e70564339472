"""MFMA rollout-policy kernels (csrc/policy.hip) against the torch fp32 ActorCritic.

Tolerances: the kernels accumulate in fp32 in a different order than hipBLASLt, so means and
values agree to |d| <= 2e-5 * (1 + |ref|) (fp32, K = 12 and 128 dot products of O(1) terms);
sampled actions are checked against mean + std * z with z restated from the oracle's Philox and
float64 Box-Muller (|d| <= 1e-5 * (1 + |a|)); integer-like outputs (rows, counters, flags) exactly.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 2e-5


def _policy(seed=0, log_std=(-0.3, 0.1, 0.4, -1.0)):
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    torch.manual_seed(seed)
    pol = ActorCritic(12, 4, (128, 128)).cuda()
    with torch.no_grad():  # asymmetric, non-trivial weights: every layout error shows up
        for p in pol.parameters():
            p.copy_(torch.randn_like(p) * (1.0 / math.sqrt(max(p.shape[-1], 1))))
        pol.log_std.copy_(torch.tensor(log_std))
    return pol


def _ref(pol, obs):
    with torch.no_grad():
        return pol.forward_heads(obs)


def _fused(pol):
    from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy
    fp = FusedPolicy(pol)
    fp.pack()
    return fp


def _close(got, want, tol=TOL):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want) / (1.0 + np.abs(want))
    assert err.max() <= tol, (err.max(), np.unravel_index(err.argmax(), err.shape))


@pytest.mark.parametrize("n", [1, 31, 1000, 100_003])
def test_deterministic_mean_and_value_match_torch(n):
    pol = _policy(1)
    fp = _fused(pol)
    obs = torch.rand(n, 12, device="cuda") * 2 - 1
    act_env = torch.empty(n, 4, device="cuda")
    act = torch.empty(1, n, 4, device="cuda")
    val = torch.empty(1, n, device="cuda")
    fp.act(obs, act_env, actions=act, value=val, deterministic=True)
    mean, v = _ref(pol, obs)
    _close(act[0].cpu(), mean.cpu())
    _close(val[0].cpu(), v.cpu())
    assert torch.equal(act_env, act[0].clamp(-1, 1))


def test_identity_like_weights_exact():
    """W1 picks obs features, W2 = I, heads pick neurons: the MFMA chain must reproduce obs
    exactly (every product is x * 1 or x * 0), which pins the fragment layouts bit for bit."""
    pol = _policy(2, log_std=(0, 0, 0, 0))
    ex = pol.mlp_extractor
    with torch.no_grad():
        for net in (ex.policy_net, ex.value_net):
            w0 = torch.zeros(128, 12)
            for i in range(12):
                w0[i, i] = 1.0          # neuron i = relu(obs_i)
                w0[64 + i, i] = -1.0    # neuron 64+i = relu(-obs_i)
            net[0].weight.copy_(w0)
            net[0].bias.zero_()
            net[2].weight.copy_(torch.eye(128))
            net[2].bias.zero_()
        wa = torch.zeros(4, 128)
        for j, f in enumerate((3, 7, 0, 11)):
            wa[j, f], wa[j, 64 + f] = 1.0, -1.0   # relu(x) - relu(-x) = x
        pol.action_net.weight.copy_(wa)
        pol.action_net.bias.zero_()
        wv = torch.zeros(1, 128)
        wv[0, 5], wv[0, 69] = 1.0, -1.0
        pol.value_net.weight.copy_(wv)
        pol.value_net.bias.copy_(torch.tensor([0.25]))
    pol = pol.cuda()
    fp = _fused(pol)
    n = 256
    obs = torch.rand(n, 12, device="cuda") * 2 - 1
    act_env = torch.empty(n, 4, device="cuda")
    act = torch.empty(1, n, 4, device="cuda")
    val = torch.empty(1, n, device="cuda")
    fp.act(obs, act_env, actions=act, value=val, deterministic=True)
    assert torch.equal(act[0], obs[:, [3, 7, 0, 11]])
    assert torch.equal(val[0], obs[:, 5] + 0.25)


def _z_ref(seed, gid, t):
    from oracle import oracle as O
    c = O.philox([gid & 0xFFFFFFFF, gid >> 32, t, 0x200], [seed & 0xFFFFFFFF, seed >> 32])
    z = []
    for k in range(2):
        u1 = ((c[2 * k] >> 8) + 1.0) * 2.0 ** -24
        u2 = (c[2 * k + 1] >> 8) * 2.0 ** -24
        r = math.sqrt(-2.0 * math.log(u1))
        z += [r * math.cos(2 * math.pi * u2), r * math.sin(2 * math.pi * u2)]
    return z


def test_sampled_actions_logp_and_rows():
    pol = _policy(3)
    fp = _fused(pol)
    n, T, seed, base = 300, 5, 0x1234_5678_9ABC, 1 << 33
    obs = torch.rand(n, 12, device="cuda") * 2 - 1
    act_env = torch.empty(n, 4, device="cuda")
    buf = dict(actions=torch.full((T, n, 4), 7.0, device="cuda"),
               log_prob=torch.full((T, n), 7.0, device="cuda"),
               value=torch.full((T, n), 7.0, device="cuda"),
               obs_copy=torch.full((T, n, 12), 7.0, device="cuda"),
               episode_starts=torch.full((T, n), 7.0, device="cuda"))
    last_start = (torch.arange(n, device="cuda") % 3 == 0).float()
    t = 7  # row 7 % 5 = 2
    cur = torch.tensor([t, 0, 0, 0], dtype=torch.int32, device="cuda")
    fp.act(obs, act_env, last_start=last_start, cursor=cur, rows=T, seed=seed, env_id_base=base, **buf)
    assert cur.tolist() == [t, 0, 0, 0]  # read-only without an epilogue
    row = t % T
    for k, b in buf.items():  # other rows untouched
        others = torch.cat([b[:row], b[row + 1:]])
        assert torch.all(others == 7.0), k
    assert torch.equal(buf["obs_copy"][row], obs)
    assert torch.equal(buf["episode_starts"][row], last_start)
    mean, v = _ref(pol, obs)
    _close(buf["value"][row].cpu(), v.cpu())
    a = buf["actions"][row].cpu().numpy().astype(np.float64)
    std = np.exp(pol.log_std.detach().cpu().numpy().astype(np.float64))
    z = np.array([_z_ref(seed, base + i, t) for i in range(n)])
    want = mean.cpu().numpy() + std * z
    _close(a, want, 1e-5)
    with torch.no_grad():
        lp_t = pol.log_prob(mean, buf["actions"][row])
    _close(buf["log_prob"][row].cpu(), lp_t.cpu(), 1e-5)
    assert torch.equal(act_env, buf["actions"][row].clamp(-1, 1))
    # the noise is a standard normal: loose moment checks on a bigger draw
    n2 = 65536
    obs2 = torch.zeros(n2, 12, device="cuda")
    a2 = torch.empty(1, n2, 4, device="cuda")
    fp.act(obs2, torch.empty(n2, 4, device="cuda"), actions=a2, seed=9)
    m2, _ = _ref(pol, obs2)
    z2 = ((a2[0] - m2) / pol.log_std.detach().exp()).double()
    assert abs(z2.mean().item()) < 0.01 and abs(z2.std().item() - 1) < 0.01
    assert abs((z2 ** 4).mean().item() - 3) < 0.1


def _epi_case(n, g):
    rew = torch.rand(n, device="cuda", generator=g)
    term = torch.rand(n, device="cuda", generator=g) < 0.05
    trunc = torch.zeros(n, dtype=torch.bool, device="cuda")
    trunc[1000:1040] = True          # a block of timeouts (some tiles need the critic)
    trunc[4990] = True
    term[1010] = True                # terminated and truncated: no bootstrap
    tobs = torch.rand(n, 12, device="cuda", generator=g) * 2 - 1
    return rew, term, trunc, tobs


@pytest.mark.parametrize("fused", [True, False], ids=["in_act", "post"])
def test_epilogue_bootstrap_stats_and_cursor(fused):
    from uav_reinforcement_learning_control_amd import _native as N
    pol = _policy(4)
    fp = _fused(pol)
    n, T, gamma = 5000, 4, 0.99
    g = torch.Generator(device="cuda").manual_seed(5)
    rew, term, trunc, tobs = _epi_case(n, g)
    buf_rew = torch.full((T, n), -5.0, device="cuda")
    last_start = torch.full((n,), 9.0, device="cuda")
    ep_ret = torch.rand(n, device="cuda", generator=g) * 10
    ep_len = torch.randint(0, 100, (n,), device="cuda", generator=g).float()
    slots = torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device="cuda")
    cur = torch.tensor([7, 1, 0, 0], dtype=torch.int32, device="cuda")  # step 6 pending
    ret0, len0 = ep_ret.clone(), ep_len.clone()
    epi = fp.make_epilogue(rew, term, trunc, tobs, buf_rew, last_start, ep_ret, ep_len, slots, T, gamma)
    obs = torch.rand(n, 12, device="cuda") * 2 - 1
    starts = torch.full((T, n), -1.0, device="cuda")
    if fused:
        fp.act(obs, torch.empty(n, 4, device="cuda"), last_start=last_start, episode_starts=starts,
               cursor=cur, rows=T, epilogue=epi)
        assert cur.tolist() == [8, 1, 0, 0]
    else:
        fp.post(epi, cur)
        assert cur.tolist() == [7, 0, 0, 0]
        fp.post(epi, cur)  # nothing pending: a no-op
    torch.cuda.synchronize()
    timeout = trunc & ~term
    done = term | trunc
    with torch.no_grad():
        tv = pol.value(tobs)
    want = torch.where(timeout, rew + gamma * tv, rew)
    _close(buf_rew[2].cpu(), want.cpu())   # row (7 - 1) % 4
    assert torch.all(torch.cat([buf_rew[:2], buf_rew[3:]]) == -5.0)
    assert torch.equal(last_start, done.float())
    if fused:  # episode_starts of step 7 (row 3) is the epilogue's last_start
        assert torch.equal(starts[3], done.float())
    assert torch.equal(ep_ret, torch.where(done, 0.0, ret0 + rew))
    assert torch.equal(ep_len, torch.where(done, 0.0, len0 + 1))
    fr, fl = (ret0 + rew)[done].double(), (len0 + 1)[done].double()
    s = slots.sum(0).cpu().numpy()
    assert s[2] == done.sum().item() and s[1] == fl.sum().item()
    assert abs(s[0] - fr.sum().item()) <= 1e-4 * (1 + abs(fr.sum().item()))


def test_cursor_advances_over_many_launches():
    """The last-block cursor update is grid-wide: 50 launches at a size with several tiles per
    wave advance t by exactly 50 and keep the pending mark."""
    from uav_reinforcement_learning_control_amd import _native as N
    pol = _policy(6)
    fp = _fused(pol)
    n, T = 200_000, 3
    f = lambda *s: torch.zeros(*s, device="cuda")
    rew, buf_rew, ls, er, el = f(n), f(T, n), f(n), f(n), f(n)
    tb = torch.zeros(n, dtype=torch.bool, device="cuda")
    slots = torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device="cuda")
    epi = fp.make_epilogue(rew, tb, tb, f(n, 12), buf_rew, ls, er, el, slots, T, 0.9)
    cur = torch.zeros(4, dtype=torch.int32, device="cuda")
    obs, ae = f(n, 12), f(n, 4)
    for _ in range(50):
        fp.act(obs, ae, cursor=cur, rows=T, epilogue=epi)
    torch.cuda.synchronize()
    assert cur.tolist() == [50, 1, 0, 0]
    assert torch.all(el == 49.0)  # 49 epilogues ran (the first launch had nothing pending)


def test_policy_rejects_bad_arguments():
    from uav_reinforcement_learning_control_amd import _native as N
    pol = _policy(5)
    fp = _fused(pol)
    obs = torch.zeros(64, 12, device="cuda")
    with pytest.raises(ValueError):
        fp.act(obs, torch.zeros(64, 3, device="cuda"))
    with pytest.raises(ValueError):
        fp.act(obs, torch.zeros(64, 4, device="cuda"), value=torch.zeros(64, device="cuda"))
    a = N.QuadPolicyAct(obs=obs.data_ptr(), actions_env=None, rows=1)
    import ctypes as C
    assert N.lib().quad_policy_act(C.c_void_p(fp.packed.data_ptr()), C.byref(a), 64, None) == N.QUAD_EINVAL
