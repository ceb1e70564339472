"""quad_permutation (the epoch permutation of PPO.train, csrc/learner.hip k_permutation) on the GPU:
a bijection of [0, n) for every n (cycle walking over a 4-round Feistel on 4^k codes), equal to
the NumPy restatement below bit for bit, keyed by the seed, and close to uniform over positions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

M32 = 0xFFFFFFFF


def _hash(x, k):
    x = (x ^ k) & M32
    x = (x * 0x7FEB352D) & M32; x ^= x >> 15
    x = (x * 0x846CA68B) & M32; x ^= x >> 16
    x = (x * 0x7FEB352D) & M32; x ^= x >> 15
    return x


def _ref_permutation(n, seed):
    bits = 2
    while (1 << bits) < n:
        bits += 2
    hb = bits // 2
    mask = (1 << hb) - 1

    def feistel(x):
        L, R = (x >> hb) & mask, x & mask
        for r in range(4):
            k = (((seed >> (32 if r & 1 else 0)) & M32) + 0x9E3779B9 * (r + 1)) & M32
            L, R = R, (L ^ _hash(R, k)) & mask
        return (L << hb) | R

    out = []
    for i in range(n):
        x = i
        while True:
            x = feistel(x)
            if x < n:
                break
        out.append(x)
    return np.array(out, dtype=np.int64)


def _perm(n, seed):
    from uav_reinforcement_learning_control_amd import _native as N
    out = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    N.check(N.lib().quad_permutation(n, seed, out.data_ptr(), torch.cuda.current_stream().cuda_stream),
            "quad_permutation")
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("n", [1, 2, 3, 5, 1000, 4096, 65539, (1 << 22) + 17, 1 << 26])
def test_is_a_permutation(n):
    p = _perm(n, 12345)
    assert torch.equal(torch.sort(p).values, torch.arange(n, device="cuda"))


@pytest.mark.parametrize("n,seed", [(1, 0), (7, 3), (1000, 2**61 + 5), (4097, 99)])
def test_matches_restatement(n, seed):
    np.testing.assert_array_equal(_perm(n, seed).cpu().numpy(), _ref_permutation(n, seed))


def test_seeded_and_near_uniform():
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.ppo.ppo import epoch_permutation
    assert torch.equal(_perm(5000, 1), _perm(5000, 1))
    assert not torch.equal(_perm(5000, 1), _perm(5000, 2))
    torch.manual_seed(3)
    a = epoch_permutation(5000, torch.device("cuda"))
    torch.manual_seed(3)
    assert torch.equal(a, epoch_permutation(5000, torch.device("cuda")))
    # position -> value counts over many keys: chi-square of a uniform 16 x 16 table
    n, keys = 16, 4000
    counts = np.zeros((n, n))
    for s in range(keys):
        p = _perm(n, s * 0x9E3779B97F4A7C15 % (1 << 63)).cpu().numpy()
        counts[np.arange(n), p] += 1
    exp = keys / n
    chi2 = ((counts - exp) ** 2 / exp).sum()
    dof = (n - 1) ** 2
    assert abs(chi2 - dof) < 6 * np.sqrt(2 * dof), (chi2, dof)
    assert N.lib().quad_permutation(0, 1, None, None) == N.QUAD_EINVAL


@pytest.mark.parametrize("seed", [0, 7, 2**61 + 5])
def test_config3_domain_statistics(seed):
    """At config 3's own domain -- a 65,536 x 1,024 rollout buffer, n = 2^26 rows, 128 minibatches of
    524,288 -- where the Feistel halves are 13 bits wide:
      * the first minibatch's values are uniform over 1,024 equal value buckets (chi-square; the
        sample is drawn without replacement, which only narrows the spread);
      * consecutive outputs are uncorrelated (lag-1 serial correlation, |r| < 6 / sqrt(m));
      * the minibatch touches as many distinct 4-KB pages of the [n, 12] float32 observation buffer
        as uniform samples of the same size (torch.randperm) do: no gather locality bias."""
    n, m = 1 << 26, 524288
    p = _perm(n, seed)
    first = p[:m]
    # value buckets
    counts = torch.bincount(first // (n // 1024), minlength=1024).double().cpu().numpy()
    exp = m / 1024
    chi2 = ((counts - exp) ** 2 / exp).sum()
    dof = 1023
    assert abs(chi2 - dof) < 6 * np.sqrt(2 * dof), (chi2, dof)
    # lag-1 serial correlation over the whole epoch and over the first minibatch
    for seq in (p, first):
        x = seq.double()
        x = (x - x.mean()) / x.std()
        r = (x[:-1] * x[1:]).mean().item()
        assert abs(r) < 6 / np.sqrt(x.numel()), r
    # distinct 4-KB pages of the observation rows (48 B each) a minibatch gathers from
    def pages(idx):
        lo, hi = (idx * 48) // 4096, (idx * 48 + 47) // 4096
        return int(torch.unique(torch.cat([lo, hi])).numel())
    got = pages(first)
    g = torch.Generator(device="cuda").manual_seed(seed & 0xFFFF)
    uni = np.array([pages(torch.randperm(n, device="cuda", generator=g)[:m]) for _ in range(4)], dtype=np.float64)
    print(f"\nseed {seed}: chi2 {chi2:.1f} (dof {dof}); distinct obs pages {got} vs uniform {uni.mean():.0f} "
          f"+- {uni.std():.0f} of {n * 48 // 4096}")
    assert abs(got - uni.mean()) <= max(6 * uni.std(), 1e-3 * uni.mean()), (got, uni)
