"""PPO with brax semantics ("Brax profile": train_brax_ppo.py:589-620) on the
GPU brax-compat env kinds.

train_brax_ppo.py drives brax's ``ppo.train`` (third-party, absent here; restated from its
published algorithm -- brax/training/agents/ppo/{train,losses,networks}.py,
brax/training/distribution.py, brax/training/acme/running_statistics.py -- so parity is unpinned):

  * networks: separate policy MLP obs -> hidden -> 2*act (loc, raw scale) and value MLP
    obs -> hidden -> 1, layers named ``hidden_i``, lecun-uniform kernels, zero biases, activation
    after every layer but the last; observations normalized inside the networks by the running
    statistics;
  * NormalTanhDistribution: scale = softplus(raw) + 0.001; raw action = loc + scale * eps; env
    action = tanh(raw); log_prob(raw) = sum(Normal.log_prob(raw) - 2 (log 2 - raw - softplus(-2 raw)));
    entropy = sum(Normal entropy + the same log-det at one sample); deterministic action = tanh(loc);
  * running statistics (acme): count += batch, mean += sum(x - mean) / count,
    summed_variance += sum((x - mean_old)(x - mean_new)), std = clip(sqrt(summed_variance / count),
    1e-6, 1e6), normalize = (x - mean) / std -- updated once per training step with all of its
    observations, AFTER the unrolls were generated with the previous statistics;
  * a training step: batch_size * num_minibatches // num_envs unrolls of unroll_length steps,
    reshaped to trajectories [M, L]; num_updates_per_batch passes, each over a fresh permutation of
    trajectories split into num_minibatches minibatches; per minibatch the loss recomputes GAE on the
    trajectories with brax's truncation masks and bootstrap V(next_obs[-1]), normalizes the
    advantages, clipped surrogate (epsilon 0.3), value loss 0.25 * mean((vs - v)^2), entropy bonus
    entropy_cost * entropy; Adam (optax defaults, eps 1e-8), no gradient clipping.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

LOG2 = math.log(2.0)
HALF_LOG_2PI = 0.5 * math.log(2.0 * math.pi)


@dataclass
class BraxPPOConfig:
    """train_brax_ppo.py argument defaults (:433-460)."""
    num_envs: int = 1024
    episode_length: int = 500
    learning_rate: float = 3e-4
    entropy_cost: float = 1e-3
    discounting: float = 0.99
    unroll_length: int = 10
    batch_size: int = 1024
    num_minibatches: int = 16
    num_updates_per_batch: int = 4
    gae_lambda: float = 0.95
    reward_scaling: float = 1.0
    clipping_epsilon: float = 0.3
    normalize_advantage: bool = True
    policy_hidden_sizes: tuple = (128, 128)
    value_hidden_sizes: tuple = (128, 128)
    activation: str = "relu"
    min_std: float = 0.001


_ACT = {"relu": F.relu, "tanh": torch.tanh, "silu": F.silu}


class BraxMLP(nn.Module):
    """brax.training.networks.MLP: Dense layers ``hidden_i`` (lecun-uniform kernel, zero bias),
    activation after all but the final layer. ``kernel`` is stored [in, out] like flax."""

    def __init__(self, sizes, activation: str = "relu"):
        super().__init__()
        self.kernels = nn.ParameterList()
        self.biases = nn.ParameterList()
        for fan_in, fan_out in zip(sizes[:-1], sizes[1:]):
            lim = math.sqrt(3.0 / fan_in)  # variance_scaling(1, fan_in, uniform)
            self.kernels.append(nn.Parameter(torch.empty(fan_in, fan_out).uniform_(-lim, lim)))
            self.biases.append(nn.Parameter(torch.zeros(fan_out)))
        self.act = _ACT[activation]

    def forward(self, x):
        n = len(self.kernels)
        for i, (k, b) in enumerate(zip(self.kernels, self.biases)):
            x = torch.addmm(b, x, k) if x.dim() == 2 else torch.matmul(x, k) + b
            if i < n - 1:
                x = self.act(x)
        return x

    def flax_params(self) -> dict:
        return {"params": {f"hidden_{i}": {"kernel": k.detach().cpu().numpy(), "bias": b.detach().cpu().numpy()}
                           for i, (k, b) in enumerate(zip(self.kernels, self.biases))}}

    @torch.no_grad()
    def load_flax_params(self, p: dict) -> None:
        p = p.get("params", p)
        for i, (k, b) in enumerate(zip(self.kernels, self.biases)):
            k.copy_(torch.as_tensor(p[f"hidden_{i}"]["kernel"]))
            b.copy_(torch.as_tensor(p[f"hidden_{i}"]["bias"]))


class RunningStats:
    """brax.training.acme.running_statistics (single-array observation)."""

    def __init__(self, dim: int, device, std_min: float = 1e-6, std_max: float = 1e6):
        f = dict(dtype=torch.float32, device=device)
        self.count = torch.zeros((), **f)
        self.mean = torch.zeros(dim, **f)
        self.summed_variance = torch.zeros(dim, **f)
        self.std = torch.ones(dim, **f)
        self.std_min, self.std_max = std_min, std_max

    @torch.no_grad()
    def update(self, x: torch.Tensor) -> None:
        x = x.reshape(-1, x.shape[-1]).float()
        self.count += x.shape[0]
        d_old = x - self.mean
        self.mean += d_old.sum(0) / self.count
        d_new = x - self.mean
        self.summed_variance += (d_old * d_new).sum(0)
        self.std = torch.clamp(torch.sqrt(self.summed_variance / self.count), self.std_min, self.std_max)

    def normalize(self, x: torch.Tensor, mean=None, std=None) -> torch.Tensor:
        return (x - (self.mean if mean is None else mean)) / (self.std if std is None else std)

    def snapshot(self):
        return self.mean.clone(), self.std.clone()


def tanh_log_det(x: torch.Tensor) -> torch.Tensor:
    """TanhBijector.forward_log_det_jacobian: 2 (log 2 - x - softplus(-2x))."""
    return 2.0 * (LOG2 - x - F.softplus(-2.0 * x))


class NormalTanh:
    """brax.training.distribution.NormalTanhDistribution."""

    def __init__(self, act_dim: int, min_std: float = 0.001):
        self.act_dim, self.min_std = act_dim, min_std

    def split(self, logits):
        loc, raw = logits[..., :self.act_dim], logits[..., self.act_dim:]
        return loc, F.softplus(raw) + self.min_std

    def sample_raw(self, logits, generator=None):
        loc, scale = self.split(logits)
        return loc + scale * torch.randn(loc.shape, dtype=loc.dtype, device=loc.device, generator=generator)

    def log_prob(self, logits, raw):
        loc, scale = self.split(logits)
        lp = -0.5 * ((raw - loc) / scale) ** 2 - HALF_LOG_2PI - torch.log(scale)
        return (lp - tanh_log_det(raw)).sum(-1)

    def entropy(self, logits, generator=None):
        loc, scale = self.split(logits)
        ent = 0.5 + HALF_LOG_2PI + torch.log(scale)
        x = loc + scale * torch.randn(loc.shape, dtype=loc.dtype, device=loc.device, generator=generator)
        return (ent + tanh_log_det(x)).sum(-1)

    def mode(self, logits):
        return torch.tanh(self.split(logits)[0])


def brax_gae(truncation, termination, rewards, values, bootstrap_value, lam, discount):
    """brax.training.agents.ppo.losses.compute_gae, time-major [T, B]; returns (vs, advantages),
    both outside the autograd graph (brax stop_gradients them)."""
    values, bootstrap_value = values.detach(), bootstrap_value.detach()
    trunc_mask = 1.0 - truncation
    v_tp1 = torch.cat([values[1:], bootstrap_value[None]], 0)
    deltas = (rewards + discount * (1.0 - termination) * v_tp1 - values) * trunc_mask
    acc = torch.zeros_like(bootstrap_value)
    out = torch.empty_like(values)
    for t in range(values.shape[0] - 1, -1, -1):
        acc = deltas[t] + discount * (1.0 - termination[t]) * trunc_mask[t] * lam * acc
        out[t] = acc
    vs = out + values
    vs_tp1 = torch.cat([vs[1:], bootstrap_value[None]], 0)
    adv = (rewards + discount * (1.0 - termination) * vs_tp1 - values) * trunc_mask
    return vs.detach(), adv.detach()


class BraxActorCritic(nn.Module):
    def __init__(self, obs_dim: int = 21, act_dim: int = 4, cfg: Optional[BraxPPOConfig] = None):
        super().__init__()
        cfg = cfg or BraxPPOConfig()
        self.policy = BraxMLP((obs_dim, *cfg.policy_hidden_sizes, 2 * act_dim), cfg.activation)
        self.value = BraxMLP((obs_dim, *cfg.value_hidden_sizes, 1), cfg.activation)
        self.dist = NormalTanh(act_dim, cfg.min_std)


def brax_ppo_loss(net: BraxActorCritic, norm_obs, norm_next_last, raw_action, behaviour_logp, reward,
                  discount, truncation, cfg: BraxPPOConfig, generator=None):
    """brax ppo ``compute_ppo_loss`` for a minibatch of trajectories, time-major [L, B, ...].
    Returns (total, policy_loss, v_loss, entropy_loss)."""
    logits = net.policy(norm_obs)
    baseline = net.value(norm_obs).squeeze(-1)
    bootstrap = net.value(norm_next_last).squeeze(-1)
    rewards = reward * cfg.reward_scaling
    termination = (1.0 - discount) * (1.0 - truncation)
    target_logp = net.dist.log_prob(logits, raw_action)
    vs, adv = brax_gae(truncation, termination, rewards, baseline, bootstrap, cfg.gae_lambda, cfg.discounting)
    if cfg.normalize_advantage:
        adv = (adv - adv.mean()) / (adv.std(unbiased=False) + 1e-8)
    rho = torch.exp(target_logp - behaviour_logp)
    s1 = rho * adv
    s2 = torch.clamp(rho, 1.0 - cfg.clipping_epsilon, 1.0 + cfg.clipping_epsilon) * adv
    policy_loss = -torch.mean(torch.minimum(s1, s2))
    v_err = vs - baseline
    v_loss = torch.mean(v_err * v_err) * 0.5 * 0.5
    entropy = torch.mean(net.dist.entropy(logits, generator))
    entropy_loss = cfg.entropy_cost * -entropy
    return policy_loss + v_loss + entropy_loss, policy_loss, v_loss, entropy_loss


@dataclass
class BraxStepStats:
    env_steps: int = 0
    seconds: float = 0.0
    episodes: int = 0
    mean_episode_reward: float = float("nan")
    losses: dict = field(default_factory=dict)


class BraxPPO:
    """brax ``ppo.train``'s training step on a ``QuadVecEnv`` brax kind (env="brax_hover" or
    "brax_jax_mjx"), one process per GPU (gradients averaged with one flat all_reduce)."""

    def __init__(self, env, cfg: Optional[BraxPPOConfig] = None, seed: int = 0):
        self.env, self.cfg = env, cfg or BraxPPOConfig()
        c = self.cfg
        if env.num_envs != c.num_envs:
            raise ValueError("env.num_envs must equal cfg.num_envs")
        if (c.batch_size * c.num_minibatches) % c.num_envs:
            raise ValueError("batch_size * num_minibatches must be a multiple of num_envs (brax)")
        self.device = env.device
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        torch.manual_seed(seed)
        self.net = BraxActorCritic(env.obs_dim, 4, c).to(self.device)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=c.learning_rate, eps=1e-8)
        self.norm = RunningStats(env.obs_dim, self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + 7919 * (dist.get_rank() if self.world > 1 else 0))
        self.num_unrolls = c.batch_size * c.num_minibatches // c.num_envs
        self.num_timesteps = 0
        self._obs = None
        self._ep_ret = torch.zeros(c.num_envs, device=self.device)
        self._flat = torch.zeros(sum(p.numel() for p in self.net.parameters()), device=self.device)
        from .ppo import bind_grad_bucket
        bind_grad_bucket(list(self.net.parameters()), self._flat)  # in-place all-reduce

    @torch.no_grad()
    def _unrolls(self):
        c, env = self.cfg, self.env
        if self._obs is None:
            self._obs = env.reset().clone()
        U, L, N = self.num_unrolls, c.unroll_length, c.num_envs
        f = dict(device=self.device)
        obs = torch.empty(U, L, N, env.obs_dim, **f)
        nxt = torch.empty(U, N, env.obs_dim, **f)  # next_observation of each unroll's last step
        raw = torch.empty(U, L, N, 4, **f)
        logp = torch.empty(U, L, N, **f)
        rew = torch.empty(U, L, N, **f)
        disc = torch.empty(U, L, N, **f)
        trunc = torch.empty(U, L, N, **f)
        mean, std = self.norm.snapshot()  # the policy of this training step: previous statistics
        finished = torch.zeros((), device=self.device)
        ret_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        for u in range(U):
            for t in range(L):
                o = self._obs
                obs[u, t] = o
                logits = self.net.policy((o - mean) / std)
                r = self.net.dist.sample_raw(logits, self.gen)
                raw[u, t] = r
                logp[u, t] = self.net.dist.log_prob(logits, r)
                no, rw, te, tr, _ = env.step(torch.tanh(r), info="raw")
                done = te | tr
                rew[u, t] = rw
                disc[u, t] = 1.0 - done.float()
                trunc[u, t] = (tr & ~te).float()   # EpisodeWrapper info['truncation']
                self._ep_ret += rw
                finished += done.sum()
                ret_sum += (self._ep_ret * done).sum().double()
                self._ep_ret *= ~done
                self._obs = no.clone()
            nxt[u] = self._obs
        return obs, nxt, raw, logp, rew, disc, trunc, finished, ret_sum

    def training_step(self) -> BraxStepStats:
        c = self.cfg
        t0 = time.perf_counter()
        obs, nxt, raw, logp, rew, disc, trunc, finished, ret_sum = self._unrolls()
        U, L, N = obs.shape[:3]
        self.norm.update(obs)  # acme running statistics, after the unrolls
        # trajectories [M = U * N, L, ...] -> time-major per minibatch
        tr = lambda x: x.transpose(1, 2).reshape(U * N, L, *x.shape[3:])
        obs_m, raw_m, logp_m, rew_m, disc_m, trunc_m = map(tr, (obs, raw, logp, rew, disc, trunc))
        nxt_m = nxt.reshape(U * N, -1)
        M = U * N
        mb = M // c.num_minibatches
        acc = torch.zeros(3, dtype=torch.float64, device=self.device)
        nsteps = 0
        for _ in range(c.num_updates_per_batch):
            perm = torch.randperm(M, device=self.device, generator=self.gen)
            for k in range(c.num_minibatches):
                idx = perm[k * mb:(k + 1) * mb]
                T = lambda x: x[idx].transpose(0, 1)
                loss, pl, vl, el = brax_ppo_loss(
                    self.net, self.norm.normalize(T(obs_m)), self.norm.normalize(nxt_m[idx]), T(raw_m),
                    T(logp_m), T(rew_m), T(disc_m), T(trunc_m), c, self.gen)
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.world > 1:
                    from .ppo import allreduce_mean_
                    allreduce_mean_(list(self.net.parameters()), self._flat, self.world)
                self.opt.step()
                acc += torch.stack([pl.detach(), vl.detach(), el.detach()]).double()
                nsteps += 1
        torch.cuda.synchronize(self.device)
        steps = U * L * N
        self.num_timesteps += steps * self.world
        a = (acc / max(nsteps, 1)).tolist()
        n_fin, r_sum = int(finished.item()), float(ret_sum.item())
        return BraxStepStats(env_steps=steps, seconds=time.perf_counter() - t0, episodes=n_fin,
                             mean_episode_reward=r_sum / n_fin if n_fin else float("nan"),
                             losses=dict(policy_loss=a[0], v_loss=a[1], entropy_loss=a[2]))

    @torch.no_grad()
    def act(self, obs: torch.Tensor, deterministic: bool = True) -> torch.Tensor:
        logits = self.net.policy(self.norm.normalize(obs))
        return self.net.dist.mode(logits) if deterministic else torch.tanh(self.net.dist.sample_raw(logits, self.gen))

    def params(self):
        """(normalizer, policy, value) as brax ppo.train returns them (numpy leaves)."""
        return (dict(count=self.norm.count.cpu().numpy(), mean=self.norm.mean.cpu().numpy(),
                     summed_variance=self.norm.summed_variance.cpu().numpy(), std=self.norm.std.cpu().numpy()),
                self.net.policy.flax_params(), self.net.value.flax_params())
