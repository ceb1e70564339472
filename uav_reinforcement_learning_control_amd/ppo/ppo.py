"""PPO with SB3 semantics on the GPU-resident env (row P of SURVEY.md section 8).

Defaults are the reference's train.py:50-68 hyperparameters. What is reproduced from SB3 PPO
(stable_baselines3, third-party, absent here, parity unpinned -- see DESIGN.md):
  * rollout: Gaussian actions from the policy, clipped to [-1, 1] only when sent to the env;
    buffers keep the unclipped action; episode_starts; TimeLimit bootstrap
    r += gamma * V(terminal_obs) when truncated and not terminated (OnPolicyAlgorithm
    .collect_rollouts);
  * GAE(lambda) reverse scan (k_gae kernel; RolloutBuffer.compute_returns_and_advantage);
  * n_epochs passes over shuffled minibatches; per-minibatch advantage normalization
    (adv - mean) / (std + 1e-8); clipped surrogate; value MSE (no value clipping); entropy
    bonus; loss = pg + ent_coef * (-entropy) + vf_coef * vf; grad-norm clip 0.5; Adam eps 1e-5.

Scale: SB3's batch_size 128 over a 65,536 x 1,024 buffer would be 524,288 optimizer steps per
update, so by default the number of minibatches per epoch (SB3: 16 x 1024 / 128 = 128) is kept
and the minibatch grows with the env count (`n_minibatches`, SURVEY.md section 7 hard part 4).

Multi-GPU: one process per GPU, each with its own env shard; after every minibatch backward the
gradients are averaged with ONE all_reduce over a single flat fp32 bucket (RCCL over xGMI).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .gae import gae
from .policy import ActorCritic


@dataclass
class PPOConfig:
    learning_rate: float = 0.0001547818138087132
    n_steps: int = 1024
    batch_size: Optional[int] = None      # SB3 batch_size; None -> derived from n_minibatches
    n_minibatches: int = 128              # 16 envs x 1024 steps / batch_size 128 (train.py)
    n_epochs: int = 20
    gamma: float = 0.9906345854291289
    gae_lambda: float = 0.9079441765099094
    clip_range: float = 0.19153175856282983
    ent_coef: float = 9.106557393423481e-05
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True
    net_arch: tuple = (128, 128)
    adam_eps: float = 1e-5


@dataclass
class RolloutStats:
    episodes: int = 0
    mean_return: float = float("nan")
    mean_length: float = float("nan")
    env_steps: int = 0
    seconds: float = 0.0
    extra: dict = field(default_factory=dict)


class PPO:
    def __init__(self, env, config: Optional[PPOConfig] = None, seed: int = 0,
                 policy: Optional[ActorCritic] = None):
        self.env = env
        self.cfg = config or PPOConfig()
        self.device = env.device
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        torch.manual_seed(seed)  # identical policy init on every rank
        self.policy = (policy or ActorCritic(12, 4, self.cfg.net_arch)).to(self.device)
        self.params = [p for p in self.policy.parameters()]
        self.opt = torch.optim.Adam(self.params, lr=self.cfg.learning_rate, eps=self.cfg.adam_eps)
        torch.manual_seed(seed + 1000 * (dist.get_rank() if self.world > 1 else 0))
        T, n = self.cfg.n_steps, env.num_envs
        f32 = dict(dtype=torch.float32, device=self.device)
        self.buf_obs = torch.zeros(T, n, 12, **f32)
        self.buf_act = torch.zeros(T, n, 4, **f32)
        self.buf_logp = torch.zeros(T, n, **f32)
        self.buf_val = torch.zeros(T, n, **f32)
        self.buf_rew = torch.zeros(T, n, **f32)
        self.buf_start = torch.zeros(T, n, **f32)
        self.buf_adv = torch.zeros(T, n, **f32)
        self.buf_ret = torch.zeros(T, n, **f32)
        self.last_obs = torch.zeros(n, 12, **f32)
        self.last_start = torch.ones(n, **f32)
        self.ep_ret = torch.zeros(n, **f32)
        self.ep_len = torch.zeros(n, **f32)
        self.num_timesteps = 0
        self._started = False
        total = T * n
        if self.cfg.batch_size is not None:
            self.batch = int(self.cfg.batch_size)
        else:
            self.batch = max(1, total // self.cfg.n_minibatches)
        self._flat = torch.zeros(sum(p.numel() for p in self.params), **f32)

    # ------------------------------------------------------------------------------------
    @torch.no_grad()
    def collect_rollouts(self) -> RolloutStats:
        env, cfg, pol = self.env, self.cfg, self.policy
        if not self._started:
            self.last_obs.copy_(env.reset())
            self.last_start.fill_(1.0)
            self._started = True
        t0 = time.perf_counter()
        done_ret = torch.zeros((), dtype=torch.float64, device=self.device)
        done_len = torch.zeros((), dtype=torch.float64, device=self.device)
        done_cnt = torch.zeros((), dtype=torch.float64, device=self.device)
        for t in range(cfg.n_steps):
            self.buf_obs[t].copy_(self.last_obs)
            self.buf_start[t].copy_(self.last_start)
            a, logp, v = pol.act(self.last_obs)
            self.buf_act[t].copy_(a)
            self.buf_logp[t].copy_(logp)
            self.buf_val[t].copy_(v)
            obs, rew, term, trunc, info = env.step(a.clamp(-1.0, 1.0).contiguous())
            done = term | trunc
            timeout = (trunc & ~term).float()
            # TimeLimit bootstrap (SB3 collect_rollouts): r += gamma * V(terminal_obs)
            tv = pol.value(info["terminal_observation"])
            r = rew + cfg.gamma * torch.where(timeout > 0, tv, torch.zeros_like(tv))
            self.buf_rew[t].copy_(r)
            # Monitor-style episode statistics (raw env reward)
            self.ep_ret += rew
            self.ep_len += 1
            df = done.float()
            done_ret += (self.ep_ret * df).sum()
            done_len += (self.ep_len * df).sum()
            done_cnt += df.sum()
            self.ep_ret *= 1 - df
            self.ep_len *= 1 - df
            self.last_obs.copy_(obs)
            self.last_start.copy_(df)
        last_v = pol.value(self.last_obs)
        gae(self.buf_rew, self.buf_val, self.buf_start, last_v, self.last_start,
            cfg.gamma, cfg.gae_lambda, self.buf_adv, self.buf_ret)
        torch.cuda.synchronize(self.device)
        steps = cfg.n_steps * env.num_envs
        self.num_timesteps += steps * self.world
        c = float(done_cnt.item())
        return RolloutStats(episodes=int(c),
                            mean_return=float(done_ret.item() / c) if c else float("nan"),
                            mean_length=float(done_len.item() / c) if c else float("nan"),
                            env_steps=steps, seconds=time.perf_counter() - t0)

    # ------------------------------------------------------------------------------------
    def _allreduce_grads(self):
        grads = [p.grad for p in self.params]
        off = 0
        for g in grads:
            k = g.numel()
            self._flat[off:off + k].copy_(g.view(-1))
            off += k
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM)
        self._flat.div_(self.world)
        off = 0
        for g in grads:
            k = g.numel()
            g.view(-1).copy_(self._flat[off:off + k])
            off += k

    def train(self, n_epochs: Optional[int] = None, max_minibatches: Optional[int] = None) -> dict:
        cfg, pol = self.cfg, self.policy
        total = cfg.n_steps * self.env.num_envs
        obs = self.buf_obs.view(total, 12)
        act = self.buf_act.view(total, 4)
        logp_old = self.buf_logp.view(total)
        adv_all = self.buf_adv.view(total)
        ret = self.buf_ret.view(total)
        B = self.batch
        nmb = max(1, total // B)
        stats = dict(pg_loss=0.0, vf_loss=0.0, entropy=0.0, clip_fraction=0.0, n=0)
        acc = torch.zeros(4, dtype=torch.float64, device=self.device)
        done = 0
        for _ in range(n_epochs if n_epochs is not None else cfg.n_epochs):
            perm = torch.randperm(total, device=self.device)
            for m in range(nmb):
                if max_minibatches is not None and done >= max_minibatches:
                    break
                idx = perm[m * B:(m + 1) * B]
                mean, v = pol.forward_heads(obs[idx])
                logp = pol.log_prob(mean, act[idx])
                adv = adv_all[idx]
                if cfg.normalize_advantage and B > 1:
                    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
                ratio = torch.exp(logp - logp_old[idx])
                pg = -torch.min(adv * ratio,
                                adv * torch.clamp(ratio, 1 - cfg.clip_range, 1 + cfg.clip_range)).mean()
                vf = nn.functional.mse_loss(ret[idx], v)
                ent = pol.entropy()
                loss = pg + cfg.ent_coef * (-ent) + cfg.vf_coef * vf
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.world > 1:
                    self._allreduce_grads()
                nn.utils.clip_grad_norm_(self.params, cfg.max_grad_norm)
                self.opt.step()
                with torch.no_grad():
                    acc += torch.stack([pg.detach().double(), vf.detach().double(), ent.detach().double(),
                                        ((ratio - 1).abs() > cfg.clip_range).float().mean().double()])
                done += 1
        a = (acc / max(done, 1)).tolist()
        stats.update(pg_loss=a[0], vf_loss=a[1], entropy=a[2], clip_fraction=a[3], n=done)
        return stats

    def learn(self, total_timesteps: int, callback: Optional[Callable] = None) -> "PPO":
        it = 0
        while self.num_timesteps < total_timesteps:
            rs = self.collect_rollouts()
            ts = self.train()
            it += 1
            if callback is not None and callback(self, it, rs, ts) is False:
                break
        return self

    def state_dict(self) -> dict:
        return {"policy": self.policy.state_dict(), "optimizer": self.opt.state_dict(),
                "num_timesteps": self.num_timesteps}
