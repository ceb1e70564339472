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

from .. import _native as N
from .fused import FusedPolicy, rollout_supported
from .gae import gae
from .learner import FusedAdam, FusedLearner
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
    fused_policy: bool = True             # rollout policy on the MFMA kernels (ppo/fused.py)
    fused_rollout: bool = True            # whole rollout as quad_rollout launches (needs fused_policy)
    rollout_chunk: int = 1024             # steps per quad_rollout launch
    fused_update: bool = True             # minibatch gradient on MFMA (ppo/learner.py, quad_ppo_grad)
    graph_update: bool = True             # single GPU: replay each epoch's optimizer steps as one hipGraph


# quad_ppo_adv_stats_epoch's grid y limit is 65,535; its [n, 512] float64 output is 4 KB per
# minibatch, so the one-launch statistics are used up to 4,096 minibatches per epoch (16 MB)
EPOCH_STATS_MAX_MINIBATCHES = 4096


def n_minibatches(total: int, batch: int) -> int:
    """SB3 RolloutBuffer.get(batch_size): slices indices[start:start + batch_size] for start = 0,
    batch_size, ... < total -- ceil(total / batch) minibatches, the last one short when batch_size
    does not divide the buffer, one minibatch of every row when batch_size >= total."""
    return max(1, -(-int(total) // int(batch)))


def epoch_permutation(total: int, device: torch.device, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The epoch's minibatch order (SB3 PPO.train: np.random.permutation(buffer_size)). On a ROCm
    GPU it is quad_permutation -- a keyed Feistel bijection of [0, total) computed one index per
    thread (torch.randperm sorts `total` random keys: 5.3 ms per epoch at config 3). The key is drawn
    from torch's default CPU generator, so torch.manual_seed fixes it and no device sync happens."""
    if device.type != "cuda":
        return torch.randperm(total, device=device)
    if out is None:
        out = torch.empty(total, dtype=torch.int64, device=device)
    seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64))
    N.check(N.lib().quad_permutation(total, seed, out.data_ptr(), torch.cuda.current_stream(device).cuda_stream),
            "quad_permutation")
    return out


def ppo_loss(policy: ActorCritic, obs, act, logp_old, adv, ret, cfg: PPOConfig):
    """SB3 PPO.train minibatch loss: returns (loss, pg_loss, vf_loss, entropy, clip_fraction)."""
    mean, v = policy.forward_heads(obs)
    logp = policy.log_prob(mean, act)
    if cfg.normalize_advantage and adv.numel() > 1:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(logp - logp_old)
    pg = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - cfg.clip_range, 1 + cfg.clip_range)).mean()
    vf = nn.functional.mse_loss(ret, v)
    ent = policy.entropy()
    loss = pg + cfg.ent_coef * (-ent) + cfg.vf_coef * vf
    clip_frac = ((ratio - 1).abs() > cfg.clip_range).float().mean()
    return loss, pg, vf, ent, clip_frac


def bind_grad_bucket(params, flat: torch.Tensor) -> None:
    """Make every parameter's .grad a view of one flat fp32 bucket (parameter order), so the
    gradient kernels (quad_ppo_grad's reduction, autograd's in-place accumulation) write straight
    into the buffer the all-reduce sends: no copies around the collective."""
    off = 0
    for p in params:
        k = p.numel()
        p.grad = flat[off:off + k].view_as(p)
        off += k
    if off != flat.numel():
        raise ValueError("bucket size does not match the parameters")


def _bucket_bound(params, flat: torch.Tensor) -> bool:
    base, off = flat.data_ptr(), 0
    for p in params:
        g = p.grad
        if g is None or g.data_ptr() != base + 4 * off or not g.is_contiguous():
            return False
        off += p.numel()
    return True


def allreduce_mean_(params, flat: torch.Tensor, world: int, between: Optional[Callable[[], None]] = None,
                    timing: Optional[list] = None) -> None:
    """Average the gradients of `params` over ranks with ONE all_reduce of a flat fp32 bucket:
    SUM, then a division by the world size -- the same two ops on RCCL and on gloo, so the gloo
    tests exercise exactly what the GPU job runs. With the .grad tensors bound to the bucket
    (bind_grad_bucket) the collective runs in place; otherwise (a caller replaced a .grad) they are
    copied in and out. `between`, if given, is called while the collective is in flight (it must
    not touch the bucket): on RCCL its launches overlap the all-reduce (work.wait() only makes the
    current stream wait on the communication stream). `timing`, if given (a list, CUDA tensors),
    receives a pair of HIP events recorded on the current stream before the collective is issued
    and after work.wait(): their interval is the time the step's own stream is held by the
    all-reduce (the exposed communication of this optimizer step; PPO.comm_stats)."""
    bound = _bucket_bound(params, flat)
    if not bound:
        off = 0
        for p in params:
            k = p.numel()
            flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
    ev = None
    if timing is not None and flat.is_cuda:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)
    if between is not None:
        between()
    work.wait()
    if ev is not None:
        ev[1].record()
        timing.append(ev)
    flat.div_(world)
    if not bound:
        off = 0
        for p in params:
            k = p.numel()
            p.grad.copy_(flat[off:off + k].view_as(p))
            off += k


def broadcast_parameters_(params, src: int = 0) -> None:
    """Every rank starts from rank `src`'s parameters (one broadcast of a flat copy): the ranks'
    identical initialization does not rest on each rank seeding torch the same way before the
    policy is built."""
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    dist.broadcast(flat, src)
    off = 0
    with torch.no_grad():
        for p in params:
            k = p.numel()
            p.copy_(flat[off:off + k].view_as(p))
            off += k


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
        self.obs_dim = int(getattr(env, "obs_dim", 12))
        self.policy = (policy or ActorCritic(self.obs_dim, 4, self.cfg.net_arch)).to(self.device)
        self.params = [p for p in self.policy.parameters()]
        if self.world > 1:
            broadcast_parameters_(self.params, 0)
        self.opt = torch.optim.Adam(self.params, lr=self.cfg.learning_rate, eps=self.cfg.adam_eps,
                                    fused=self.device.type == "cuda")  # one kernel per step
        torch.manual_seed(seed + 1000 * (dist.get_rank() if self.world > 1 else 0))
        T, n = self.cfg.n_steps, env.num_envs
        f32 = dict(dtype=torch.float32, device=self.device)
        self.buf_obs = torch.zeros(T, n, self.obs_dim, **f32)
        self.buf_act = torch.zeros(T, n, 4, **f32)
        self.buf_logp = torch.zeros(T, n, **f32)
        self.buf_val = torch.zeros(T, n, **f32)
        self.buf_rew = torch.zeros(T, n, **f32)
        self.buf_start = torch.zeros(T, n, **f32)
        self.buf_adv = torch.zeros(T, n, **f32)
        self.buf_ret = torch.zeros(T, n, **f32)
        self.last_obs = torch.zeros(n, self.obs_dim, **f32)
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
        bind_grad_bucket(self.params, self._flat)  # .grad tensors are views of the all-reduce bucket
        self._t = torch.zeros(1, dtype=torch.long, device=self.device)
        self._act_env = torch.zeros(n, 4, **f32)
        self._last_v = torch.zeros(1, n, **f32)
        self._done_stats = torch.zeros(3, dtype=torch.float64, device=self.device)
        self._graph = None
        # fused path: cursor {t, pending} (buffer row = t % n_steps; t keys the action noise),
        # per-block episode-statistic slots, the epilogue descriptor
        # (the MFMA kernels are built for the 12-D HoverEnv obs and 128-128 nets)
        fusable = self.obs_dim == 12 and tuple(self.cfg.net_arch) == (128, 128)
        self._fp = FusedPolicy(self.policy) if self.cfg.fused_policy and fusable else None
        self._cursor = torch.zeros(4, dtype=torch.int32, device=self.device)
        self._slots = torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device=self.device)
        if self._fp is not None:
            self._epi = self._fp.make_epilogue(env.reward, env.terminated, env.truncated,
                                               env.terminal_obs, self.buf_rew, self.last_start,
                                               self.ep_ret, self.ep_len, self._slots, T, self.cfg.gamma)
        # one launch per chunk of steps: policy + env + bootstrap + statistics (csrc/rollout.hip)
        self._one_launch = (self._fp is not None and self.cfg.fused_rollout and rollout_supported(env))
        # the update's minibatch gradient as quad_ppo_grad launches (same fusability as the rollout)
        self._learner = (FusedLearner(self.policy, self.cfg.clip_range, self.cfg.ent_coef, self.cfg.vf_coef,
                                      self.cfg.normalize_advantage)
                         if self.cfg.fused_update and fusable and self.device.type == "cuda" else None)
        self._adam = FusedAdam(self.opt, self.cfg.max_grad_norm) if self._learner is not None else None
        self._epoch_graph = None  # (key, graph, perm, sums, mstats) of _train_fused's captured epoch
        self._t_host = 0  # running step counter of the one-launch path (keys the action noise)
        self._cursor_resume = None  # the two-launch path's noise counter after load_state_dict
        self._noise_seed = (int(seed) * 0x9E3779B97F4A7C15 + 0x5851F42D4C957F2D) & (2**64 - 1)
        self.comm_events: Optional[list] = None  # a list: time each gradient all-reduce (comm_stats)

    # ------------------------------------------------------------------------------------
    @torch.no_grad()
    def _rollout_step(self):
        """One rollout step on static tensors; capturable into a hipGraph (no host sync).
        Writes row t = self._t of the time-major buffers and advances self._t on the device."""
        env, cfg, pol = self.env, self.cfg, self.policy
        t = self._t
        self.buf_obs.index_copy_(0, t, self.last_obs.unsqueeze(0))
        self.buf_start.index_copy_(0, t, self.last_start.unsqueeze(0))
        mean, v = pol.forward_heads(self.last_obs)
        a = mean + pol.log_std.exp() * torch.randn_like(mean)
        self.buf_act.index_copy_(0, t, a.unsqueeze(0))
        self.buf_logp.index_copy_(0, t, pol.log_prob(mean, a).unsqueeze(0))
        self.buf_val.index_copy_(0, t, v.unsqueeze(0))
        torch.clamp(a, -1.0, 1.0, out=self._act_env)   # clipped only when sent to the env
        obs, rew, term, trunc, info = env.step(self._act_env)
        done = (term | trunc).float()
        timeout = (trunc & ~term).float()
        # TimeLimit bootstrap (SB3 collect_rollouts): r += gamma * V(terminal_obs)
        tv = pol.value(info["terminal_observation"])
        r = rew + cfg.gamma * timeout * torch.nan_to_num(tv)
        self.buf_rew.index_copy_(0, t, r.unsqueeze(0))
        # Monitor-style episode statistics (raw env reward)
        self.ep_ret += rew
        self.ep_len += 1
        self._done_stats += torch.stack([(self.ep_ret * done).sum(), (self.ep_len * done).sum(),
                                         done.sum()]).double()
        self.ep_ret *= 1 - done
        self.ep_len *= 1 - done
        self.last_obs.copy_(obs)
        self.last_start.copy_(done)
        self._t += 1

    def _rollout_step_fused(self):
        """The same step as two launches (graph-capturable): the MFMA policy kernel, which also
        finishes the previous step (bootstrap, reward row, statistics), and the env step."""
        env = self.env
        self._fp.act(self.last_obs, self._act_env, actions=self.buf_act, log_prob=self.buf_logp,
                     value=self.buf_val, obs_copy=self.buf_obs, last_start=self.last_start,
                     episode_starts=self.buf_start, cursor=self._cursor, rows=self.cfg.n_steps,
                     seed=self._noise_seed, env_id_base=env.env_id_base, epilogue=self._epi)
        env.step(self._act_env, obs=self.last_obs, info="raw")

    def _step_fn(self):
        return self._rollout_step_fused if self._fp is not None else self._rollout_step

    def _capture(self):
        # warm the kernels (rocBLAS handles, allocator) on a side stream, then capture one step
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        step = self._step_fn()
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._t.zero_()
        self._cursor.zero_()
        # several steps per graph (the step index lives on the device), fewer replay gaps
        self._graph_steps = next(k for k in (16, 8, 4, 2, 1) if self.cfg.n_steps % k == 0)
        self._graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._graph):
            for _ in range(self._graph_steps):
                step()
        torch.cuda.synchronize(self.device)

    @torch.no_grad()
    def collect_rollouts(self, use_graph: bool = True) -> RolloutStats:
        env, cfg, pol = self.env, self.cfg, self.policy
        if self._fp is not None:
            self._fp.pack()  # the kernels' copy of the weights the last update produced
        if not self._started:
            self.last_obs.copy_(env.reset())
            self.last_start.fill_(1.0)
            self._started = True
            if use_graph and not self._one_launch:
                self._capture()
            if self._cursor_resume is not None:  # (after _capture's zeroing) resume the noise counter
                self._cursor[0] = self._cursor_resume
                self._cursor_resume = None
        if self._one_launch:
            return self._collect_one_launch()
        t0 = time.perf_counter()
        self._t.zero_()
        self._done_stats.zero_()
        step = self._step_fn()
        self._slots.zero_()
        if use_graph and self._graph is not None:
            for _ in range(cfg.n_steps // self._graph_steps):
                self._graph.replay()
        else:
            for _ in range(cfg.n_steps):
                step()
        if self._fp is not None:
            self._fp.post(self._epi, self._cursor)   # finish the last step
            self._done_stats.copy_(self._slots.sum(0))
        last_v = self._bootstrap_value()
        gae(self.buf_rew, self.buf_val, self.buf_start, last_v, self.last_start,
            cfg.gamma, cfg.gae_lambda, self.buf_adv, self.buf_ret)
        return self._rollout_stats(t0)

    @torch.no_grad()
    def _collect_one_launch(self) -> RolloutStats:
        """collect_rollouts as quad_rollout launches (rollout_chunk steps each): same buffers, same
        semantics as the two-launch path, no per-step launches or HBM round trips of env state."""
        env, cfg, pol = self.env, self.cfg, self.policy
        t0 = time.perf_counter()
        self._slots.zero_()
        chunk = max(1, min(int(cfg.rollout_chunk), cfg.n_steps))
        s = 0
        while s < cfg.n_steps:
            k = min(chunk, cfg.n_steps - s)
            self._fp.rollout(env, obs_copy=self.buf_obs, actions=self.buf_act, log_prob=self.buf_logp,
                             value=self.buf_val, episode_starts=self.buf_start, rewards=self.buf_rew,
                             last_obs=self.last_obs, last_start=self.last_start, ep_ret=self.ep_ret,
                             ep_len=self.ep_len, stats=self._slots, t0=self._t_host + s, steps=k,
                             seed=self._noise_seed, gamma=cfg.gamma)
            s += k
        self._t_host += cfg.n_steps
        self._done_stats.copy_(self._slots.sum(0))
        last_v = self._bootstrap_value()
        gae(self.buf_rew, self.buf_val, self.buf_start, last_v, self.last_start,
            cfg.gamma, cfg.gae_lambda, self.buf_adv, self.buf_ret)
        return self._rollout_stats(t0)

    def _rollout_stats(self, t0: float) -> RolloutStats:
        """Monitor-style statistics of the episodes that finished during the rollout, over every
        rank's envs (one small all-reduce per rollout -- the sums of returns, lengths
        and counts, float64), so the logged mean return is the whole job's, not rank 0's shard."""
        local = self._done_stats.clone()
        if self.world > 1:
            dist.all_reduce(self._done_stats, op=dist.ReduceOp.SUM)
        # one host read of the reduced sums and this rank's count (the synchronize of the copy)
        ret_sum, len_sum, c, local_c = torch.cat([self._done_stats, local[2:]]).tolist()
        steps = self.cfg.n_steps * self.env.num_envs
        self.num_timesteps += steps * self.world
        return RolloutStats(episodes=int(c), mean_return=ret_sum / c if c else float("nan"),
                            mean_length=len_sum / c if c else float("nan"),
                            env_steps=steps, seconds=time.perf_counter() - t0,
                            extra={"local_episodes": int(local_c), "ranks": self.world})

    def comm_stats(self, clear: bool = True) -> Optional[dict]:
        """The gradient all-reduces timed since comm_events was set to a list (HIP events around the
        collective and work.wait(), allreduce_mean_): count, mean / median / max microseconds of the
        time each held the optimizer step's stream. None when nothing was timed."""
        if not self.comm_events:
            return None
        torch.cuda.synchronize(self.device)
        us = sorted(a.elapsed_time(b) * 1e3 for a, b in self.comm_events)
        if clear:
            self.comm_events = []
        return {"count": len(us), "mean_us": sum(us) / len(us), "median_us": us[len(us) // 2], "max_us": us[-1]}

    def _bootstrap_value(self) -> torch.Tensor:
        """V(last_obs) for GAE: the MFMA policy kernel when fused (batch-independent rows), else torch."""
        if self._fp is not None:
            return self._fp.value(self.last_obs, self._last_v, self._act_env)
        return self.policy.value(self.last_obs)

    def n_minibatches_per_epoch(self) -> int:
        """Optimizer steps per epoch of train(): SB3's partition of the rollout buffer."""
        return n_minibatches(self.cfg.n_steps * self.env.num_envs, self.batch)

    # ------------------------------------------------------------------------------------
    def train(self, n_epochs: Optional[int] = None, max_minibatches: Optional[int] = None) -> dict:
        cfg, pol = self.cfg, self.policy
        total = cfg.n_steps * self.env.num_envs
        obs = self.buf_obs.view(total, self.obs_dim)
        act = self.buf_act.view(total, 4)
        logp_old = self.buf_logp.view(total)
        adv_all = self.buf_adv.view(total)
        ret = self.buf_ret.view(total)
        B = self.batch
        nmb = n_minibatches(total, B)
        stats = dict(pg_loss=0.0, vf_loss=0.0, entropy=0.0, clip_fraction=0.0, n=0)
        acc = torch.zeros(4, dtype=torch.float64, device=self.device)
        epochs = n_epochs if n_epochs is not None else cfg.n_epochs
        if self._learner is not None:
            return self._train_fused(obs, act, logp_old, adv_all, ret, B, nmb, epochs, max_minibatches, stats)
        done = 0
        for _ in range(epochs):
            perm = epoch_permutation(total, self.device)
            for m in range(nmb):
                if max_minibatches is not None and done >= max_minibatches:
                    break
                idx = perm[m * B:min(total, (m + 1) * B)]
                loss, pg, vf, ent, cf = ppo_loss(pol, obs[idx], act[idx], logp_old[idx],
                                                 adv_all[idx], ret[idx], cfg)
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.world > 1:
                    allreduce_mean_(self.params, self._flat, self.world, timing=self.comm_events)
                nn.utils.clip_grad_norm_(self.params, cfg.max_grad_norm)
                self.opt.step()
                with torch.no_grad():
                    acc += torch.stack([pg.detach().double(), vf.detach().double(),
                                        ent.detach().double(), cf.double()])
                done += 1
        a = (acc / max(done, 1)).tolist()
        stats.update(pg_loss=a[0], vf_loss=a[1], entropy=a[2], clip_fraction=a[3], n=done)
        return stats

    def _train_fused(self, obs, act, logp_old, adv, ret, B, nmb, epochs, max_minibatches, stats) -> dict:
        """PPO.train with the minibatch gradient from quad_ppo_grad (no autograd graph, no
        minibatch copies), the flat-bucket all-reduce, then clip_grad_norm_ + Adam as quad_clip_adam."""
        cfg = self.cfg
        total = obs.shape[0]
        if (cfg.graph_update and self.world == 1 and max_minibatches is None and total % B == 0
                and 1 <= nmb <= EPOCH_STATS_MAX_MINIBATCHES and epochs >= 1):
            return self._train_graphed(obs, act, logp_old, adv, ret, B, nmb, epochs, stats)
        steps = epochs * nmb if max_minibatches is None else min(epochs * nmb, max_minibatches)
        mstats = torch.zeros(max(steps, 1), 4, dtype=torch.float32, device=self.device)
        perms, sums = {}, {}
        # the full minibatches' advantage statistics of an epoch in one launch when that launch fits
        # (grid y <= 65,535 minibatches, 4 KB of float64 sums each); a short last minibatch (SB3
        # yields one when batch_size does not divide the buffer) and larger counts run grads' own
        # statistics pre-pass -- the same sums either way
        n_full = total // B
        epoch_stats = 1 <= n_full <= EPOCH_STATS_MAX_MINIBATCHES

        def index_of(k):  # the k-th minibatch of the update: epoch k // nmb, slot k % nmb
            e, m = divmod(k, nmb)
            if e not in perms:  # drawn in epoch order, as the per-epoch loop drew them
                perms[e] = epoch_permutation(total, self.device)
                # every minibatch's advantage statistics of the epoch in one launch (the rollout
                # buffer's advantages do not change during the update)
                sums[e] = self._learner.adv_stats_epoch(adv, perms[e], B, n_full) if epoch_stats else None
            row = sums[e][m] if sums[e] is not None and m < n_full else None
            return perms[e][m * B:min(total, (m + 1) * B)], row

        done = 0
        for k in range(steps):
            idx, adv_sums = index_of(k)
            self._learner.grads(obs, act, logp_old, adv, ret, idx, mstats[k], adv_sums=adv_sums)
            if self.world > 1:
                allreduce_mean_(self.params, self._flat, self.world, timing=self.comm_events)
            self._adam.step()  # clip_grad_norm_ + Adam.step (quad_clip_adam)
            perms.pop(k // nmb - 1, None)
            sums.pop(k // nmb - 1, None)
            done += 1
        a = mstats[:done].double().mean(0).tolist() if done else [0.0] * 4
        stats.update(pg_loss=a[0], vf_loss=a[1], entropy=a[2], clip_fraction=a[3], n=done)
        return stats

    def _epoch_steps(self, obs, act, logp_old, adv, ret, B, nmb, perm, sums, mstats) -> None:
        """One epoch of the fused update on fixed buffers: the epoch's advantage statistics (one
        launch), then per minibatch quad_ppo_grad + quad_clip_adam -- the launch sequence
        _train_fused issues, on the permutation in `perm`."""
        if self._learner.normalize_advantage:
            self._learner.adv_stats_epoch(adv, perm, B, nmb, out=sums)
        for m in range(nmb):
            self._learner.grads(obs, act, logp_old, adv, ret, perm[m * B:(m + 1) * B], mstats[m],
                                adv_sums=sums[m] if self._learner.normalize_advantage else None)
            self._adam.step()

    def _train_graphed(self, obs, act, logp_old, adv, ret, B, nmb, epochs, stats) -> dict:
        """_train_fused for one GPU when the minibatches tile the buffer: every epoch's launches
        (advantage statistics + nmb x (quad_ppo_grad + quad_clip_adam)) captured once as a hipGraph
        on persistent permutation / statistics buffers and replayed per epoch after the epoch's
        permutation is drawn into its buffer -- the same kernels on the same data in the same
        order as the eager loop (the same bits), without its per-launch host work (at train.py's
        scale, 8 envs x 1,024 steps in minibatches of 128, that host work was most of the update).
        The first epoch after a (re)capture runs eagerly; its launches warm the workspaces. The graph
        is recaptured whenever anything its launches took by value changes: the buffers, the batch
        partition, or the optimizer's state tensors / hyperparameters (FusedAdam.signature)."""
        total, dev = obs.shape[0], self.device
        key = (B, nmb, tuple(t.data_ptr() for t in (obs, act, logp_old, adv, ret)),
               self._learner.normalize_advantage, self._adam.signature())
        mstats = torch.zeros(epochs * nmb, 4, dtype=torch.float32, device=dev)
        e0 = 0
        if self._epoch_graph is None or self._epoch_graph[0] != key:
            perm = torch.empty(total, dtype=torch.int64, device=dev)
            sums = torch.empty(nmb, N.ADV_SUM_DOUBLES, dtype=torch.float64, device=dev)
            mst = torch.zeros(nmb, 4, dtype=torch.float32, device=dev)
            epoch_permutation(total, dev, out=perm)
            self._epoch_steps(obs, act, logp_old, adv, ret, B, nmb, perm, sums, mstats[:nmb])
            e0 = 1
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    self._epoch_steps(obs, act, logp_old, adv, ret, B, nmb, perm, sums, mst)
            torch.cuda.current_stream(dev).wait_stream(s)
            self._epoch_graph = (key, g, perm, sums, mst)
        _, g, perm, sums, mst = self._epoch_graph
        for e in range(e0, epochs):
            epoch_permutation(total, dev, out=perm)
            g.replay()
            mstats[e * nmb:(e + 1) * nmb].copy_(mst)
        a = mstats.double().mean(0).tolist()
        stats.update(pg_loss=a[0], vf_loss=a[1], entropy=a[2], clip_fraction=a[3], n=epochs * nmb)
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
        """What a resumed run needs: policy, optimizer (Adam moments, step counts), the timestep
        count and the rollout's action-noise counter (so resumed rollouts draw fresh noise)."""
        noise = self._t_host if self._one_launch else int(self._cursor[0].item())
        return {"policy": self.policy.state_dict(), "optimizer": self.opt.state_dict(),
                "num_timesteps": self.num_timesteps, "noise_step": noise}

    def load_state_dict(self, sd: dict) -> None:
        """Restore state_dict() (parameters are copied in place, so the gradient bucket binding
        and the fused kernels' pointers stay valid). Envs restart from reset, as SB3's
        PPO.load + learn(reset_num_timesteps=False) does."""
        self.policy.load_state_dict(sd["policy"])
        self.opt.load_state_dict(sd["optimizer"])
        for st in self.opt.state.values():  # fused Adam keeps its step counters on the device
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = st["step"].to(device=self.device, dtype=torch.float32)
        self._epoch_graph = None  # its launches hold the replaced Adam state tensors
        self.num_timesteps = int(sd["num_timesteps"])
        ns = int(sd.get("noise_step", 0))
        self._t_host = ns
        # the two-launch path keys its noise on the device cursor, whose step count also selects the
        # buffer row (t % n_steps): resume at the next rollout boundary
        T = self.cfg.n_steps
        self._cursor_resume = ((ns + T - 1) // T) * T
        self._started = False
