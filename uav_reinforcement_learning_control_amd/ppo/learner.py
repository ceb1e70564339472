"""The PPO minibatch gradient on MFMA (csrc/learner.hip via quad_ppo_grad), bound to a torch
ActorCritic.

SB3 PPO.train (the learner the reference's train.py:50-68 configures; ppo/ppo.py `ppo_loss` restates
its loss) computes, per minibatch, the clipped-surrogate + entropy + value loss and backpropagates it
through both MLPs. `FusedLearner.grads` writes that gradient straight into the parameters' `.grad`
tensors in three launches (advantage statistics, the fused forward/backward of both nets, a
deterministic reduction of the per-block partials), gathering the minibatch rows from the rollout
buffer through the permutation slice -- no minibatch copies, no autograd graph. After the
(multi-GPU) gradient all-reduce, `FusedAdam.step` does clip_grad_norm_ + Adam.step in two launches
on torch's own optimizer state.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from .. import _native as N
from .fused import FusedPolicy, _need
from .policy import ActorCritic


def _ordered(policy: ActorCritic):
    ex = policy.mlp_extractor
    return [ex.policy_net[0].weight, ex.policy_net[0].bias, ex.policy_net[2].weight, ex.policy_net[2].bias,
            policy.action_net.weight, policy.action_net.bias,
            ex.value_net[0].weight, ex.value_net[0].bias, ex.value_net[2].weight, ex.value_net[2].bias,
            policy.value_net.weight, policy.value_net.bias, policy.log_std]


class FusedLearner:
    """quad_ppo_grad for a 12-128-128-(4|1) ActorCritic (SB3 PPO loss semantics)."""

    def __init__(self, policy: ActorCritic, clip_range: float, ent_coef: float, vf_coef: float,
                 normalize_advantage: bool = True):
        FusedPolicy._check_shapes(policy)
        self.policy = policy
        self.device = policy.log_std.device
        if self.device.type != "cuda":
            raise N.QuadError("FusedLearner needs the policy on a ROCm GPU")
        self.clip_range, self.ent_coef, self.vf_coef = float(clip_range), float(ent_coef), float(vf_coef)
        self.normalize_advantage = bool(normalize_advantage)
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self._lib = N.lib()

    def _structs(self):
        ps = _ordered(self.policy)
        for p in ps:
            if not p.is_contiguous() or p.dtype != torch.float32:
                raise ValueError("policy parameters must be contiguous float32")
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            elif not p.grad.is_contiguous():
                raise ValueError("parameter gradients must be contiguous")
        return (N.QuadPolicyParams(*[p.data_ptr() for p in ps]),
                N.QuadPolicyGrads(*[p.grad.data_ptr() for p in ps]))

    def _workspace(self, B: int) -> None:
        need = int(self._lib.quad_ppo_workspace_bytes(B))
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)

    def adv_stats(self, advantages: torch.Tensor, index: torch.Tensor) -> None:
        """Enqueue the advantage statistics of minibatch `index` (quad_ppo_adv_stats) into the
        workspace the next grads(..., adv_ready=True) reads; nothing else may run grads in between."""
        if not self.normalize_advantage:
            return
        B = int(index.numel())
        self._workspace(B)
        b = N.QuadPPOBatch(0, 0, 0, advantages.data_ptr(), 0, index.data_ptr(), B, 1, 0.2, 0.0, 0.0, None)
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(self._lib.quad_ppo_adv_stats(C.byref(b), C.c_void_p(self._ws.data_ptr()), C.c_int64(self._ws.numel()),
                                             stream), "quad_ppo_adv_stats")

    def adv_stats_epoch(self, advantages: torch.Tensor, perm: torch.Tensor, batch: int, n_minibatches: int,
                        out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """The advantage statistics of every minibatch of an epoch in one launch
        (quad_ppo_adv_stats_epoch): minibatch m = perm[m * batch:(m + 1) * batch]; row m of the
        returned float64 [n_minibatches, 512] tensor is what grads(..., adv_sums=row) normalizes with
        (bit-identical to the per-minibatch pre-pass). None without advantage normalization."""
        if not self.normalize_advantage:
            return None
        if perm.dtype != torch.int64 or not perm.is_contiguous() or perm.numel() < batch * n_minibatches:
            raise ValueError("perm: a contiguous int64 vector of at least batch * n_minibatches rows")
        if out is None or tuple(out.shape) != (n_minibatches, N.ADV_SUM_DOUBLES):
            out = torch.empty(n_minibatches, N.ADV_SUM_DOUBLES, dtype=torch.float64, device=self.device)
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(self._lib.quad_ppo_adv_stats_epoch(C.c_void_p(advantages.data_ptr()), C.c_void_p(perm.data_ptr()),
                                                   int(batch), int(n_minibatches), C.c_void_p(out.data_ptr()), stream),
                "quad_ppo_adv_stats_epoch")
        return out

    def grads(self, obs: torch.Tensor, actions: torch.Tensor, log_prob: torch.Tensor, advantages: torch.Tensor,
              returns: torch.Tensor, index: torch.Tensor, stats: Optional[torch.Tensor] = None,
              hidden: Optional[torch.Tensor] = None, adv_ready: bool = False,
              adv_sums: Optional[torch.Tensor] = None) -> None:
        """Overwrite every parameter's .grad with the gradient of the PPO loss on rows `index` of the
        flattened buffers (obs [M,12], actions [M,4], log_prob / advantages / returns [M]).
        `stats` (float32 [4], optional) receives pg_loss, vf_loss, entropy, clip_fraction.
        `hidden` (float32 [2, B, 256], diagnostics): run the kernel's dump build (quad_ppo_hidden),
        which also records each row's hidden pre-activations [net][pos][h1 | h2].
        `adv_ready`: adv_stats(advantages, index) was already enqueued for this minibatch, so the
        launch sequence skips its own statistics pre-pass. `adv_sums`: this minibatch's row of
        adv_stats_epoch (the statistics pre-pass is skipped; same bits)."""
        dev = self.device
        M = obs.shape[0]
        _need(obs, (M, 12), torch.float32, dev, "obs")
        _need(actions, (M, 4), torch.float32, dev, "actions")
        for t, n in ((log_prob, "log_prob"), (advantages, "advantages"), (returns, "returns")):
            _need(t, (M,), torch.float32, dev, n)
        if index.dtype != torch.int64 or index.dim() != 1 or not index.is_contiguous() or index.device != dev:
            raise ValueError("index: expected a contiguous int64 vector on the policy's device")
        B = int(index.numel())
        if B < 1:
            raise ValueError("empty minibatch")
        if stats is not None:
            _need(stats, (4,), torch.float32, dev, "stats")
        self._workspace(B)
        prm, grd = self._structs()
        norm = int(self.normalize_advantage)
        if norm and adv_sums is not None:
            if adv_sums.dtype != torch.float64 or adv_sums.numel() != N.ADV_SUM_DOUBLES or not adv_sums.is_contiguous():
                raise ValueError("adv_sums: one contiguous float64 row of adv_stats_epoch")
            norm = N.QUAD_ADV_GIVEN
        elif norm and adv_ready:
            norm = N.QUAD_ADV_PRECOMPUTED
        b = N.QuadPPOBatch(obs.data_ptr(), actions.data_ptr(), log_prob.data_ptr(), advantages.data_ptr(),
                           returns.data_ptr(), index.data_ptr(), B, norm,
                           self.clip_range, self.ent_coef, self.vf_coef,
                           None if stats is None else stats.data_ptr(),
                           adv_sums.data_ptr() if norm == N.QUAD_ADV_GIVEN else None)
        stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        if hidden is not None:
            _need(hidden, (2, B, 256), torch.float32, dev, "hidden")
            N.check(self._lib.quad_ppo_hidden(C.byref(prm), C.byref(b), C.byref(grd), C.c_void_p(hidden.data_ptr()),
                                              C.c_void_p(self._ws.data_ptr()), C.c_int64(self._ws.numel()), stream),
                    "quad_ppo_hidden")
            return
        N.check(self._lib.quad_ppo_grad(C.byref(prm), C.byref(b), C.byref(grd), C.c_void_p(self._ws.data_ptr()),
                                        C.c_int64(self._ws.numel()), stream), "quad_ppo_grad")


def adam_state(opt: torch.optim.Adam, params) -> list:
    """torch.optim.Adam's per-parameter state (step, exp_avg, exp_avg_sq), created the way Adam's
    first step() does (fused/capturable: the step counter is a float32 tensor on the device)."""
    out = []
    for p in params:
        st = opt.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        if st["step"].device != p.device:
            st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
        out.append(st)
    return out


class FusedAdam:
    """clip_grad_norm_(params, max_grad_norm) + opt.step() for a torch.optim.Adam as two launches
    (quad_clip_adam), on the optimizer's own state tensors so state_dict()/checkpoints are unchanged."""

    def __init__(self, opt: torch.optim.Adam, max_grad_norm: float):
        if len(opt.param_groups) != 1:
            raise ValueError("FusedAdam expects one parameter group")
        grp = opt.param_groups[0]
        if grp.get("amsgrad") or grp.get("maximize") or grp.get("weight_decay", 0.0) != 0.0:
            raise ValueError("FusedAdam implements plain Adam (no amsgrad / maximize / weight decay)")
        self.opt, self.params = opt, list(grp["params"])
        if len(self.params) > N.ADAM_MAX_TENSORS:
            raise ValueError("too many parameter tensors")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device.type != "cuda":
                raise ValueError("parameters must be contiguous float32 on a ROCm GPU")
        self.max_grad_norm = float(max_grad_norm)
        self._lib = N.lib()
        self._ws = None

    def _build(self):
        grp = self.opt.param_groups[0]
        st = adam_state(self.opt, self.params)
        a = N.QuadAdam()
        for i, (p, s) in enumerate(zip(self.params, st)):
            if p.grad is None or not p.grad.is_contiguous():
                raise ValueError("every parameter needs a contiguous .grad")
            a.params[i], a.grads[i] = p.data_ptr(), p.grad.data_ptr()
            a.exp_avg[i], a.exp_avg_sq[i], a.step[i] = (s["exp_avg"].data_ptr(), s["exp_avg_sq"].data_ptr(),
                                                        s["step"].data_ptr())
            a.numel[i] = p.numel()
        a.count = len(self.params)
        b1, b2 = grp["betas"]
        a.lr, a.beta1, a.beta2, a.eps, a.max_grad_norm = float(grp["lr"]), b1, b2, float(grp["eps"]), self.max_grad_norm
        return a

    def signature(self) -> tuple:
        """Everything a quad_clip_adam launch takes by value: the parameter, gradient and Adam-state
        pointers and the hyperparameters. A hipGraph that captured step() replays correctly only
        while this is unchanged (Optimizer.load_state_dict replaces the state tensors; a changed
        lr is a new kernel argument)."""
        a = self._build()
        return tuple((a.params[i], a.grads[i], a.exp_avg[i], a.exp_avg_sq[i], a.step[i]) for i in range(a.count)) + \
            (a.lr, a.beta1, a.beta2, a.eps, a.max_grad_norm)

    def step(self) -> None:
        a = self._build()
        if self._ws is None:
            self._ws = torch.empty(max(int(self._lib.quad_adam_workspace_bytes(C.byref(a))), 4), dtype=torch.uint8,
                                   device=self.params[0].device)
        stream = C.c_void_p(torch.cuda.current_stream(self.params[0].device).cuda_stream)
        N.check(self._lib.quad_clip_adam(C.byref(a), C.c_void_p(self._ws.data_ptr()), C.c_int64(self._ws.numel()),
                                         stream), "quad_clip_adam")
