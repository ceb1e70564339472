"""Actor-critic matching SB3's ActorCriticPolicy as configured by the reference (train.py:50-68):
net_arch [128, 128], ReLU, separate policy / value MLPs, state-independent log_std (init 0),
orthogonal init (gain sqrt(2) hidden, 0.01 action head, 1 value head, zero biases), diagonal
Gaussian actions (not squashed; clipped to the action box only when sent to the env).

Parameter names follow SB3's state_dict (mlp_extractor.policy_net.{0,2}, mlp_extractor.value_net.
{0,2}, action_net, value_net, log_std) so a trained policy can be exported for the reference's
consumers (evaluate.py / ROS2 policy_node.py load SB3 zips).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn


class _SplitKLinear(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is split over row chunks.

    PPO minibatches are tall (524,288 rows at the default schedule) while W is at most 128 x 128,
    so dW = dY^T X is a GEMM with a tiny output and a huge K; the BLAS picks un-split tiles for it
    (~1 ms each on MI355X). Chunking K into C slabs of ~4k rows turns it into a batched GEMM with
    C x the parallelism plus a cheap reduction over C.
    """

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy @ w if ctx.needs_input_grad[0] else None
        m = gy.shape[0]
        c = _chunks(m)
        if c > 1:
            gw = torch.bmm(gy.reshape(c, m // c, -1).transpose(1, 2), x.reshape(c, m // c, -1)).sum(0)
        else:
            gw = gy.t() @ x
        return gx, gw, gy.sum(0)


def _chunks(m: int, rows: int = 4096) -> int:
    """Largest power-of-two chunk count with >= `rows` rows per chunk that divides m."""
    c = 1
    while m % (2 * c) == 0 and m // (2 * c) >= rows:
        c *= 2
    return c


def _linear(x: torch.Tensor, layer: nn.Linear) -> torch.Tensor:
    if torch.is_grad_enabled() and x.dim() == 2 and x.shape[0] >= 65536:
        return _SplitKLinear.apply(x, layer.weight, layer.bias)
    return layer(x)


def _trunk(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    for mod in seq:
        x = _linear(x, mod) if isinstance(mod, nn.Linear) else mod(x)
    return x


def _mlp(in_dim: int, hidden=(128, 128)) -> nn.Sequential:
    layers, d = [], in_dim
    for h in hidden:
        layers += [nn.Linear(d, h), nn.ReLU()]
        d = h
    return nn.Sequential(*layers)


class MlpExtractor(nn.Module):
    def __init__(self, obs_dim: int, hidden=(128, 128)):
        super().__init__()
        self.policy_net = _mlp(obs_dim, hidden)
        self.value_net = _mlp(obs_dim, hidden)


class ActorCritic(nn.Module):
    def __init__(self, obs_dim: int = 12, act_dim: int = 4, hidden=(128, 128),
                 log_std_init: float = 0.0):
        super().__init__()
        self.mlp_extractor = MlpExtractor(obs_dim, hidden)
        self.action_net = nn.Linear(hidden[-1], act_dim)
        self.value_net = nn.Linear(hidden[-1], 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))
        self.act_dim = act_dim
        # SB3 ActorCriticPolicy._build: orthogonal init with these gains
        for mod, gain in ((self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01),
                          (self.value_net, 1.0)):
            for m in mod.modules():
                if isinstance(m, nn.Linear):
                    nn.init.orthogonal_(m.weight, gain=gain)
                    nn.init.zeros_(m.bias)

    def forward_heads(self, obs: torch.Tensor):
        mean = _linear(_trunk(self.mlp_extractor.policy_net, obs), self.action_net)
        value = _linear(_trunk(self.mlp_extractor.value_net, obs), self.value_net).squeeze(-1)
        return mean, value

    def value(self, obs: torch.Tensor) -> torch.Tensor:
        return self.value_net(self.mlp_extractor.value_net(obs)).squeeze(-1)

    def log_prob(self, mean: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
        std = self.log_std.exp()
        z = (actions - mean) / std
        return (-0.5 * z * z - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self) -> torch.Tensor:
        return (0.5 + 0.5 * math.log(2 * math.pi) + self.log_std).sum()

    @torch.no_grad()
    def act(self, obs: torch.Tensor, deterministic: bool = False):
        mean, value = self.forward_heads(obs)
        if deterministic:
            a = mean
        else:
            a = mean + self.log_std.exp() * torch.randn_like(mean)
        return a, self.log_prob(mean, a), value
