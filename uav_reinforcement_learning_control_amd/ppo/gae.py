"""GAE(lambda) reverse scan on the GPU (k_gae in csrc/quadenv.hip).

Semantics of SB3 RolloutBuffer.compute_returns_and_advantage (the learner train.py:50-68 uses):
time-major [T, N] buffers, episode_starts[t] = 1 where obs t began an episode, `dones` the done
flags after the last step, returns = advantages + values.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from .. import _native as N


def gae(rewards: torch.Tensor, values: torch.Tensor, episode_starts: torch.Tensor,
        last_values: torch.Tensor, dones: torch.Tensor, gamma: float, gae_lambda: float,
        advantages: Optional[torch.Tensor] = None, returns: Optional[torch.Tensor] = None):
    T, n = rewards.shape
    dev = rewards.device
    for t, shp in ((rewards, (T, n)), (values, (T, n)), (episode_starts, (T, n)),
                   (last_values, (n,)), (dones, (n,))):
        if t.dtype != torch.float32 or tuple(t.shape) != shp or not t.is_contiguous() or t.device != dev:
            raise ValueError(f"gae: expected contiguous float32 {shp} on {dev}")
    advantages = torch.empty_like(rewards) if advantages is None else advantages
    returns = torch.empty_like(rewards) if returns is None else returns
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda x: C.c_void_p(x.data_ptr())
    N.check(N.lib().quad_gae(p(rewards), p(values), p(episode_starts), p(last_values), p(dones),
                             T, n, float(gamma), float(gae_lambda), p(advantages), p(returns), s),
            "quad_gae")
    return advantages, returns
