"""Wrapper registry (envs/wrappers.py:10-36 of the reference): get_wrapper(name) is the plugin
point drivers use via config.json["wrapper"] (train.py:95, evaluate.py:320)."""
from __future__ import annotations

import numpy as np

from .rate_wrapper import RateControlWrapper


class RelPosActWrapper:
    """7-D observation [normalized rel pos (3), previous action (4)] (wrappers.py:13-25)."""

    def __init__(self, env):
        from ..utils.spaces import Box
        self.env = env
        self.observation_space = Box(-1.0, 1.0, (7,), np.float32)
        self.action_space = env.action_space

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def observation(self, obs):
        return np.concatenate([obs[0:3], self.unwrapped._prev_action]).astype(np.float32)

    def reset(self, **kw):
        o, i = self.env.reset(**kw)
        return self.observation(o), i

    def step(self, a):
        o, r, te, tr, i = self.env.step(a)
        return self.observation(o), r, te, tr, i


WRAPPER_REGISTRY = {"RelPosActWrapper": RelPosActWrapper,
                    "RateControlWrapper": RateControlWrapper}


def get_wrapper(name):
    if name is None or name == "none":
        return None
    return WRAPPER_REGISTRY[name]
