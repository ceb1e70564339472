"""Minimal stand-in for gymnasium (golden-vector generation only; see ../README.md)."""
import numpy as np

from . import spaces  # noqa: F401


class Env:
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random = np.random.default_rng(seed)

    @property
    def unwrapped(self):
        return self


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)


class ActionWrapper(Wrapper):
    def step(self, action):
        return self.env.step(self.action(action))


class ObservationWrapper(Wrapper):
    def step(self, action):
        o, r, te, tr, i = self.env.step(action)
        return self.observation(o), r, te, tr, i

    def reset(self, **kwargs):
        o, i = self.env.reset(**kwargs)
        return self.observation(o), i
