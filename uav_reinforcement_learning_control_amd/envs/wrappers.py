"""Wrapper registry (envs/wrappers.py:10-36 of the reference): get_wrapper(name) is the plugin
point drivers use via config.json["wrapper"] (train.py:95, evaluate.py:320)."""
from __future__ import annotations

import numpy as np

from .rate_wrapper import RateControlWrapper


class RelPosActWrapper:
    """gym.ObservationWrapper-shaped facade of RelPosActWrapper (wrappers.py:13-25): 7-D
    observation [normalized rel pos (3), previous action (4)].

    The observation is produced by the step kernel's output stage (QuadCfg.wrapper =
    QUAD_WRAP_RELPOS, k_step_relpos): wrapping rebuilds `env` (a QuadVecEnv or a HoverEnv /
    TrajectoryFollowEnv facade) with that wrapper kind -- same seed, env ids and cfg overrides --
    so step/reset already return obs7. Wrapping a RateControlWrapper (the README's
    RelPosActWrapper(RateControlWrapper(HoverEnv())) stack) rebuilds the env under it with the
    combined kind QUAD_WRAP_CTBR_RELPOS: the rate controller stays in the step and obs7 carries the
    rate action (rate_wrapper.py:100-106); `env` is then that RateControlWrapper.
    `observation(obs12)` is the reference's mapping, for callers that apply it themselves."""

    def __init__(self, env):
        from ..utils.spaces import Box
        from .rate_wrapper import _wrapper_of, rebuild
        if isinstance(env, RateControlWrapper):
            old = env.env
            env.env = rebuild(old, "ctbr_relpos")  # gains travel in the cfg overrides
            old.close()
            env.observation_space = env.env.observation_space  # the wrapper below now returns obs7
            self.env = env
        else:
            # an env built with a wrapper kind already: CTBR stacks (the rate controller must stay in
            # the step), an observation wrapper twice is refused
            kind = _wrapper_of(env)
            if kind in ("RateControlWrapper", "ctbr"):
                target = "ctbr_relpos"
            elif kind in (None, "none"):
                target = "RelPosActWrapper"
            else:
                raise TypeError(f"RelPosActWrapper: the env already has the {kind!r} wrapper kind")
            inner = rebuild(env, target)
            env.close()
            self.env = inner
        self.observation_space = Box(-1.0, 1.0, (7,), np.float32)
        self.action_space = self.env.action_space

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def observation(self, obs):
        return np.concatenate([obs[0:3], self.unwrapped._prev_action]).astype(np.float32)

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, a, *args, **kw):
        return self.env.step(a, *args, **kw)

    def close(self) -> None:
        self.env.close()


WRAPPER_REGISTRY = {"RelPosActWrapper": RelPosActWrapper,
                    "RateControlWrapper": RateControlWrapper}


def get_wrapper(name):
    if name is None or name == "none":
        return None
    return WRAPPER_REGISTRY[name]
