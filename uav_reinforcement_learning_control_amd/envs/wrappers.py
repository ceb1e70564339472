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
    TrajectoryFollowEnv facade) with that wrapper kind, so step/reset already return obs7.
    `observation(obs12)` is the reference's mapping, for callers that apply it themselves."""

    def __init__(self, env):
        from ..utils.spaces import Box
        from .hover_env import HoverEnv
        from .vec_env import QuadVecEnv
        if isinstance(env, QuadVecEnv):
            inner = QuadVecEnv(env.num_envs, env=env.env_kind, wrapper="RelPosActWrapper", device=env.device,
                               seed=env.seed_value, env_id_base=env.env_id_base,
                               max_episode_steps=env.max_episode_steps, auto_reset=bool(env.cfg.auto_reset))
        elif isinstance(env, HoverEnv):
            inner = type(env)(render_mode=env.render_mode, max_episode_steps=env.max_episode_steps,
                              device=env._vec.device, wrapper="RelPosActWrapper")
        else:
            raise TypeError(f"cannot wrap {type(env).__name__}")
        env.close()
        self.env = inner
        self.observation_space = Box(-1.0, 1.0, (7,), np.float32)
        self.action_space = inner.action_space

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
