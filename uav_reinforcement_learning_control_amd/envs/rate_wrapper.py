"""RateControlWrapper (envs/rate_wrapper.py:26-111 of the reference).

The CTBR rate controller is fused into the step kernel (QuadCfg.wrapper = QUAD_WRAP_CTBR) with
the reference's defaults from pid_gains.json:43-52 (kd 26/26/18, ki 0.025, imax 0.01,
360 deg/s). Wrapping an env therefore rebuilds it with the wrapper enabled.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .hover_env import HoverEnv
from .vec_env import QuadVecEnv


def rebuild(env, wrapper: str, extra: Optional[dict] = None):
    """A copy of `env` (a QuadVecEnv or a HoverEnv / TrajectoryFollowEnv facade) with the kernel's
    wrapper kind `wrapper`: same size, device, seed, env ids, episode length, auto-reset and
    cfg overrides (+ `extra`), so wrapping never changes the dynamics or bounds of a customized env."""
    if isinstance(env, QuadVecEnv):
        return QuadVecEnv(env.num_envs, env=env.env_kind, wrapper=wrapper, device=env.device,
                          seed=env.seed_value, env_id_base=env.env_id_base,
                          max_episode_steps=env.max_episode_steps, auto_reset=bool(env.cfg.auto_reset),
                          cfg_overrides={**env.cfg_overrides, **(extra or {})})
    if isinstance(env, HoverEnv):
        return type(env)(render_mode=env.render_mode, max_episode_steps=env.max_episode_steps,
                         device=env._vec.device, wrapper=wrapper, seed=env._seed,
                         **{**env._overrides, **(extra or {})})
    raise TypeError(f"cannot wrap {type(env).__name__}")


def _gain_overrides(max_rate, kd, ki_rate_torque, integral_max):
    o = {}
    if max_rate is not None:
        o["rate_max_rad"] = float(np.deg2rad(max_rate))
    if kd is not None:
        o["rate_kd"] = [float(x) for x in kd]
    if ki_rate_torque is not None:
        o["rate_ki"] = float(ki_rate_torque)
    if integral_max is not None:
        o["rate_imax"] = float(integral_max)
    return o


def _wrapper_of(env):
    if isinstance(env, QuadVecEnv):
        return env.wrapper
    if isinstance(env, HoverEnv):
        return env._vec.wrapper
    raise TypeError(f"cannot wrap {type(env).__name__}")


class RateControlWrapper:
    """gym.ActionWrapper-shaped facade of the reference's RateControlWrapper (rate_wrapper.py:26-111).

    The PID rate controller itself runs inside the step kernel (QuadCfg.wrapper = QUAD_WRAP_CTBR,
    csrc/quad_physics.h env_step<.., CTBR>): wrapping rebuilds `env` (a QuadVecEnv or a
    HoverEnv / TrajectoryFollowEnv facade) with the controller on and the given gains, and this
    object forwards the env API to it. What the reference exposes is kept: `env`, `unwrapped`,
    `max_rate_rad`, `inertia`, `kd`, `ki_rate_torque`, `integral_max`, `_dt`, and
    `_rate_int_torque` (the integral state, read from / written to the device: [3] for a single
    env, [N, 3] for a vectorized one, float64 like the reference's). `step` takes the rate action
    [thrust, roll rate, pitch rate, yaw rate] in [-1, 1]; `reset` zeroes the integral (in-kernel).
    """

    def __init__(self, env, max_rate: Optional[float] = None, kd=None,
                 ki_rate_torque: Optional[float] = None, integral_max: Optional[float] = None):
        o = _gain_overrides(max_rate, kd, ki_rate_torque, integral_max)
        if isinstance(env, (QuadVecEnv, HoverEnv)) and _wrapper_of(env) not in (None, "none"):
            raise TypeError("RateControlWrapper wraps the bare env; stack RelPosActWrapper on top of it "
                            "(RelPosActWrapper(RateControlWrapper(env)), as the reference README does)")
        inner = rebuild(env, "RateControlWrapper", o)
        cfg = inner.cfg if isinstance(inner, QuadVecEnv) else inner._vec.cfg
        env.close()
        self.env = inner
        self._single = not isinstance(inner, QuadVecEnv)
        self.max_rate_rad = float(cfg.rate_max_rad)
        self.inertia = np.array(cfg.inertia[:], np.float64)
        self.kd = np.array(cfg.rate_kd[:], np.float64)
        self.ki_rate_torque = float(cfg.rate_ki)
        self.integral_max = float(cfg.rate_imax)
        self._dt = float(cfg.timestep)
        self.action_space = inner.action_space
        self.observation_space = inner.observation_space

    def __getattr__(self, name):  # everything else is the wrapped env's (num_envs, cfg, ...)
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def _vec_env(self) -> QuadVecEnv:
        return self.env._vec if self._single else self.env

    @property
    def _rate_int_torque(self) -> np.ndarray:
        ri = self._vec_env.get_state()["rate_int"].astype(np.float64)
        return ri[0] if self._single else ri

    @_rate_int_torque.setter
    def _rate_int_torque(self, value) -> None:
        v = np.asarray(value, np.float32).reshape(self._vec_env.num_envs, 3)
        self._vec_env.set_state(rate_int=v)

    def step(self, action, *args, **kw):
        out = self.env.step(action, *args, **kw)
        if self._single:  # rate_wrapper.py:105: observation wrappers see the rate action
            self.unwrapped._prev_action = np.asarray(action, np.float32).reshape(4).copy()
        return out

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def close(self) -> None:
        self.env.close()
