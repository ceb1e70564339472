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


def RateControlWrapper(env, max_rate: Optional[float] = None, kd=None,
                       ki_rate_torque: Optional[float] = None,
                       integral_max: Optional[float] = None):
    """Return `env` rebuilt with the CTBR controller in the step kernel."""
    o = _gain_overrides(max_rate, kd, ki_rate_torque, integral_max)
    if isinstance(env, QuadVecEnv):
        over = {}
        new = QuadVecEnv(env.num_envs, env=env.env_kind, wrapper="RateControlWrapper",
                         device=env.device, seed=env.seed_value, env_id_base=env.env_id_base,
                         max_episode_steps=env.max_episode_steps,
                         auto_reset=bool(env.cfg.auto_reset), cfg_overrides={**over, **o})
        env.close()
        return new
    if isinstance(env, HoverEnv):
        new = type(env)(render_mode=env.render_mode, max_episode_steps=env.max_episode_steps,
                        device=env._vec.device, wrapper="RateControlWrapper", **o)
        env.close()
        return new
    raise TypeError(f"cannot wrap {type(env).__name__}")
