"""Gymnasium-style single-env facades with the reference's API (numpy in / numpy out).

HoverEnv           -> envs/hover_env.py:13-257 of the reference
TrajectoryFollowEnv-> envs/trajectory_follow_env.py:14-269 (obs/reward target = start
                      position, as in the reference; the moving spline is info-only there)

Each instance is a 1-env QuadVecEnv without auto-reset, so stepping a terminated env keeps
integrating exactly like the reference. Every call round-trips to the GPU: use QuadVecEnv for
throughput; these exist so code written against the reference's env API runs unchanged.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .vec_env import QuadVecEnv


class _QuadState:
    """The subset of utils.state.QuadState the reference's wrappers read."""

    def __init__(self):
        self.state = np.zeros(12, np.float32)

    position = property(lambda s: s.state[0:3])
    attitude = property(lambda s: s.state[3:6])
    velocity = property(lambda s: s.state[6:9])
    angular_velocity = property(lambda s: s.state[9:12])

    def vec(self):
        return self.state.copy()


class HoverEnv:
    _KIND = "hover"

    def __init__(self, render_mode: Optional[str] = None, max_episode_steps: Optional[int] = None,
                 device=None, wrapper: Optional[str] = None, seed: int = 0, **cfg_overrides):
        self.render_mode = render_mode
        self._seed, self._overrides = int(seed), dict(cfg_overrides)  # (wrappers rebuild with them)
        self._vec = QuadVecEnv(1, env=self._KIND, wrapper=wrapper, device=device, seed=seed,
                               max_episode_steps=max_episode_steps, auto_reset=False,
                               cfg_overrides=cfg_overrides or None)
        self.max_episode_steps = self._vec.max_episode_steps
        self.action_space = self._vec.action_space
        self.observation_space = self._vec.observation_space
        self.dt = self._vec.dt
        self._state = _QuadState()
        self.target_state = _QuadState()
        self._prev_action = np.zeros(4, np.float32)
        self._step_count = 0

    @property
    def unwrapped(self):
        return self

    @property
    def voltage(self) -> float:
        return float(self._vec.get_state()["voltage"][0])

    def _sync_state(self):
        st = self._vec.get_state()
        self.target_state.state[0:3] = st["target"][0]
        self._step_count = int(st["step_count"][0])
        return st

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        obs = self._vec.reset(seed=seed).cpu().numpy()[0].copy()
        self._prev_action = np.zeros(4, np.float32)
        st = self._sync_state()
        # the reset state is the drawn state (QuadState round trip, hover_env.py:219-230)
        self._state.state[:] = self._state_from(st)
        info = {"state": self._state.vec(), "target": self.target_state.position.copy(),
                "voltage": float(st["voltage"][0]),
                "voltage_scale": float(min(max(st["voltage"][0] / self._vec.cfg.nominal_voltage,
                                               0.0), 1.0))}
        return obs, info

    def _state_from(self, st):
        _, s12 = self._vec.observe(state=True)
        return s12.cpu().numpy()[0]

    def step(self, action):
        a = np.asarray(action, dtype=np.float32).reshape(1, 4)
        self._prev_action = a[0].copy()
        at = torch.from_numpy(a).to(self._vec.device)
        obs, r, te, tr, inf = self._vec.step(at, info="full")
        obs = obs.cpu().numpy()[0].copy()
        self._state.state[:] = inf["state"].cpu().numpy()[0]
        st = self._sync_state()
        info = {"state": self._state.vec(),
                "motor_commands": inf["motor_commands"].cpu().numpy()[0].astype(np.float64),
                "target": inf["target"].cpu().numpy()[0].copy(),
                "voltage": float(st["voltage"][0]),
                "voltage_scale": float(inf["voltage_scale"].cpu().numpy()[0])}
        if self._KIND == "trajectory":  # trajectory_follow_env.py:163-168 (spline sample)
            info["target_vel"] = inf["target_vel"].cpu().numpy()[0].copy()
            info["target_acc"] = inf["target_acc"].cpu().numpy()[0].copy()
        return obs, float(r.cpu().numpy()[0]), bool(te.cpu()[0]), bool(tr.cpu()[0]), info

    def set_state(self, qpos, qvel):
        """HoverEnv.set_state (hover_env.py:143-148): base qpos[:7] / qvel[:6]."""
        st = self._vec.get_state()
        qp = st["qpos"].copy(); qv = st["qvel"].copy()
        qp[0, :7] = qpos; qv[0, :6] = qvel
        self._vec.set_state(qpos=qp, qvel=qv)

    def render(self):
        return None

    def close(self):
        self._vec.close()


class TrajectoryFollowEnv(HoverEnv):
    _KIND = "trajectory"
