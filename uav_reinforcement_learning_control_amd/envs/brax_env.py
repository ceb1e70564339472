"""brax Env API over the batched kernels.

The reference's second public API for this path is brax's functional ``Env``
(train_brax_ppo.py:39-368): ``reset(rng) -> State``, ``step(State, action) -> State``, properties
``observation_size``, ``action_size``, ``backend``, and ``State(pipeline_state, obs, reward, done,
metrics, info)``. ``QuadBraxEnv`` presents that API for a whole batch at once, i.e. the env as
brax's ``ppo.train`` sees it after ``wrap_for_training`` (VmapWrapper + EpisodeWrapper +
AutoResetWrapper):

  * ``env="hover"``        QuadHoverBraxEnv   (fixed target (0,0,1), reward exp(-2 e^2), done
                           outside |x|,|y| <= 3, z in [0.02, 4]);
  * ``env="jax_mjx_quad"`` JaxMJXQuadBraxEnv  (sinusoid target, NaN/velocity guards, reward
                           exp(-e^2) - 0.001 |a|^2 or -1);
  * ``done`` = env done or ``steps >= episode_length`` (EpisodeWrapper), ``info["truncation"]``
    = episode-length cut of a not-done env, and done envs come back in the FIRST state of their
    episode (AutoResetWrapper);
  * ``obs`` = raw ``[qpos(11), qvel(10)]`` float32, ``pipeline_state`` = ``{"q", "qd"}`` views.

Unlike JAX, the state lives on the GPU inside the handle: ``step`` must be given the State that
the previous ``reset``/``step`` returned (stepping an older State is not supported). The reset
noise is Philox (JAX threefry is absent here): same distribution, different stream.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Optional

import torch

from .vec_env import QuadVecEnv

_KINDS = {"hover": "brax_hover", "QuadHoverBraxEnv": "brax_hover",
          "jax_mjx_quad": "brax_jax_mjx", "JaxMJXQuadBraxEnv": "brax_jax_mjx"}


@dataclass
class State:
    """brax.envs.base.State for a batch (tensors [N, ...] on the env's device)."""
    pipeline_state: dict
    obs: torch.Tensor
    reward: torch.Tensor
    done: torch.Tensor
    metrics: dict = field(default_factory=dict)
    info: dict = field(default_factory=dict)

    def replace(self, **kw) -> "State":
        return replace(self, **kw)


class QuadBraxEnv:
    def __init__(self, num_envs: int, env: str = "hover", episode_length: int = 500,
                 device=None, seed: int = 0, env_id_base: int = 0,
                 cfg_overrides: Optional[dict] = None):
        if env not in _KINDS:
            raise ValueError(f"unknown brax env {env!r}; expected one of {sorted(_KINDS)}")
        self.env_name = env
        self._env = QuadVecEnv(num_envs, env=_KINDS[env], device=device, seed=seed,
                               env_id_base=env_id_base, max_episode_steps=episode_length,
                               auto_reset=True, cfg_overrides=cfg_overrides)
        self.num_envs = self._env.num_envs
        self.device = self._env.device
        self.episode_length = int(episode_length)
        self._version = 0

    # brax Env properties (train_brax_ppo.py:232-242)
    @property
    def observation_size(self) -> int:
        return 21

    @property
    def action_size(self) -> int:
        return 4

    @property
    def backend(self) -> str:
        return "mjx"

    @property
    def unwrapped(self) -> QuadVecEnv:
        return self._env

    def _state(self, obs, reward, done, trunc, term) -> State:
        self._version += 1
        return State(pipeline_state={"q": obs[:, :11], "qd": obs[:, 11:]}, obs=obs, reward=reward,
                     done=done, metrics={"reward": reward},
                     info={"truncation": trunc, "terminated": term, "_version": self._version})

    def reset(self, rng: Optional[int] = None) -> State:
        """env.reset(rng) for every env: ``rng`` (an int) re-keys the reset draw like a new
        PRNG key; None keeps the current key and draws the next episode."""
        obs = self._env.reset(seed=rng).clone()
        z = torch.zeros(self.num_envs, device=self.device)
        return self._state(obs, z, z.clone(), z.clone(), z.clone())

    def step(self, state: State, action: torch.Tensor) -> State:
        if state.info.get("_version") != self._version:
            raise ValueError("QuadBraxEnv.step needs the State returned by the latest reset/step "
                             "(the batch state lives on the GPU, not in the State)")
        obs, rew, term, trunc, _ = self._env.step(action.to(torch.float32).contiguous(), info="raw")
        done = (term | trunc).float()
        truncation = (trunc & ~term).float()
        return self._state(obs.clone(), rew.clone(), done, truncation, term.float())

    def close(self) -> None:
        self._env.close()
