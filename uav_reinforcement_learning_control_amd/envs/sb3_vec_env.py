"""SB3 VecEnv-shaped facade over the batched GPU env.

The reference hands Stable-Baselines3's PPO a vectorized env built by
`make_vec_env(make_env, n_envs=16)` (reference train.py:48-50): a DummyVecEnv of Monitor-wrapped
HoverEnv / RateControlWrapper instances. What that object promises its caller (SB3 2.x
`stable_baselines3.common.vec_env.base_vec_env.VecEnv`, a third-party API restated here, absent
from this image):

  * reset() -> obs [N, obs_dim] (no info tuple; per-env reset infos in `reset_infos`);
  * step_async(actions) / step_wait() -> (obs, rewards [N], dones [N], infos: list of N dicts),
    step(actions) = both; done = terminated or truncated, the returned obs row of a done env is the
    reset observation, infos[i]["terminal_observation"] the final one and
    infos[i]["TimeLimit.truncated"] = truncated and not terminated (DummyVecEnv.step_wait);
    Monitor adds infos[i]["episode"] = {"r": return, "l": length, "t": seconds since start};
  * num_envs, observation_space, action_space, get_attr / set_attr / env_method /
    env_is_wrapped (with `indices`), seed(seed) -> per-env seeds, close(), render().

Here the N envs are ONE QuadVecEnv (one kernel launch per step, auto-reset fused in the kernel),
so the facade only converts: device tensors -> NumPy (the SB3 contract; `as_tensors=True` keeps
torch tensors on the GPU for GPU learners) and the batched info tensors -> per-env dicts. By default
the dicts carry only what SB3's PPO reads (the auto-reset and Monitor keys of the envs that
finished; {} for the others); `full_info=True` adds HoverEnv's own step info (state,
motor_commands, target, voltage_scale, ...) to every env's dict, as DummyVecEnv passes it through.
"""
from __future__ import annotations

import time
from typing import Any, Callable, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch

from .hover_env import HoverEnv
from .vec_env import QuadVecEnv

Indices = Union[None, int, Iterable[int]]


class QuadSB3VecEnv:
    """SB3 `VecEnv` API over a QuadVecEnv (one GPU, SB3 auto-reset semantics)."""

    metadata = {"render_modes": []}
    render_mode = None

    def __init__(self, env: QuadVecEnv, as_tensors: bool = False, full_info: bool = False):
        if not isinstance(env, QuadVecEnv):
            raise TypeError("QuadSB3VecEnv wraps a QuadVecEnv")
        if not env.cfg.auto_reset:
            raise ValueError("SB3 VecEnvs auto-reset: build the QuadVecEnv with auto_reset=True")
        self.venv = env
        self.num_envs = env.num_envs
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self.as_tensors = bool(as_tensors)
        self.full_info = bool(full_info)
        self.reset_infos: List[dict] = [{} for _ in range(self.num_envs)]
        self._actions: Optional[torch.Tensor] = None
        self._ep_ret = torch.zeros(self.num_envs, dtype=torch.float64, device=env.device)
        self._ep_len = torch.zeros(self.num_envs, dtype=torch.int64, device=env.device)
        self._t_start = time.time()  # Monitor.__init__ sets t_start once; reset() keeps it
        self._seeds: List[Optional[int]] = [None] * self.num_envs
        self.closed = False

    # ---- VecEnv core ---------------------------------------------------------------------
    def _out(self, t: torch.Tensor):
        return t.clone() if self.as_tensors else t.cpu().numpy().copy()

    def reset(self):
        """VecEnv.reset: every env restarts (pending seed() applied first); returns obs [N, obs_dim]."""
        seed = self._seeds[0]
        obs = self.venv.reset(seed=seed)
        self._seeds = [None] * self.num_envs
        self._ep_ret.zero_()
        self._ep_len.zero_()
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return self._out(obs)

    def step_async(self, actions) -> None:
        a = torch.as_tensor(np.asarray(actions, np.float32) if not torch.is_tensor(actions) else actions)
        a = a.to(device=self.venv.device, dtype=torch.float32).reshape(self.num_envs, 4).contiguous()
        self._actions = a

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        a, self._actions = self._actions, None
        obs, rew, te, tr, inf = self.venv.step(a, info="full" if self.full_info else "basic")
        done = te | tr
        # Monitor: the episode statistics of the envs that finished this step
        self._ep_ret += rew.double()
        self._ep_len += 1
        ret_done, len_done = self._ep_ret[done], self._ep_len[done]
        self._ep_ret.masked_fill_(done, 0.0)
        self._ep_len.masked_fill_(done, 0)
        d_idx = torch.nonzero(done).flatten()
        tobs = inf["terminal_observation"][d_idx]
        tl = inf["TimeLimit.truncated"][d_idx]
        # one host transfer of the per-step outputs the dicts need
        d_np = d_idx.cpu().numpy()
        tobs_h = tobs if self.as_tensors else tobs.cpu().numpy()
        tl_h, r_h, l_h = tl.cpu().numpy(), ret_done.cpu().numpy(), len_done.cpu().numpy()
        infos: List[dict] = [{} for _ in range(self.num_envs)]
        elapsed = round(time.time() - self._t_start, 6)
        for k, i in enumerate(d_np.tolist()):
            infos[i] = {"TimeLimit.truncated": bool(tl_h[k]), "terminal_observation": tobs_h[k],
                        "episode": {"r": round(float(r_h[k]), 6), "l": int(l_h[k]), "t": elapsed}}
        if self.full_info:  # HoverEnv's own info keys for every env (rows of the batched tensors)
            extra = {k: v.cpu().numpy() for k, v in inf.items()
                     if k not in ("terminal_observation", "TimeLimit.truncated")}
            for i in range(self.num_envs):
                for k, v in extra.items():
                    infos[i][k] = v[i]
        return self._out(obs), self._out(rew), self._out(done), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        if not self.closed:
            self.venv.close()
            self.closed = True

    def render(self, mode: Optional[str] = None):
        return None  # the reference HoverEnv.render returns None as well

    def get_images(self) -> Sequence[Optional[np.ndarray]]:
        return [None] * self.num_envs

    # ---- per-env attribute / method access ------------------------------------------------
    def _indices(self, indices: Indices) -> List[int]:
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    def get_attr(self, attr_name: str, indices: Indices = None) -> List[Any]:
        """The attribute of each selected env. All N envs share one configuration (the batched
        env's), so every entry is the batched env's attribute, except `np_random`-free per-env
        state, which is not exposed."""
        v = getattr(self.venv, attr_name)
        return [v for _ in self._indices(indices)]

    def set_attr(self, attr_name: str, value: Any, indices: Indices = None) -> None:
        idx = self._indices(indices)
        if len(idx) != self.num_envs:
            raise ValueError("the batched env has one configuration: set_attr applies to all envs")
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name: str, *method_args, indices: Indices = None, **method_kwargs) -> List[Any]:
        """Call a method of the batched env once and hand its result to each selected env; a
        per-env result ([N, ...] array / tensor) is split by rows."""
        idx = self._indices(indices)
        res = getattr(self.venv, method_name)(*method_args, **method_kwargs)
        if (torch.is_tensor(res) or isinstance(res, np.ndarray)) and res.ndim >= 1 and res.shape[0] == self.num_envs:
            return [res[i] for i in idx]
        return [res for _ in idx]

    def env_is_wrapped(self, wrapper_class, indices: Indices = None) -> List[bool]:
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        kind = self.venv.wrapper or "none"
        wrapped = {"RateControlWrapper": kind in ("RateControlWrapper", "ctbr", "ctbr_relpos",
                                                  "RelPosActWrapper(RateControlWrapper)"),
                   "RelPosActWrapper": kind in ("RelPosActWrapper", "relpos", "ctbr_relpos",
                                                "RelPosActWrapper(RateControlWrapper)"),
                   "Monitor": True}.get(name, False)
        return [wrapped for _ in self._indices(indices)]

    def seed(self, seed: Optional[int] = None) -> List[Optional[int]]:
        """VecEnv.seed: the seed takes effect at the next reset(); env i gets seed + i in SB3's
        numbering (here: one Philox key for the batch, the env id keys each env's stream)."""
        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1))
        self._seeds = [seed + i for i in range(self.num_envs)]
        return list(self._seeds)

    @property
    def unwrapped(self):
        return self

    def __len__(self) -> int:
        return self.num_envs


def _facade_spec(env):
    """(env kind, kernel wrapper kind, max_episode_steps, cfg overrides) of a HoverEnv /
    TrajectoryFollowEnv facade, bare or under RateControlWrapper / RelPosActWrapper."""
    base = getattr(env, "unwrapped", env)
    if not isinstance(base, HoverEnv):
        raise TypeError(f"make_vec_env: the env factory must build a HoverEnv / TrajectoryFollowEnv facade, "
                        f"got {type(base).__name__}")
    vec = base._vec
    return vec.env_kind, vec.wrapper, vec.max_episode_steps, dict(vec.cfg_overrides), vec.device


def make_vec_env(env_id: Union[str, Callable[[], Any]], n_envs: int = 1, seed: Optional[int] = None,
                 start_index: int = 0, env_kwargs: Optional[dict] = None, device=None,
                 as_tensors: bool = False, **_ignored) -> QuadSB3VecEnv:
    """stable_baselines3.common.env_util.make_vec_env as reference train.py:48 calls it: `env_id` is
    the script's make_env (a callable building HoverEnv() optionally wrapped) or an env name
    ("HoverEnv", "TrajectoryFollowEnv"); the n_envs copies become ONE batched GPU env with the same
    kind, wrapper, episode length and overrides. `start_index` offsets the global env ids (so
    ranks/processes draw disjoint streams)."""
    if callable(env_id):
        proto = env_id(**(env_kwargs or {}))
        kind, wrapper, max_steps, overrides, dev = _facade_spec(proto)
        proto.close()
    else:
        kind, wrapper, max_steps, overrides, dev = env_id, None, None, dict(env_kwargs or {}), None
    venv = QuadVecEnv(int(n_envs), env=kind, wrapper=wrapper, device=device if device is not None else dev,
                      seed=0 if seed is None else int(seed), env_id_base=int(start_index),
                      max_episode_steps=max_steps, auto_reset=True, cfg_overrides=overrides or None)
    return QuadSB3VecEnv(venv, as_tensors=as_tensors)
