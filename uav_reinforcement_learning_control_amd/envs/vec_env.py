"""QuadVecEnv: N reference envs stepped by the gfx950 kernels, torch tensors in HBM.

Mirrors the reference's hot path and the vectorized interface its learners drive:
  * HoverEnv.reset / step                 envs/hover_env.py:200-238, :159-198
  * RateControlWrapper (wrapper="RateControlWrapper")       envs/rate_wrapper.py:26-111
  * TrajectoryFollowEnv (env="trajectory")                  envs/trajectory_follow_env.py:14-253
  * brax-compat kinds (env="brax_hover" QuadHoverBraxEnv, env="brax_jax_mjx" JaxMJXQuadBraxEnv,
    train_brax_ppo.py:39-368): 21-D raw obs; auto-reset restores the episode's first state
    (brax AutoResetWrapper); the functional brax API sits on top in envs/brax_env.py
  * SB3 VecEnv auto-reset (make_vec_env, train.py:48): on terminated|truncated the returned
    obs is the reset obs, info["terminal_observation"] the final one and
    info["TimeLimit.truncated"] = truncated & ~terminated.

All outputs stay on the GPU; no host synchronization happens inside step().  The work is
enqueued on torch's current stream of the env's device, so step() can be captured in a
torch.cuda.CUDAGraph.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from .. import _native as N
from ..utils.spaces import Box

_ENV_KINDS = {"hover": N.ENV_HOVER, "HoverEnv": N.ENV_HOVER,
              "trajectory": N.ENV_TRAJ, "TrajectoryFollowEnv": N.ENV_TRAJ,
              "brax_hover": N.ENV_BRAX_HOVER, "QuadHoverBraxEnv": N.ENV_BRAX_HOVER,
              "brax_jax_mjx": N.ENV_BRAX_TRAJ, "jax_mjx_quad": N.ENV_BRAX_TRAJ,
              "JaxMJXQuadBraxEnv": N.ENV_BRAX_TRAJ}
_WRAPPERS = {None: N.WRAP_NONE, "none": N.WRAP_NONE, "RateControlWrapper": N.WRAP_CTBR,
             "ctbr": N.WRAP_CTBR, "RelPosActWrapper": N.WRAP_RELPOS, "relpos": N.WRAP_RELPOS,
             # RelPosActWrapper(RateControlWrapper(env)), the stack the reference README documents
             "RelPosActWrapper(RateControlWrapper)": N.WRAP_CTBR_RELPOS, "ctbr_relpos": N.WRAP_CTBR_RELPOS}


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class QuadVecEnv:
    """Batched quadrotor env on one GPU (one process per GPU for multi-GPU)."""

    def __init__(self, num_envs: int, env: str = "hover", wrapper: Optional[str] = None,
                 device=None, seed: int = 0, env_id_base: int = 0,
                 max_episode_steps: Optional[int] = None, auto_reset: bool = True,
                 cfg_overrides: Optional[dict] = None):
        if not torch.cuda.is_available():
            raise N.QuadError("QuadVecEnv needs a ROCm GPU (the env runs only as HIP kernels)")
        if env not in _ENV_KINDS:
            raise ValueError(f"unknown env {env!r}; expected one of {sorted(_ENV_KINDS)}")
        if wrapper not in _WRAPPERS:
            raise ValueError(f"unknown wrapper {wrapper!r}")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.env_kind = env
        self.wrapper = wrapper if wrapper not in (None, "none") else None
        self.seed_value = int(seed)
        self.env_id_base = int(env_id_base)
        self.cfg_overrides = dict(cfg_overrides or {})  # kept so a wrapper can rebuild the same env
        L = N.lib()
        cfg = N.default_cfg(_ENV_KINDS[env], _WRAPPERS[wrapper])
        if max_episode_steps is not None:
            cfg.max_episode_steps = int(max_episode_steps)
        cfg.auto_reset = 1 if auto_reset else 0
        for k, v in (cfg_overrides or {}).items():
            cur = getattr(cfg, k)
            if isinstance(cur, (int, float)):
                setattr(cfg, k, v)
            else:
                for i, x in enumerate(v):
                    cur[i] = x
        self.cfg = cfg
        self.max_episode_steps = cfg.max_episode_steps
        self.dt = cfg.timestep
        h = C.c_void_p()
        N.check(L.quad_create(C.byref(cfg), self.device.index, self.seed_value, self.env_id_base,
                              self.num_envs, C.byref(h)), "quad_create")
        self._h = h
        self.action_space = Box(-1.0, 1.0, (4,), np.float32)
        self.brax = cfg.env_kind >= N.ENV_BRAX_HOVER
        self.obs_dim = 21 if self.brax else (7 if cfg.wrapper in (N.WRAP_RELPOS, N.WRAP_CTBR_RELPOS) else 12)
        self.observation_space = (Box(-np.inf, np.inf, (21,), np.float32) if self.brax
                                  else Box(-1.0, 1.0, (self.obs_dim,), np.float32))
        n, dev = self.num_envs, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs = torch.zeros(n, self.obs_dim, **f32)
        self.reward = torch.zeros(n, **f32)
        self.terminated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.truncated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.terminal_obs = torch.zeros(n, self.obs_dim, **f32)
        self.motor_commands = torch.zeros(n, 4, **f32)
        self.voltage_scale = torch.zeros(n, **f32)
        self.state12 = torch.zeros(n, 12, **f32)
        self.target_info = torch.zeros(n, 9, **f32)

    # ------------------------------------------------------------------------------------
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            N.lib().quad_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def unwrapped(self):
        return self

    # ------------------------------------------------------------------------------------
    def seed(self, seed: int) -> None:
        self.seed_value = int(seed)
        N.check(N.lib().quad_seed(self._h, self.seed_value, self._stream()), "quad_seed")

    def reset(self, seed: Optional[int] = None, mask: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """HoverEnv.reset for all envs (or those with mask != 0); returns obs [N,12] ([N,21] for
        the brax kinds)."""
        if seed is not None:
            self.seed(seed)
        out = self.obs if out is None else out
        self._check(out, (self.num_envs, self.obs_dim), torch.float32)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            self._check(m, (self.num_envs,), torch.uint8)
        N.check(N.lib().quad_reset(self._h, _ptr(m), _ptr(out), self._stream()), "quad_reset")
        return out

    def step(self, actions: torch.Tensor, obs: Optional[torch.Tensor] = None,
             reward: Optional[torch.Tensor] = None, info: str = "basic"):
        """One step of every env. Returns (obs, reward, terminated, truncated, info).

        actions: float32 [N,4] on the env's device (not clipped by the env, like HoverEnv).
        The returned tensors are the env's own buffers (overwritten by the next step) unless
        obs/reward are given. info="basic": terminal_observation + TimeLimit.truncated;
        info="full": also motor_commands, voltage_scale, state, target (+ target_vel / target_acc:
        TrajectoryFollowEnv's spline sample) -- HoverEnv's / TrajectoryFollowEnv's info dict;
        info="raw": terminal_observation only (no extra device op; for graph-captured loops).
        """
        self._check(actions, (self.num_envs, 4), torch.float32)
        obs = self.obs if obs is None else obs
        reward = self.reward if reward is None else reward
        self._check(obs, (self.num_envs, self.obs_dim), torch.float32)
        self._check(reward, (self.num_envs,), torch.float32)
        full = info == "full"
        o = N.QuadStepOut(
            obs=obs.data_ptr(), reward=reward.data_ptr(),
            terminated=self.terminated.data_ptr(), truncated=self.truncated.data_ptr(),
            terminal_obs=self.terminal_obs.data_ptr(),
            motor_commands=self.motor_commands.data_ptr() if full else None,
            voltage_scale=self.voltage_scale.data_ptr() if full else None,
            state12=self.state12.data_ptr() if full and not self.brax else None,
            target_info=self.target_info.data_ptr() if full else None)
        N.check(N.lib().quad_step(self._h, C.c_void_p(actions.data_ptr()), C.byref(o),
                                  self._stream()), "quad_step")
        inf = {"terminal_observation": self.terminal_obs}
        if info != "raw":
            inf["TimeLimit.truncated"] = self.truncated & ~self.terminated
        if full:
            inf.update(motor_commands=self.motor_commands, voltage_scale=self.voltage_scale,
                       state=self.state12, target=self.target_info[:, 0:3],
                       target_vel=self.target_info[:, 3:6], target_acc=self.target_info[:, 6:9])
        return obs, reward, self.terminated, self.truncated, inf

    def observe(self, out: Optional[torch.Tensor] = None, state: bool = False):
        """HoverEnv._get_obs of the current state; with state=True also the absolute 12-D
        QuadState vector (returns (obs, state12))."""
        out = self.obs if out is None else out
        self._check(out, (self.num_envs, self.obs_dim), torch.float32)
        if state and self.brax:
            raise ValueError("state=True: the brax kinds have no QuadState (obs is the raw state)")
        N.check(N.lib().quad_observe(self._h, _ptr(out), _ptr(self.state12) if state else None,
                                     self._stream()), "quad_observe")
        return (out, self.state12) if state else out

    def is_terminated(self, state12: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """HoverEnv._is_terminated (hover_env.py:150-157) for given absolute 12-D states [M,12]
        (float32 on this env's GPU): the step kernels' own predicate with this env's bounds."""
        if self.brax:
            raise ValueError("the brax kinds have no QuadState bounds")
        m = int(state12.shape[0])
        self._check(state12, (m, 12), torch.float32)
        out = torch.empty(m, dtype=torch.bool, device=self.device) if out is None else out
        self._check(out, (m,), torch.bool)
        N.check(N.lib().quad_terminated(self._h, _ptr(state12), m, _ptr(out), self._stream()),
                "quad_terminated")
        return out

    def step_random(self, steps: int, step0: int = 0, terminal_obs: bool = True, actions: bool = False) -> dict:
        """`steps` consecutive steps with action_space.sample()-style actions (the map of
        random_actions(step0 + s)) in ONE launch (quad_step_random, SURVEY config 2): returns
        time-major tensors obs [steps, N, 12], reward, terminated, truncated [steps, N], and
        terminal_observation [steps, N, 12] (rows of envs that finished) / actions [steps, N, 4]
        when asked. Identical to calling random_actions + step `steps` times."""
        if self.brax or self.obs_dim != 12:
            raise ValueError("step_random drives the hover / trajectory kinds (12-D obs)")
        n, dev, T = self.num_envs, self.device, int(steps)
        res = {"obs": torch.empty(T, n, 12, dtype=torch.float32, device=dev),
               "reward": torch.empty(T, n, dtype=torch.float32, device=dev),
               "terminated": torch.empty(T, n, dtype=torch.bool, device=dev),
               "truncated": torch.empty(T, n, dtype=torch.bool, device=dev)}
        if terminal_obs:
            res["terminal_observation"] = torch.zeros(T, n, 12, dtype=torch.float32, device=dev)
        if actions:
            res["actions"] = torch.empty(T, n, 4, dtype=torch.float32, device=dev)
        out = N.QuadStepOut(obs=res["obs"].data_ptr(), reward=res["reward"].data_ptr(),
                            terminated=res["terminated"].data_ptr(), truncated=res["truncated"].data_ptr(),
                            terminal_obs=_ptr(res.get("terminal_observation")))
        N.check(N.lib().quad_step_random(self._h, int(step0) & 0xFFFFFFFF, T, C.byref(out),
                                         _ptr(res.get("actions")), self._stream()), "quad_step_random")
        return res

    def random_actions(self, step_index: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """action_space.sample() for every env (Philox(seed, env id, step_index))."""
        out = torch.empty(self.num_envs, 4, dtype=torch.float32, device=self.device) \
            if out is None else out
        self._check(out, (self.num_envs, 4), torch.float32)
        N.check(N.lib().quad_random_actions(self._h, int(step_index) & 0xFFFFFFFF, _ptr(out),
                                            self._stream()), "quad_random_actions")
        return out

    # ------------------------------------------------------------------------------------
    _FIELDS = (("qpos", 11, np.float32), ("qvel", 10, np.float32), ("voltage", 1, np.float32),
               ("target", 3, np.float32), ("rate_int", 3, np.float32),
               ("step_count", 1, np.int32), ("episode", 1, np.uint32),
               ("prev_action", 4, np.float32))

    def get_state(self) -> dict:
        """Env state as host numpy arrays, env-major ([N, fields])."""
        n = self.num_envs
        arrs = {k: np.zeros((f, n), dt) for k, f, dt in self._FIELDS}
        soa = N.QuadStateSoA(**{k: a.ctypes.data for k, a in arrs.items()})
        N.check(N.lib().quad_get_state(self._h, C.byref(soa), 1, self._stream()), "quad_get_state")
        return {k: (a[0] if a.shape[0] == 1 else a.T.copy()) for k, a in arrs.items()}

    def set_state(self, **fields) -> None:
        """Overwrite (some of) qpos [N,11], qvel [N,10], voltage [N], target [N,3],
        rate_int [N,3], step_count [N], episode [N], prev_action [N,4] (HoverEnv.set_state
        analogue)."""
        keep = []
        kw = {}
        for k, f, dt in self._FIELDS:
            if k not in fields:
                continue
            a = np.asarray(fields[k], dtype=dt)
            a = a.reshape(self.num_envs, f) if f > 1 else a.reshape(1, self.num_envs)
            a = np.ascontiguousarray(a.T if f > 1 else a)
            keep.append(a)
            kw[k] = a.ctypes.data
        soa = N.QuadStateSoA(**kw)
        N.check(N.lib().quad_set_state(self._h, C.byref(soa), 1, self._stream()), "quad_set_state")
        del keep

    # ------------------------------------------------------------------------------------
    def _check(self, t: torch.Tensor, shape, dtype):
        if t.device != self.device or t.dtype != dtype or tuple(t.shape) != tuple(shape) \
                or not t.is_contiguous():
            raise ValueError(f"expected a contiguous {dtype} tensor of shape {shape} on "
                             f"{self.device}, got {t.dtype} {tuple(t.shape)} on {t.device}")
