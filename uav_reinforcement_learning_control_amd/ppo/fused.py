"""The rollout policy as MFMA kernels (csrc/policy.hip via quad_policy_pack / quad_policy_act /
quad_rollout_post), bound to a torch ActorCritic.

One rollout step of SB3 OnPolicyAlgorithm.collect_rollouts (the learner the reference's
train.py:50-68 configures) becomes three launches -- policy (both MLPs on MFMA, Gaussian sample,
log-prob, clip, buffer rows), env step, epilogue (TimeLimit bootstrap, episode_starts, Monitor
statistics) -- instead of ~25 torch kernels. The torch ActorCritic stays the trained model;
`pack()` refreshes the kernels' copy of its parameters (call it after each update).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from .. import _native as N
from .policy import ActorCritic


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _need(t: torch.Tensor, shape, dtype, dev, name):
    if t.dtype != dtype or tuple(t.shape) != tuple(shape) or not t.is_contiguous() or t.device != dev:
        raise ValueError(f"{name}: expected contiguous {dtype} {tuple(shape)} on {dev}, got "
                         f"{t.dtype} {tuple(t.shape)} on {t.device}")


class FusedPolicy:
    """Packed fp32 image of an ActorCritic (12 -> 128 -> 128 -> 4 / 1) for the MFMA kernels."""

    @staticmethod
    def _check_shapes(policy: ActorCritic) -> None:
        ex = policy.mlp_extractor
        shapes = [tuple(l.weight.shape) for l in (ex.policy_net[0], ex.policy_net[2], ex.value_net[0],
                                                  ex.value_net[2], policy.action_net, policy.value_net)]
        if shapes != [(128, 12), (128, 128), (128, 12), (128, 128), (4, 128), (1, 128)]:
            raise ValueError(f"the MFMA policy kernels are built for 12-128-128-(4|1) nets, got {shapes}")

    def __init__(self, policy: ActorCritic):
        self._check_shapes(policy)
        self.policy = policy
        self.device = policy.log_std.device
        if self.device.type != "cuda":
            raise N.QuadError("FusedPolicy needs the policy on a ROCm GPU")
        L = N.lib()
        self.packed = torch.empty(L.quad_policy_packed_floats(), dtype=torch.float32, device=self.device)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @torch.no_grad()
    def pack(self) -> None:
        pol, ex = self.policy, self.policy.mlp_extractor
        ts = [ex.policy_net[0].weight, ex.policy_net[0].bias, ex.policy_net[2].weight, ex.policy_net[2].bias,
              pol.action_net.weight, pol.action_net.bias,
              ex.value_net[0].weight, ex.value_net[0].bias, ex.value_net[2].weight, ex.value_net[2].bias,
              pol.value_net.weight, pol.value_net.bias, pol.log_std]
        for t in ts:
            if not t.is_contiguous() or t.dtype != torch.float32:
                raise ValueError("policy parameters must be contiguous float32")
        prm = N.QuadPolicyParams(*[t.data_ptr() for t in ts])
        N.check(N.lib().quad_policy_pack(C.byref(prm), _p(self.packed), self._stream()), "quad_policy_pack")

    def act(self, obs: torch.Tensor, actions_env: torch.Tensor, *, actions=None, log_prob=None,
            value=None, obs_copy=None, last_start=None, episode_starts=None,
            cursor: Optional[torch.Tensor] = None, rows: int = 1, seed: int = 0,
            env_id_base: int = 0, deterministic: bool = False,
            epilogue: Optional[N.QuadRolloutPost] = None) -> None:
        """quad_policy_act: row buffers are [rows, N, ...] (row t % rows, t = cursor[0]); with
        `epilogue` (from make_epilogue) the pending previous step is finished in the same launch
        and the cursor advances."""
        n, dev, f32 = obs.shape[0], self.device, torch.float32
        _need(obs, (n, 12), f32, dev, "obs")
        _need(actions_env, (n, 4), f32, dev, "actions_env")
        for t, shp, name in ((actions, (rows, n, 4), "actions"), (log_prob, (rows, n), "log_prob"),
                             (value, (rows, n), "value"), (obs_copy, (rows, n, 12), "obs_copy"),
                             (last_start, (n,), "last_start"), (episode_starts, (rows, n), "episode_starts")):
            if t is not None:
                _need(t, shp, f32, dev, name)
        if cursor is not None:
            _need(cursor, (4,), torch.int32, dev, "cursor")
        a = N.QuadPolicyAct(obs=obs.data_ptr(), actions_env=actions_env.data_ptr(),
                            actions=_p(actions), log_prob=_p(log_prob), value=_p(value),
                            obs_copy=_p(obs_copy), last_start=_p(last_start),
                            episode_starts=_p(episode_starts), cursor=_p(cursor), rows=int(rows),
                            deterministic=int(bool(deterministic)), seed=int(seed) & (2**64 - 1),
                            env_id_base=int(env_id_base),
                            epilogue=C.pointer(epilogue) if epilogue is not None else None)
        N.check(N.lib().quad_policy_act(_p(self.packed), C.byref(a), n, self._stream()), "quad_policy_act")

    def value(self, obs: torch.Tensor, out: torch.Tensor, scratch: torch.Tensor) -> torch.Tensor:
        """V(obs) [N] into out ([1, N]) on the MFMA kernel: per-row results do not depend on the
        batch (no GEMM tiling choice), so a rank's shard bootstraps exactly as in one process.
        `scratch` ([N, 4]) receives the deterministic actions."""
        self.act(obs, scratch, value=out, rows=1, deterministic=True)
        return out[0]

    def make_epilogue(self, reward, terminated, truncated, terminal_obs, buf_rew, last_start, ep_ret,
                      ep_len, stats, rows: int, gamma: float) -> N.QuadRolloutPost:
        """The QuadRolloutPost of a rollout (buffers are referenced, not copied: keep them alive)."""
        n, dev, f32 = reward.shape[0], self.device, torch.float32
        _need(reward, (n,), f32, dev, "reward")
        _need(terminated, (n,), torch.bool, dev, "terminated")
        _need(truncated, (n,), torch.bool, dev, "truncated")
        _need(terminal_obs, (n, 12), f32, dev, "terminal_obs")
        _need(buf_rew, (rows, n), f32, dev, "buf_rew")
        for t, name in ((last_start, "last_start"), (ep_ret, "ep_ret"), (ep_len, "ep_len")):
            _need(t, (n,), f32, dev, name)
        _need(stats, (N.POLICY_STAT_SLOTS, 3), torch.float64, dev, "stats")
        e = N.QuadRolloutPost(reward=reward.data_ptr(), terminated=terminated.data_ptr(),
                              truncated=truncated.data_ptr(), terminal_obs=terminal_obs.data_ptr(),
                              buf_rew=buf_rew.data_ptr(), last_start=last_start.data_ptr(),
                              ep_ret=ep_ret.data_ptr(), ep_len=ep_len.data_ptr(),
                              stats=stats.data_ptr(), rows=int(rows), gamma=float(gamma))
        e._n = n
        return e

    def post(self, epilogue: N.QuadRolloutPost, cursor: torch.Tensor) -> None:
        """quad_rollout_post: finish the pending step (end of a rollout)."""
        _need(cursor, (4,), torch.int32, self.device, "cursor")
        N.check(N.lib().quad_rollout_post(_p(self.packed), C.byref(epilogue), _p(cursor), epilogue._n,
                                          self._stream()), "quad_rollout_post")

    def rollout(self, env, *, obs_copy, actions, log_prob, value, episode_starts, rewards, last_obs,
                last_start, ep_ret, ep_len, stats, t0: int, steps: int, seed: int, gamma: float,
                deterministic: bool = False) -> None:
        """quad_rollout: `steps` whole rollout steps (policy + env step + bootstrap + statistics)
        of `env` (a QuadVecEnv: hover/trajectory, no wrapper or RateControlWrapper, auto-reset) in
        one launch; step t = t0 + s writes row t % rows of the [rows, N, ...] buffers."""
        n, dev, f32 = env.num_envs, self.device, torch.float32
        rows = rewards.shape[0]
        for t, shp, name in ((obs_copy, (rows, n, 12), "obs_copy"), (actions, (rows, n, 4), "actions"),
                             (log_prob, (rows, n), "log_prob"), (value, (rows, n), "value"),
                             (episode_starts, (rows, n), "episode_starts"), (rewards, (rows, n), "rewards"),
                             (last_obs, (n, 12), "last_obs"), (last_start, (n,), "last_start"),
                             (ep_ret, (n,), "ep_ret"), (ep_len, (n,), "ep_len")):
            _need(t, shp, f32, dev, name)
        _need(stats, (N.POLICY_STAT_SLOTS, 3), torch.float64, dev, "stats")
        r = N.QuadRollout(obs_copy=obs_copy.data_ptr(), actions=actions.data_ptr(),
                          log_prob=log_prob.data_ptr(), value=value.data_ptr(),
                          episode_starts=episode_starts.data_ptr(), rewards=rewards.data_ptr(),
                          last_obs=last_obs.data_ptr(), last_start=last_start.data_ptr(),
                          ep_ret=ep_ret.data_ptr(), ep_len=ep_len.data_ptr(), stats=stats.data_ptr(),
                          rows=int(rows), t0=int(t0), steps=int(steps),
                          deterministic=int(bool(deterministic)), seed=int(seed) & (2**64 - 1),
                          gamma=float(gamma))
        N.check(N.lib().quad_rollout(env._h, _p(self.packed), C.byref(r), self._stream()), "quad_rollout")


def rollout_supported(env) -> bool:
    """quad_rollout drives hover / trajectory envs (12-D obs) with SB3 auto-reset."""
    cfg = getattr(env, "cfg", None)
    return (cfg is not None and getattr(env, "_h", None) is not None and cfg.auto_reset == 1
            and cfg.env_kind in (N.ENV_HOVER, N.ENV_TRAJ) and cfg.wrapper in (N.WRAP_NONE, N.WRAP_CTBR))
