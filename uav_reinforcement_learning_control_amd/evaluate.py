"""Batched GPU evaluation of a deterministic policy.

The reference evaluates one env at a time in Python loops (evaluate.py): ``evaluate`` runs
``num_episodes`` episodes from random resets (:296-437) and ``evaluate_trajectory`` follows a
waypoint lap (:440-612). Here N evaluations run at once on the GPU:

  * ``evaluate_episodes``  -- N episodes in parallel (HoverEnv resets, no auto-reset), each to
    termination or truncation; per-episode return and length (the reference's summary).
  * ``evaluate_waypoints`` -- N waypoint laps in parallel (one waypoint set per env, e.g. the
    eight / circle / square generators at several spacings); the bookkeeping -- reward sum, step
    count, waypoint switching within ``reach_radius``, lap completion, target update -- is the
    ``quad_waypoints_update`` kernel after each step.

Actions are ``model.predict(obs, deterministic=True)``: the Gaussian mean clipped to the action
box (SB3 clips Box actions in predict), computed by the MFMA policy kernel for 12-D obs and by the
torch policy otherwise (RelPosActWrapper's 7-D obs). The model is an SB3 archive (the reference's
``hover_policy_final.zip`` or one written by ``export.save_sb3_zip``), a ``policy.pt`` state dict or
an ``ActorCritic``; with an archive the wrapper is read from the sibling ``config.json`` like
evaluate.py:314-321.

    python -m uav_reinforcement_learning_control_amd.evaluate --model models_trained/<run>/hover_policy_final.zip \\
        --trajectory eight circle square --spacing 0.25 0.5 --max-steps 5000
"""
from __future__ import annotations

import argparse
import copy
import ctypes as C
import json
import os
from typing import Optional, Sequence, Union

import numpy as np
import torch

from . import _native as N
from .envs import QuadVecEnv
from .ppo.policy import ActorCritic
from .utils.trajectories import make_trajectory


def load_policy(model: Union[str, ActorCritic], device) -> tuple:
    """(ActorCritic on device, wrapper name or None from config.json)."""
    wrapper = None
    if isinstance(model, ActorCritic):  # a copy: the caller's module stays where it is
        return copy.deepcopy(model).to(device), wrapper
    path = str(model)
    cfg_path = os.path.join(os.path.dirname(os.path.abspath(path)), "config.json")
    if os.path.exists(cfg_path):
        w = json.load(open(cfg_path)).get("wrapper", "none")
        wrapper = None if w in (None, "none") else w
    if path.endswith(".zip"):
        from .export import load_sb3_policy
        return load_sb3_policy(path, device), wrapper
    sd = torch.load(path, map_location="cpu", weights_only=True)
    obs_dim = sd["mlp_extractor.policy_net.0.weight"].shape[1]
    pol = ActorCritic(obs_dim, sd["action_net.weight"].shape[0])
    pol.load_state_dict(sd)
    return pol.to(device), wrapper


class _Actor:
    """Deterministic actions into a fixed [N,4] buffer."""

    def __init__(self, policy: ActorCritic, n: int, device):
        self.policy = policy
        self.out = torch.zeros(n, 4, device=device)
        self.fp = None
        ex = policy.mlp_extractor
        if ex.policy_net[0].in_features == 12 and ex.policy_net[0].out_features == 128 \
                and ex.policy_net[2].out_features == 128:
            from .ppo.fused import FusedPolicy
            self.fp = FusedPolicy(policy)
            self.fp.pack()

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor) -> torch.Tensor:
        if self.fp is not None:
            self.fp.act(obs, self.out, deterministic=True)
        else:
            mean, _ = self.policy.forward_heads(obs)
            torch.clamp(mean, -1.0, 1.0, out=self.out)
        return self.out


def _waypoint_sets(trajectories, spacings) -> list:
    sets = []
    for t in trajectories:
        if isinstance(t, str):
            for sp in spacings:
                sets.append((f"{t}@{sp}", make_trajectory(t, spacing=sp)))
        else:
            sets.append((f"custom{len(sets)}", np.asarray(t, np.float64)))
    return sets


@torch.no_grad()
def evaluate_waypoints(model, trajectories: Sequence = ("eight",), spacings: Sequence[float] = (0.5,),
                       reach_radius: float = 0.25, max_steps: int = 5000, replicas: int = 1,
                       wrapper: Optional[str] = "auto", env: str = "hover", device="cuda",
                       seed: int = 0, record: bool = False) -> dict:
    """One lap per (waypoint set x replica) env, all at once. Returns per-env numpy arrays
    (name, steps, reached, laps, status, total_reward; with record=True also positions /
    actions / rewards [T, N, ...]) -- status 1 = lap completed, 2 = terminated, 3 = max steps."""
    device = torch.device(device)
    policy, cfg_wrapper = load_policy(model, device)
    wrapper = cfg_wrapper if wrapper == "auto" else wrapper
    sets = _waypoint_sets(trajectories, spacings)
    n = len(sets) * replicas
    maxp = max(len(p) for _, p in sets)
    pts = np.zeros((len(sets), maxp, 3), np.float64)
    for k, (_, p) in enumerate(sets):
        pts[k, :len(p)] = p
    points = torch.from_numpy(pts).to(device)
    counts = torch.tensor([len(p) for _, p in sets], dtype=torch.int32, device=device)
    set_of = (torch.arange(n, device=device, dtype=torch.int32) % len(sets)).contiguous()
    w = N.QuadWaypoints(points=points.data_ptr(), counts=counts.data_ptr(), set_of=set_of.data_ptr(),
                        max_points=maxp, reach_radius=float(reach_radius))
    trk = {k: torch.zeros(n, dtype=torch.int32, device=device) for k in ("wp_idx", "reached", "laps", "steps", "status")}
    trk["total_reward"] = torch.zeros(n, dtype=torch.float64, device=device)
    st = N.QuadWaypointState(**{k: v.data_ptr() for k, v in trk.items()})
    e = QuadVecEnv(n, env=env, wrapper=wrapper, device=device, seed=seed,
                   max_episode_steps=max_steps, auto_reset=False)
    e.reset()
    obs = torch.zeros(n, e.obs_dim, device=device)
    L = N.lib()
    N.check(L.quad_waypoints_begin(e._h, C.byref(w), C.byref(st), C.c_void_p(obs.data_ptr()), e._stream()),
            "quad_waypoints_begin")
    act = _Actor(policy, n, device)
    rec = {"positions": [], "actions": [], "rewards": []} if record else None
    for t in range(max_steps):
        a = act(obs)
        _, rew, te, tr, info = e.step(a, obs=obs, info="full")
        if rec is not None:
            rec["positions"].append(info["state"][:, :3].clone())
            rec["actions"].append(a.clone())
            rec["rewards"].append(rew.clone())
        N.check(L.quad_waypoints_update(e._h, C.byref(w), C.byref(st), C.c_void_p(info["state"].data_ptr()),
                                        C.c_void_p(rew.data_ptr()), C.c_void_p(te.data_ptr()),
                                        C.c_void_p(tr.data_ptr()), e._stream()), "quad_waypoints_update")
        if (t + 1) % 128 == 0 and bool((trk["status"] != 0).all()):
            break
    torch.cuda.synchronize(device)
    out = {k: v.cpu().numpy() for k, v in trk.items()}
    out["name"] = np.array([sets[i % len(sets)][0] for i in range(n)])
    out["n_waypoints"] = np.array([len(sets[i % len(sets)][1]) for i in range(n)])
    if rec is not None:
        out["positions"] = torch.stack(rec["positions"]).cpu().numpy()
        out["actions"] = torch.stack(rec["actions"]).cpu().numpy()
        out["rewards"] = torch.stack(rec["rewards"]).cpu().numpy()
    e.close()
    return out


@torch.no_grad()
def evaluate_episodes(model, num_episodes: int = 1024, wrapper: Optional[str] = "auto", env: str = "hover",
                      max_episode_steps: Optional[int] = None, device="cuda", seed: int = 0) -> dict:
    """``num_episodes`` episodes at once from HoverEnv resets, deterministic policy, each run to
    termination or truncation (evaluate.py:296-437 without the viewer). Returns per-episode
    rewards / lengths / terminated flags and their mean / std."""
    device = torch.device(device)
    policy, cfg_wrapper = load_policy(model, device)
    wrapper = cfg_wrapper if wrapper == "auto" else wrapper
    e = QuadVecEnv(num_episodes, env=env, wrapper=wrapper, device=device, seed=seed,
                   max_episode_steps=max_episode_steps, auto_reset=False)
    obs = e.reset().clone()
    act = _Actor(policy, num_episodes, device)
    ret = torch.zeros(num_episodes, dtype=torch.float64, device=device)
    length = torch.zeros(num_episodes, dtype=torch.int32, device=device)
    running = torch.ones(num_episodes, dtype=torch.bool, device=device)
    terminated = torch.zeros(num_episodes, dtype=torch.bool, device=device)
    for t in range(e.max_episode_steps):
        a = act(obs)
        _, rew, te, tr, _ = e.step(a, obs=obs, info="raw")
        ret += torch.where(running, rew.double(), 0.0)
        length += running.int()
        terminated |= running & te
        running &= ~(te | tr)
        if (t + 1) % 64 == 0 and not bool(running.any()):
            break
    r, l = ret.cpu().numpy(), length.cpu().numpy()
    e.close()
    return {"rewards": r, "lengths": l, "terminated": terminated.cpu().numpy(),
            "mean_reward": float(r.mean()), "std_reward": float(r.std()),
            "mean_length": float(l.mean()), "std_length": float(l.std())}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--model", required=True)
    ap.add_argument("--mode", choices=["episodes", "trajectory"], default="trajectory")
    ap.add_argument("--trajectory", nargs="+", default=["eight"], choices=["eight", "circle", "square"])
    ap.add_argument("--spacing", nargs="+", type=float, default=[0.5])
    ap.add_argument("--reach-radius", type=float, default=0.25)
    ap.add_argument("--max-steps", type=int, default=5000)
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--num-episodes", type=int, default=1024)
    a = ap.parse_args(argv)
    if a.mode == "episodes":
        r = evaluate_episodes(a.model, a.num_episodes)
        print(f"Episodes: {a.num_episodes}\nMean reward: {r['mean_reward']:.2f} +/- {r['std_reward']:.2f}\n"
              f"Mean length: {r['mean_length']:.1f} +/- {r['std_length']:.1f}")
        return r
    r = evaluate_waypoints(a.model, a.trajectory, a.spacing, a.reach_radius, a.max_steps, a.replicas)
    status = {0: "running", 1: "lap", 2: "terminated", 3: "max steps"}
    for i in range(len(r["name"])):
        print(f"{r['name'][i]:>12}: steps {r['steps'][i]:5d}  waypoints {r['reached'][i]:3d}/"
              f"{r['n_waypoints'][i]:3d}  laps {r['laps'][i]}  reward {r['total_reward'][i]:9.2f}  "
              f"{status[int(r['status'][i])]}")
    return r


if __name__ == "__main__":
    main()
