#!/usr/bin/env python3
"""Generate golden vectors from the reference's own env code.

RUN ONLY WHERE /root/reference EXISTS (this build container).  The reference never travels to the
GPU box; only the .npz fixtures written to tests/golden/ are committed and shipped.

What is pinned: everything in HoverEnv / RateControlWrapper / TrajectoryFollowEnv / QuadState /
normalize / denormalize (reference code, executed unmodified), with gymnasium and mujoco replaced
by the stubs in tools/refstubs (see its README).  The physics inside mj_step is the CPU oracle's
restatement of MuJoCo (oracle/quad_oracle.c), so these fixtures pin the env semantics and the
oracle's env layer, not MuJoCo itself ("parity unpinned" for the physics).

Usage:  python tools/gen_golden.py  [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _setup():
    if not os.path.isdir(REF):
        raise SystemExit("gen_golden.py needs /root/reference (build container only)")
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REPO, "tools", "refstubs"))
    sys.path.insert(0, REPO)
    import mujoco  # the stub

    from oracle import oracle as O

    opt = O.default_opt()

    def step_fn(qpos, qvel, ctrl):
        qp, qv, ct, _ = O.mj_step(qpos, qvel, ctrl, opt)
        qpos[:] = qp
        qvel[:] = qv
        ctrl[:] = ct

    mujoco.STEP_FN = step_fn


def _draws_from(rng_state, n_state=12, low=None, high=None, tlow=None, thigh=None):
    g = np.random.default_rng()
    g.bit_generator.state = rng_state
    init12 = g.uniform(low, high).astype(np.float32)
    target = g.uniform(tlow, thigh).astype(np.float32)
    return init12, target


def euler_fixture():
    from utils.state import QuadState

    rng = np.random.default_rng(1234)
    quats = [rng.normal(size=4) for _ in range(300)]
    quats = [q / np.linalg.norm(q) for q in quats]
    quats += [np.array([1.0, 0, 0, 0]), np.array([0.0, 1, 0, 0]), np.array([0.0, 0, 1, 0]),
              np.array([0.0, 0, 0, 1])]
    for p in [np.pi / 2, -np.pi / 2, np.pi / 2 - 1e-4, -np.pi / 2 + 1e-4, np.pi / 2 - 3e-3,
              np.pi / 2 - 1e-9]:
        for y in [0.0, 0.7, -2.5]:
            cr, sr, cp, sp = np.cos(0.3 / 2), np.sin(0.3 / 2), np.cos(p / 2), np.sin(p / 2)
            cy, sy = np.cos(y / 2), np.sin(y / 2)
            quats.append(np.array([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                                   cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy]))
    quats += [rng.normal(size=4) * 1.7 for _ in range(20)]  # non-unit (scipy normalizes)
    quats = np.array(quats)
    states = []
    for q in quats:
        s = QuadState()
        qpos = np.concatenate([[0.1, -0.2, 0.3], q])
        s.set_from_mujoco(qpos, np.arange(6, dtype=np.float64) * 0.1)
        states.append(s.vec())
    eul = rng.uniform(-np.pi, np.pi, size=(200, 3)).astype(np.float32)
    qposs = []
    for e in eul:
        s = QuadState()
        s.state[3:6] = e
        qp, _ = s.get_mujoco_state()
        qposs.append(qp)
    return dict(quat_wxyz=quats, state12=np.array(states, np.float32), euler_in=eul,
                qpos_from_euler=np.array(qposs))


def termination_fixture():
    from envs.hover_env import HoverEnv
    from envs.trajectory_follow_env import TrajectoryFollowEnv

    out = {}
    for name, env in (("hover", HoverEnv()), ("traj", TrajectoryFollowEnv())):
        lo, hi = env._state_bounds.low, env._state_bounds.high
        rng = np.random.default_rng(7)
        S = []
        for _ in range(200):
            S.append(rng.uniform(lo * 1.1, hi * 1.1).astype(np.float32))
        for i in range(12):
            for v in (lo[i], hi[i], np.nextafter(lo[i], np.float32(-np.inf)),
                      np.nextafter(hi[i], np.float32(np.inf)), np.nextafter(lo[i], np.float32(0)),
                      np.nextafter(hi[i], np.float32(0))):
                s = np.zeros(12, np.float32)
                s[2] = 1.0
                s[i] = v
                S.append(s)
            for v in (np.nan, np.inf, -np.inf):
                s = np.zeros(12, np.float32)
                s[2] = 1.0
                s[i] = v
                S.append(s)
        S = np.array(S, np.float32)
        T = []
        for s in S:
            env._state.state = s.copy()
            T.append(env._is_terminated())
        out[f"{name}_states"] = S
        out[f"{name}_terminated"] = np.array(T, np.bool_)
    return out


def rollout_fixture(kind: str, wrapper, n_steps: int, seeds, max_episode_steps=None,
                    action_mode="mixed"):
    """wrapper: False/None, True (RateControlWrapper), "relpos" (RelPosActWrapper: the recorded
    obs / reset_obs are then the wrapper's 7-D observations, plus pre_prev_action) or "ctbr_relpos"
    (RelPosActWrapper(RateControlWrapper(env)), the stack the reference README documents)."""
    from envs.hover_env import HoverEnv
    from envs.rate_wrapper import RateControlWrapper
    from envs.trajectory_follow_env import TrajectoryFollowEnv
    from envs.wrappers import RelPosActWrapper

    kw = {} if max_episode_steps is None else dict(max_episode_steps=max_episode_steps)
    base = HoverEnv(**kw) if kind == "hover" else TrajectoryFollowEnv(**kw)
    relpos = wrapper in ("relpos", "ctbr_relpos")
    if wrapper == "ctbr_relpos":
        ctbr_env = RateControlWrapper(base)
        env = RelPosActWrapper(ctbr_env)
    else:
        env = RelPosActWrapper(base) if relpos else RateControlWrapper(base) if wrapper else base
        ctbr_env = env
    wrapper = bool(wrapper) and wrapper != "relpos"  # the CTBR integrator fields below
    u = env.unwrapped
    arng = np.random.default_rng(99)
    rec = {k: [] for k in ("pre_qpos", "pre_qvel", "pre_voltage", "pre_target", "pre_step",
                           "pre_state12", "pre_rate_int", "action", "obs", "reward", "terminated",
                           "truncated", "motor", "voltage", "vscale", "post_qpos", "post_qvel",
                           "post_state12", "post_rate_int", "info_state", "pre_prev_action")}
    resets = {k: [] for k in ("init12", "target3", "obs", "qpos", "qvel", "state12")}

    def do_reset(seed):
        st = u.np_random.bit_generator.state if seed is None else None
        obs, info = env.reset(seed=seed)
        if seed is not None:
            g = np.random.default_rng(seed)
        else:
            g = np.random.default_rng()
            g.bit_generator.state = st
        init12 = g.uniform(u._initial_state_bounds.low, u._initial_state_bounds.high).astype(np.float32)
        if kind == "hover":
            target = g.uniform(u._target_pos_bounds.low, u._target_pos_bounds.high).astype(np.float32)
            assert np.array_equal(target, u.target_state.position)
        else:
            target = u.target_state.position.copy()
            assert np.array_equal(target, init12[:3])
        resets["init12"].append(init12)
        resets["target3"].append(target)
        resets["obs"].append(obs)
        resets["qpos"].append(u.data.qpos.copy())
        resets["qvel"].append(u.data.qvel.copy())
        resets["state12"].append(u._state.vec())

    seeds = list(seeds)
    do_reset(seeds.pop(0))
    for t in range(n_steps):
        if action_mode == "mixed":
            m = t % 5
            if m == 0:
                a = arng.uniform(-1, 1, 4)
            elif m == 1:
                a = arng.uniform(-1.6, 1.6, 4)  # policies' raw Gaussians exceed the box
            elif m == 2:
                a = np.array([-0.91, 0.0, 0.0, 0.0]) + arng.normal(0, 0.05, 4)  # near hover
            elif m == 3:
                a = arng.choice([-1.0, 0.0, 1.0], 4)
            else:
                a = arng.uniform(-0.3, 0.3, 4)
        elif action_mode == "nan":
            a = arng.uniform(-1, 1, 4)
            if t % 7 == 3:
                a[t % 4] = np.nan
        else:
            a = arng.uniform(-1, 1, 4)
        a = a.astype(np.float32)
        rec["pre_qpos"].append(u.data.qpos.copy())
        rec["pre_qvel"].append(u.data.qvel.copy())
        rec["pre_voltage"].append(u.voltage)
        rec["pre_target"].append(u.target_state.position.copy())
        rec["pre_step"].append(u._step_count)
        rec["pre_state12"].append(u._state.vec())
        rec["pre_rate_int"].append(ctbr_env._rate_int_torque.copy() if wrapper else np.zeros(3))
        rec["pre_prev_action"].append(u._prev_action.copy())
        rec["action"].append(a)
        obs, r, te, tr, info = env.step(a)
        rec["obs"].append(obs)
        rec["reward"].append(float(r))
        rec["terminated"].append(bool(te))
        rec["truncated"].append(bool(tr))
        rec["motor"].append(info["motor_commands"])
        rec["voltage"].append(info["voltage"])
        rec["vscale"].append(info["voltage_scale"])
        rec["info_state"].append(info["state"])
        rec["post_qpos"].append(u.data.qpos.copy())
        rec["post_qvel"].append(u.data.qvel.copy())
        rec["post_state12"].append(u._state.vec())
        rec["post_rate_int"].append(ctbr_env._rate_int_torque.copy() if wrapper else np.zeros(3))
        if te or tr:
            do_reset(seeds.pop(0) if seeds else None)
    out = {k: np.array(v) for k, v in rec.items()}
    out.update({"reset_" + k: np.array(v) for k, v in resets.items()})
    for k in ("action", "obs", "pre_target", "pre_state12", "pre_prev_action", "post_state12", "info_state",
              "reset_init12", "reset_target3", "reset_obs", "reset_state12"):
        out[k] = out[k].astype(np.float32)
    return out


def trajectories_fixture():
    """utils/trajectories.py waypoint sets (evaluate.py's --trajectory options) for several
    spacings / sizes / centers."""
    from utils.trajectories import TRAJECTORY_GENERATORS as G
    out = {}
    for name, fn in G.items():
        for spacing in (0.2, 0.5, 0.8):
            out[f"{name}_s{spacing}"] = np.asarray(fn(spacing=spacing), np.float64)
    out["eight_r1.5_c"] = np.asarray(G["eight"](spacing=0.3, radius=1.5, center=np.array([0.5, -0.2, 1.2])))
    out["circle_r0.7_c"] = np.asarray(G["circle"](spacing=0.3, radius=0.7, center=np.array([0.1, 0.2, 0.8])))
    out["square_l2_c"] = np.asarray(G["square"](spacing=0.3, side_length=2.0, center=np.array([-0.3, 0.0, 1.5])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    ap.add_argument("--only", default=None, help="comma-separated fixture file names")
    args = ap.parse_args()
    _setup()
    os.makedirs(args.out, exist_ok=True)
    if args.only:
        lazy = {"golden_trajectories.npz": trajectories_fixture,
                "golden_relpos_steps.npz": lambda: rollout_fixture("hover", "relpos", 400, range(4000, 4100),
                                                                   max_episode_steps=60),
                "golden_traj_relpos_steps.npz": lambda: rollout_fixture("traj", "relpos", 300, range(5000, 5100),
                                                                        max_episode_steps=50),
                "golden_ctbr_relpos_steps.npz": lambda: rollout_fixture("hover", "ctbr_relpos", 400,
                                                                        range(6000, 6100), max_episode_steps=60),
                "golden_traj_ctbr_relpos_steps.npz": lambda: rollout_fixture("traj", "ctbr_relpos", 300,
                                                                             range(7000, 7100), max_episode_steps=50)}
        for name in args.only.split(","):
            d = lazy[name]()
            np.savez_compressed(os.path.join(args.out, name), **d)
            print(name, {k: v.shape for k, v in d.items()})
        return
    fx = {
        "golden_trajectories.npz": trajectories_fixture(),
        "golden_euler.npz": euler_fixture(),
        "golden_termination.npz": termination_fixture(),
        "golden_hover_steps.npz": rollout_fixture("hover", False, 1500, range(100, 400)),
        "golden_hover_trunc.npz": rollout_fixture("hover", False, 300, range(500, 600),
                                                  max_episode_steps=15, action_mode="hover"),
        "golden_hover_nan.npz": rollout_fixture("hover", False, 120, range(700, 800),
                                                action_mode="nan"),
        "golden_ctbr_steps.npz": rollout_fixture("hover", True, 1500, range(1000, 1300)),
        "golden_traj_ctbr_steps.npz": rollout_fixture("traj", True, 800, range(2000, 2300)),
        "golden_traj_steps.npz": rollout_fixture("traj", False, 400, range(3000, 3300)),
        "golden_relpos_steps.npz": rollout_fixture("hover", "relpos", 400, range(4000, 4100), max_episode_steps=60),
        "golden_traj_relpos_steps.npz": rollout_fixture("traj", "relpos", 300, range(5000, 5100),
                                                        max_episode_steps=50),
        "golden_ctbr_relpos_steps.npz": rollout_fixture("hover", "ctbr_relpos", 400, range(6000, 6100),
                                                        max_episode_steps=60),
        "golden_traj_ctbr_relpos_steps.npz": rollout_fixture("traj", "ctbr_relpos", 300, range(7000, 7100),
                                                             max_episode_steps=50),
    }
    for name, d in fx.items():
        path = os.path.join(args.out, name)
        np.savez_compressed(path, **d)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB",
              {k: v.shape for k, v in list(d.items())[:3]})


if __name__ == "__main__":
    main()
