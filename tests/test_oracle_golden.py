"""The CPU oracle (oracle/) against golden vectors produced by the reference's own env code.

Fixtures: tests/golden/*.npz, written by tools/gen_golden.py (reference HoverEnv /
RateControlWrapper / TrajectoryFollowEnv / QuadState / normalize executed unmodified; physics
inside mj_step = the oracle's MuJoCo restatement, so these pin the env layer).
Bar: obs / state / flags / voltage bit-exact; reward and float64 physics to 1e-13.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

ROLL = [("hover_steps", O.ENV_HOVER, O.WRAP_NONE, None),
        ("hover_trunc", O.ENV_HOVER, O.WRAP_NONE, 15),
        ("hover_nan", O.ENV_HOVER, O.WRAP_NONE, None),
        ("ctbr_steps", O.ENV_HOVER, O.WRAP_CTBR, None),
        ("traj_ctbr_steps", O.ENV_TRAJ, O.WRAP_CTBR, None),
        ("traj_steps", O.ENV_TRAJ, O.WRAP_NONE, None)]


def _eq_nan(a, b):
    a = np.asarray(a); b = np.asarray(b)
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("name,kind,wrap,maxsteps", ROLL)
def test_env_step_matches_reference(golden_dir, name, kind, wrap, maxsteps):
    d = np.load(os.path.join(golden_dir, f"golden_{name}.npz"))
    cfg = O.default_cfg(kind, wrap)
    if maxsteps:
        cfg.max_episode_steps = maxsteps
    env = O.Env(cfg=cfg)
    for t in range(len(d["action"])):
        env.set_full_state(d["pre_qpos"][t], d["pre_qvel"][t], d["pre_voltage"][t],
                           d["pre_target"][t], d["pre_step"][t], d["pre_rate_int"][t],
                           d["pre_state12"][t])
        o = O.out_to_dict(env.step(d["action"][t]))
        assert _eq_nan(o["obs"], d["obs"][t]), (name, t)
        assert _eq_nan(o["state12"], d["post_state12"][t]), (name, t)
        assert o["terminated"] == d["terminated"][t] and o["truncated"] == d["truncated"][t]
        assert _eq_nan(o["voltage"], d["voltage"][t]) and _eq_nan(o["voltage_scale"], d["vscale"][t])
        np.testing.assert_allclose(o["reward"], d["reward"][t], rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(o["motor_commands"], d["motor"][t], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(env.qpos, d["post_qpos"][t], rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(env.qvel, d["post_qvel"][t], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(np.array(env.s.rate_int[:]), d["post_rate_int"][t],
                                   rtol=1e-13, atol=1e-16)


@pytest.mark.parametrize("name,kind,wrap,maxsteps", ROLL)
def test_env_reset_matches_reference(golden_dir, name, kind, wrap, maxsteps):
    d = np.load(os.path.join(golden_dir, f"golden_{name}.npz"))
    env = O.Env(kind, wrap)
    for i in range(len(d["reset_init12"])):
        obs = env.reset_with(d["reset_init12"][i], d["reset_target3"][i])
        assert np.array_equal(obs, d["reset_obs"][i])
        np.testing.assert_allclose(env.qpos, d["reset_qpos"][i], rtol=0, atol=2e-16)
        assert np.array_equal(env.qvel, d["reset_qvel"][i])


def test_euler_conversions_match_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "golden_euler.npz"))
    env = O.Env()
    for q, s in zip(d["quat_wxyz"], d["state12"]):
        env.s.qpos[:] = [0.1, -0.2, 0.3] + list(q) + [0, 0, 0, 0]
        env.s.qvel[:] = list(np.arange(6) * 0.1) + [0, 0, 0, 0]
        O.lib().oracle_get_obs(O.C.byref(env.cfg), O.C.byref(env.s),
                               np.zeros(12, np.float32).ctypes.data_as(O.C.POINTER(O.C.c_float)))
        got = np.array(env.s.state12[:], np.float32)
        assert np.array_equal(got, s), (q, got, s)
    for e, qp in zip(d["euler_in"], d["qpos_from_euler"]):
        np.testing.assert_allclose(O.euler_to_quat(e.astype(np.float64)), qp[3:7], atol=2e-16)


def test_termination_matches_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "golden_termination.npz"))
    for kind, name in ((O.ENV_HOVER, "hover"), (O.ENV_TRAJ, "traj")):
        cfg = O.default_cfg(kind, O.WRAP_NONE)
        lo = np.array(cfg.term_low[:], np.float32)
        hi = np.array(cfg.term_high[:], np.float32)
        for s, t in zip(d[f"{name}_states"], d[f"{name}_terminated"]):
            mine = (not np.isfinite(s).all()) or (not ((s >= lo) & (s <= hi)).all())
            assert mine == bool(t)


@pytest.mark.parametrize("name,kind,wrap", [("relpos_steps", O.ENV_HOVER, O.WRAP_RELPOS),
                                             ("traj_relpos_steps", O.ENV_TRAJ, O.WRAP_RELPOS),
                                             ("ctbr_relpos_steps", O.ENV_HOVER, O.WRAP_CTBR_RELPOS),
                                             ("traj_ctbr_relpos_steps", O.ENV_TRAJ, O.WRAP_CTBR_RELPOS)])
def test_relpos_wrapper_matches_reference(golden_dir, name, kind, wrap):
    """RelPosActWrapper(HoverEnv / TrajectoryFollowEnv) (envs/wrappers.py:13-25), the reference's
    wrapper executed unmodified: obs7 = [obs12[0:3], _prev_action] bit-exact for every step (the
    previous action is the one just taken) and every reset (zeros, hover_env.py:212). The
    *_ctbr_relpos fixtures are RelPosActWrapper(RateControlWrapper(env)) (the README's stack): the
    rate controller's torques drive the step and obs7 carries the RATE action (rate_wrapper.py:105)."""
    d = np.load(os.path.join(golden_dir, f"golden_{name}.npz"))
    cfg = O.default_cfg(kind, wrap)
    cfg.max_episode_steps = 60 if kind == O.ENV_HOVER else 50
    env = O.Env(cfg=cfg)
    for t in range(len(d["action"])):
        env.set_full_state(d["pre_qpos"][t], d["pre_qvel"][t], d["pre_voltage"][t], d["pre_target"][t],
                           d["pre_step"][t], d["pre_rate_int"][t], d["pre_state12"][t], d["pre_prev_action"][t])
        o = O.out_to_dict(env.step(d["action"][t]))
        assert np.array_equal(o["obs7"], d["obs"][t]), (name, t)
        if wrap == O.WRAP_CTBR_RELPOS:
            np.testing.assert_allclose(env.rate_int, d["post_rate_int"][t], rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(o["motor_commands"], d["motor"][t], rtol=1e-13, atol=1e-13)
        assert o["terminated"] == d["terminated"][t] and o["truncated"] == d["truncated"][t]
        np.testing.assert_allclose(o["reward"], d["reward"][t], rtol=1e-13, atol=1e-15)
    assert d["terminated"].any() or d["truncated"].any()
    for i in range(len(d["reset_init12"])):
        e = O.Env(cfg=cfg)
        obs = e.reset_with(d["reset_init12"][i], d["reset_target3"][i])
        assert np.array_equal(e.relpos_obs(obs), d["reset_obs"][i]), (name, i)
