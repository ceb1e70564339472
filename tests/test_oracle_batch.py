"""The CPU oracle's batch entry points (oracle_reset_draw_batch, oracle_env_reset_batch,
oracle_env_prepare_batch + oracle_env_step_batch; oracle/oracle.py reset_draw_batch /
reset_obs_batch / step_batch) against its per-env path, bit for bit. The full-batch GPU parity
tests (tests/test_gpu_parity_full.py) check the 65,536-env step kernels against these batch
functions, so they must be the same restatement as the per-env one the golden vectors pin
(tests/test_oracle_golden.py). Test infrastructure only; no GPU."""
import numpy as np
import pytest

from oracle import oracle as O

KINDS = [(O.ENV_HOVER, O.WRAP_NONE), (O.ENV_HOVER, O.WRAP_CTBR), (O.ENV_TRAJ, O.WRAP_NONE),
         (O.ENV_TRAJ, O.WRAP_CTBR)]


def _states(n, rng):
    """Random float32 states across the termination bounds (the GPU parity tests' generator)."""
    qpos = np.zeros((n, 11), np.float32)
    qpos[:, :3] = rng.uniform([-1.9, -1.9, 0.05], [1.9, 1.9, 1.95], (n, 3))
    q = rng.normal(size=(n, 4))
    qpos[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    qpos[:, 7:] = rng.uniform(-60, 60, (n, 4))
    qvel = np.zeros((n, 10), np.float32)
    qvel[:, :3] = rng.normal(0, 3.0, (n, 3))
    qvel[:, 3:6] = rng.normal(0, 6.0, (n, 3))
    qvel[:, 6:] = rng.normal(0, 30.0, (n, 4))
    return dict(qpos=qpos, qvel=qvel, voltage=rng.uniform(7.6, 8.4, n).astype(np.float32),
                target=rng.uniform([-1.5, -1.5, 0.3], [1.5, 1.5, 1.8], (n, 3)).astype(np.float32),
                step_count=rng.integers(0, 512, n).astype(np.int32),
                rate_int=rng.uniform(-0.01, 0.01, (n, 3)).astype(np.float32))


@pytest.mark.parametrize("kind,wrap", KINDS)
def test_reset_batch_is_the_per_env_reset(kind, wrap):
    cfg = O.default_cfg(kind, wrap)
    rng = np.random.default_rng(3 + kind)
    gids = rng.integers(0, 1 << 40, 200, dtype=np.uint64)
    eps = rng.integers(0, 1 << 20, 200).astype(np.uint32)
    seed = 0x1234_5678_9ABC
    i12, t3 = O.reset_draw_batch(cfg, seed, gids, eps)
    obs = O.reset_obs_batch(cfg, seed, gids, eps)
    for r in range(len(gids)):
        a12, a3 = O.reset_draw(cfg, seed, int(gids[r]), int(eps[r]))
        assert np.array_equal(i12[r], a12) and np.array_equal(t3[r], a3), r
        assert np.array_equal(obs[r], O.Env(cfg=cfg).reset_with(a12, a3)), r


@pytest.mark.parametrize("kind,wrap", KINDS)
def test_step_batch_is_the_per_env_step(kind, wrap):
    cfg = O.default_cfg(kind, wrap)
    n = 300
    rng = np.random.default_rng(11 + 2 * kind + wrap)
    st = _states(n, rng)
    st["step_count"][::7] = cfg.max_episode_steps - 1  # time-limit truncations in the batch
    st["qpos"][3::13, 2] = 0.001  # falling through the floor: terminations
    st["qvel"][3::13, 2] = -5.0
    acts = rng.uniform(-1.3, 1.3, (n, 4)).astype(np.float32)
    acts[5] = np.nan  # a bad control
    b = O.step_batch(cfg, st, acts)
    assert b["truncated"].any() and b["terminated"].any()
    for i in range(n):
        e = O.Env(cfg=cfg)
        e.set_full_state(st["qpos"][i], st["qvel"][i], st["voltage"][i], st["target"][i],
                         st["step_count"][i], st["rate_int"][i])
        o = O.out_to_dict(e.step(acts[i]))
        for k in ("obs", "state12", "motor_commands", "env_action"):
            assert np.array_equal(b[k][i], o[k], equal_nan=True), (k, i)
        for k in ("reward", "voltage", "voltage_scale", "terminated", "truncated"):
            assert np.array_equal(b[k][i], o[k], equal_nan=True), (k, i)
        assert np.array_equal(b["qpos"][i], e.qpos, equal_nan=True), i
        assert np.array_equal(b["qvel"][i], e.qvel, equal_nan=True), i
        assert np.array_equal(b["rate_int"][i], np.array(e.s.rate_int[:]), equal_nan=True), i
        assert b["step_count"][i] == e.s.step_count, i
