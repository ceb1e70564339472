"""The reference's utils API (utils/normalization.py:7-30, utils/state.py:9-108,
utils/trajectories.py:6-81) as this package exposes it, against golden vectors produced by the
reference's own code (tools/gen_golden.py)."""
import os

import numpy as np

from uav_reinforcement_learning_control_amd.utils import Box, QuadState, denormalize, normalize
from uav_reinforcement_learning_control_amd.utils import trajectories as T
from uav_reinforcement_learning_control_amd.envs import hover_env  # noqa: F401  (import check)


def _obs_box():
    from oracle import oracle as O
    cfg = O.default_cfg(O.ENV_HOVER, O.WRAP_NONE)
    return Box(np.array(cfg.obs_low[:], np.float32), np.array(cfg.obs_high[:], np.float32), (12,), np.float32)


def test_normalize_reproduces_reference_observations(golden_dir):
    """HoverEnv._get_obs = normalize(state with rel pos, obs bounds) in float32: bit-exact."""
    d = np.load(os.path.join(golden_dir, "golden_hover_steps.npz"))
    box = _obs_box()
    for t in range(len(d["obs"])):
        x = d["post_state12"][t].copy()
        if d["terminated"][t] or d["truncated"][t]:
            continue  # the recorded obs is still the step's obs, but keep the loop simple
        x[0:3] = d["pre_target"][t] - x[0:3]
        got = normalize(x, box)
        assert got.dtype == np.float32
        assert np.array_equal(got, d["obs"][t]), t


def test_denormalize_inverts_normalize_on_action_bounds():
    box = Box(np.array([0.0, -0.5, -0.5, -0.5], np.float32), np.array([52.0, 0.5, 0.5, 0.5], np.float32),
              (4,), np.float32)
    assert np.array_equal(denormalize(np.full(4, -1.0, np.float32), box), box.low)
    assert np.array_equal(denormalize(np.full(4, 1.0, np.float32), box), box.high)
    a = np.random.default_rng(0).uniform(-1, 1, (100, 4)).astype(np.float32)
    np.testing.assert_allclose(normalize(denormalize(a, box), box), a, atol=2e-7)


def test_quadstate_matches_reference_euler(golden_dir):
    g = np.load(os.path.join(golden_dir, "golden_euler.npz"))
    for q, s in zip(g["quat_wxyz"], g["state12"]):
        st = QuadState()
        st.set_from_mujoco(np.concatenate([[0.1, -0.2, 0.3], q]), np.arange(6, dtype=np.float64) * 0.1)
        assert np.array_equal(st.vec(), s), (q, st.vec(), s)
    for e, qp in zip(g["euler_in"], g["qpos_from_euler"]):
        st = QuadState()
        st.state[3:6] = e
        qpos, qvel = st.get_mujoco_state()
        np.testing.assert_allclose(qpos[3:7], qp[3:7], atol=2e-16)
        assert qvel.shape == (6,)


def test_quadstate_accessors_and_random_reset():
    st = QuadState()
    st.reset_uav_state(np.array([1.0, 2.0, 3.0]), np.array([1.0, 0, 0, 0]), np.array([0.1, 0.2, 0.3]),
                       np.array([0.4, 0.5, 0.6]))
    assert np.array_equal(st.position, np.float32([1, 2, 3])) and np.array_equal(st.attitude, np.zeros(3))
    assert np.allclose(st.velocity, [0.1, 0.2, 0.3]) and np.allclose(st.angular_velocity, [0.4, 0.5, 0.6])
    b = Box(np.full(12, -1.0, np.float32), np.full(12, 1.0, np.float32), (12,), np.float32)
    st.random_reset(np.random.default_rng(3), b)
    assert st.state.dtype == np.float32 and np.all(np.abs(st.state) <= 1)
    assert np.array_equal(st.state, np.random.default_rng(3).uniform(b.low, b.high).astype(np.float32))
    assert "QuadState(" in repr(st)


def test_reference_named_generators_return_lists(golden_dir):
    g = np.load(os.path.join(golden_dir, "golden_trajectories.npz"))
    for name, fn in (("eight", T.generate_figure_eight), ("circle", T.generate_circle),
                     ("square", T.generate_square)):
        for sp in (0.2, 0.5, 0.8):
            wps = fn(spacing=sp)
            assert isinstance(wps, list) and all(w.shape == (3,) for w in wps)
            np.testing.assert_allclose(np.array(wps), g[f"{name}_s{sp}"], rtol=0, atol=1e-12)
        assert T.TRAJECTORY_GENERATORS[name] is fn
