"""Host-side checks of the SB3 VecEnv facade (no GPU): argument validation and the factory probe."""
import pytest


def test_make_vec_env_needs_a_quad_env_factory():
    from uav_reinforcement_learning_control_amd.envs.sb3_vec_env import QuadSB3VecEnv, _facade_spec

    class NotAnEnv:
        unwrapped = object()

    with pytest.raises(TypeError):
        _facade_spec(NotAnEnv())
    with pytest.raises(TypeError):
        QuadSB3VecEnv(object())
