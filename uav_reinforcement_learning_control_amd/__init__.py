"""MI355X-native vectorized quadrotor env (HoverEnv / RateControlWrapper / TrajectoryFollowEnv
hot path of Karl-Liu-ch/uav_reinforcement_learning_control) with a PyTorch-ROCm PPO learner.

The env step/reset run only as HIP kernels from libquadenv.so (C ABI: include/quadenv.h).
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401

__all__ = ["_native", "__version__"]
