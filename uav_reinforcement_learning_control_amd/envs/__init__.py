from .hover_env import HoverEnv, TrajectoryFollowEnv
from .rate_wrapper import RateControlWrapper
from .vec_env import QuadVecEnv
from .wrappers import WRAPPER_REGISTRY, RelPosActWrapper, get_wrapper

__all__ = ["HoverEnv", "TrajectoryFollowEnv", "RateControlWrapper", "RelPosActWrapper",
           "QuadVecEnv", "WRAPPER_REGISTRY", "get_wrapper"]
