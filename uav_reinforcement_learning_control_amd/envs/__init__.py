from .hover_env import HoverEnv, TrajectoryFollowEnv
from .rate_wrapper import RateControlWrapper
from .sb3_vec_env import QuadSB3VecEnv, make_vec_env
from .vec_env import QuadVecEnv
from .wrappers import WRAPPER_REGISTRY, RelPosActWrapper, get_wrapper

__all__ = ["HoverEnv", "TrajectoryFollowEnv", "RateControlWrapper", "RelPosActWrapper",
           "QuadVecEnv", "QuadSB3VecEnv", "make_vec_env", "WRAPPER_REGISTRY", "get_wrapper"]
