from . import drone_config
from .normalization import denormalize, normalize
from .spaces import Box
from .state import QuadState

__all__ = ["Box", "drone_config", "normalize", "denormalize", "QuadState"]
