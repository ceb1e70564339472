from . import drone_config
from .spaces import Box

__all__ = ["Box", "drone_config"]
