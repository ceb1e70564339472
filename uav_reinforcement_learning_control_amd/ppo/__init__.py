from .gae import gae

__all__ = ["gae"]
