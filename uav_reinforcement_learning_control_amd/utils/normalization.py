"""normalize / denormalize with the reference's signatures (utils/normalization.py:7-30): affine
maps between a Box's [low, high] and [-1, 1], element-wise in the Box's dtype (float32 for the
env's spaces). The step kernels do the same arithmetic per element (csrc/quad_physics.h norm_obs1,
denorm1); these are the host-side helpers callers of the reference import."""
from __future__ import annotations

import numpy as np


def normalize(x: np.ndarray, space) -> np.ndarray:
    """[space.low, space.high] -> [-1, 1] (not clipped): 2 (x - low) / (high - low) - 1."""
    span = space.high - space.low
    return 2.0 * (x - space.low) / span - 1.0


def denormalize(x_normed: np.ndarray, space) -> np.ndarray:
    """[-1, 1] -> [space.low, space.high] (not clipped): (x + 1) / 2 (high - low) + low."""
    span = space.high - space.low
    return (x_normed + 1.0) / 2.0 * span + space.low
