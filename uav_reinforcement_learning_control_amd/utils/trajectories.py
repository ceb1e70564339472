"""Waypoint trajectories for evaluation (reference utils/trajectories.py:6-81), as float64 numpy
arrays [n, 3]. Same curves and sampling rules as the reference's generators:

  eight   lemniscate x = r cos t, y = (r/2) sin 2t at altitude z, sampled at equal arc length
          (arc length from a 1000-point rectangle-rule integral of |dp/dt| over [0, 2 pi)),
          n = max(ceil(L / spacing), 8) points
  circle  n = max(ceil(2 pi r / spacing), 4) equal-angle points
  square  corners (+h,+h), (-h,+h), (-h,-h), (+h,-h) (h = side / 2), each edge split into
          max(ceil(side / spacing), 1) equal pieces (corner included, next corner excluded)
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

_DEFAULT_CENTER = (0.0, 0.0, 1.0)


def _center(c) -> np.ndarray:
    return np.asarray(_DEFAULT_CENTER if c is None else c, np.float64)


def figure_eight(spacing: float = 0.5, radius: float = 1.0, center=None) -> np.ndarray:
    c = _center(center)
    m = 1000
    t = np.arange(m, dtype=np.float64) * (2.0 * math.pi / m)
    speed = np.hypot(radius * np.sin(t), radius * np.cos(2.0 * t))   # |d/dt (r cos t, r/2 sin 2t)|
    s = np.cumsum(speed * (2.0 * math.pi / m))                        # arc length at each sample
    n = max(int(math.ceil(s[-1] / spacing)), 8)
    tq = np.interp(np.arange(n) * (s[-1] / n), s, t)
    return np.stack([c[0] + radius * np.cos(tq), c[1] + 0.5 * radius * np.sin(2.0 * tq),
                     np.full(n, c[2])], axis=1)


def circle(spacing: float = 0.5, radius: float = 1.0, center=None) -> np.ndarray:
    c = _center(center)
    n = max(int(math.ceil(2.0 * math.pi * radius / spacing)), 4)
    th = 2.0 * math.pi * np.arange(n) / n
    return np.stack([c[0] + radius * np.cos(th), c[1] + radius * np.sin(th), np.full(n, c[2])], axis=1)


def square(spacing: float = 0.5, side_length: float = 1.5, center=None) -> np.ndarray:
    c = _center(center)
    h = 0.5 * side_length
    corners = c + np.array([[h, h, 0.0], [-h, h, 0.0], [-h, -h, 0.0], [h, -h, 0.0]])
    pts = []
    for k in range(4):
        a, b = corners[k], corners[(k + 1) % 4]
        pieces = max(int(math.ceil(np.linalg.norm(b - a) / spacing)), 1)
        for j in range(pieces):
            pts.append(a + (j / pieces) * (b - a))
    return np.array(pts)


def generate_figure_eight(spacing: float = 0.5, radius: float = 1.0, center=None) -> list:
    """The reference's name and return type (utils/trajectories.py:6): a list of [3] arrays."""
    return list(figure_eight(spacing, radius, center))


def generate_circle(spacing: float = 0.5, radius: float = 1.0, center=None) -> list:
    """utils/trajectories.py:37."""
    return list(circle(spacing, radius, center))


def generate_square(spacing: float = 0.5, side_length: float = 1.5, center=None) -> list:
    """utils/trajectories.py:53."""
    return list(square(spacing, side_length, center))


# the reference's registry (utils/trajectories.py:76-81): list-returning generators
TRAJECTORY_GENERATORS = {"eight": generate_figure_eight, "circle": generate_circle, "square": generate_square}
_ARRAYS = {"eight": figure_eight, "circle": circle, "square": square}


def make_trajectory(name: str, spacing: float = 0.5, center: Optional[np.ndarray] = None, **kw) -> np.ndarray:
    """The named waypoint set as one float64 [n, 3] array (what the batched evaluator uploads)."""
    return _ARRAYS[name](spacing=spacing, center=center, **kw)
