"""Synthetic trajectory inputs for benchmarks and tests.

Only the two shapes the measurement plan uses are restated here (the other
generators of robot/position_generator.py are out of scope):
  * random_dist: per-axis truncated normal, mean 0, sd 0.5, truncated to the
    workspace box (position_generator.py:81-97, 'normal'); drawn here with
    numpy's default_rng + rejection so a seed gives the same batch everywhere;
  * spring: position_generator.py:73-78.
"""
from __future__ import annotations

import numpy as np

from .robot import SixDOFRobot


def random_dist(n: int, seed: int = 0, std_dev: float = 0.5,
                limits=SixDOFRobot.effector_workspace_limits) -> np.ndarray:
    rng = np.random.default_rng(seed)
    out = np.empty((n, 3), np.float64)
    for c, (lo, hi) in enumerate(limits.values()):
        got = 0
        while got < n:
            need = n - got
            v = rng.normal(0.0, std_dev, int(need * 1.3) + 64)
            v = v[(v >= lo) & (v <= hi)][:need]
            out[got:got + v.shape[0], c] = v
            got += v.shape[0]
    return out


def spring(no_of_samples: int, len_x: float, len_y: float, len_z: float) -> np.ndarray:
    axis_z = np.linspace(0, len_z, no_of_samples)
    axis_x = (np.sin(axis_z) * len_x) + len_x
    axis_y = (np.cos(axis_z) * len_y) + len_y
    return np.stack([axis_x / 2, axis_y / 2, axis_z], axis=1)
