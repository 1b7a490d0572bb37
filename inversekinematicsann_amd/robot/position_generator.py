"""Trajectory / point-cloud inputs: the reference's TrainingDataGenerator
shapes (robot/position_generator.py:23-97), behind the CLI's --generate-data,
plus the seeded batch generator the benchmarks use.

  * random_dist: the benchmarks' batch -- per-axis truncated normal, mean 0,
    sd 0.5, truncated to the workspace box (position_generator.py:81-97,
    'normal'), drawn with numpy's default_rng + rejection so that a seed gives the
    same batch on every machine (the reference draws from the global state);
  * circle, cube, cube_random, random, spring, random_distribution: the
    reference's generators, same arithmetic and the same draws from the same
    global random states (numpy's legacy RandomState, Python's `random`), so a
    seeded reference run and a seeded run here give the same points
    (tests/golden/make_shapes.py, tests/test_shapes_cpu.py).  Each returns an
    (n, 3) float64 array instead of a list of lists.
"""
from __future__ import annotations

import math
import random as _pyrandom

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


def circle(radius: float, no_of_samples: int, centre) -> np.ndarray:
    """position_generator.py:26-32: sample t = 0, 1, 2, ... radians (integer steps,
    as the reference), [c0, c1 + r sin t, c2 + r cos t] with libm's sin / cos."""
    c0, c1, c2 = (float(v) for v in centre)
    return np.array([[c0, c1 + radius * math.sin(t), c2 + radius * math.cos(t)]
                     for t in range(no_of_samples)], np.float64).reshape(-1, 3)


def cube(step: float, len_x: float, len_y: float, len_z: float, start=(0, 0, 0)) -> np.ndarray:
    """position_generator.py:39-46: the grid np.arange(0, len, step) per axis plus
    start, z slowest and x fastest."""
    xs, ys, zs = (np.arange(0, ln, step) for ln in (len_x, len_y, len_z))
    pts = np.empty((zs.size, ys.size, xs.size, 3), np.float64)
    pts[..., 0] = xs[None, None, :] + start[0]
    pts[..., 1] = ys[None, :, None] + start[1]
    pts[..., 2] = zs[:, None, None] + start[2]
    return pts.reshape(-1, 3)


def cube_random(step: float, len_x: float, len_y: float, len_z: float,
                start=(0, 0, 0)) -> np.ndarray:
    """position_generator.py:48-55: as many points as np.arange(0, lx ly lz, step)
    has entries, each len * rand() + start per axis, drawn x, y, z point by point
    from numpy's global RandomState."""
    count = np.arange(0, len_x * len_y * len_z, step).size
    u = np.random.rand(count, 3)  # the same stream as 3 count single draws
    return u * np.array([len_x, len_y, len_z], np.float64) + np.array(start, np.float64)


def _minmax_scale(v: np.ndarray, lo: float, hi: float) -> np.ndarray:
    """sklearn.preprocessing.minmax_scale(v, (lo, hi)) for one feature, the
    MinMaxScaler arithmetic: scale = (hi - lo) / range (a range below 10 eps counts
    as 1), min = lo - data_min * scale, v * scale + min."""
    dmin, dmax = np.nanmin(v), np.nanmax(v)
    rng = dmax - dmin
    if rng < 10 * np.finfo(np.float64).eps:
        rng = 1.0
    scale = (hi - lo) / rng
    return v * scale + (lo - dmin * scale)


def random(no_of_samples: int, limits) -> np.ndarray:  # noqa: A001 -- the reference's name
    """position_generator.py:65-70: per axis x, y, z, np.random.randn(n) min-max
    scaled onto the axis' limits."""
    cols = [_minmax_scale(np.random.randn(no_of_samples), float(limits[a][0]),
                          float(limits[a][1])) for a in ("x", "y", "z")]
    return np.stack(cols, axis=1)


def spring(no_of_samples: int, len_x: float, len_y: float, len_z: float) -> np.ndarray:
    """position_generator.py:72-78."""
    axis_z = np.linspace(0, len_z, no_of_samples)
    axis_x = (np.sin(axis_z) * len_x) + len_x
    axis_y = (np.cos(axis_z) * len_y) + len_y
    return np.stack([axis_x / 2, axis_y / 2, axis_z], axis=1)


def random_distribution(no_of_samples: int, limits, distribution: str = "normal",
                        std_dev: float = 0.5) -> np.ndarray:
    """position_generator.py:80-97, per axis in the dict's order: 'normal' --
    scipy's truncnorm (mean 0, sd std_dev, truncated to the axis' limits) drawn
    from numpy's global state; 'uniform' -- Python's random.uniform per value;
    'random' -- np.linspace over the limits, shuffled by np.random.shuffle."""
    cols = []
    for lo, hi in limits.values():
        lo, hi = float(lo), float(hi)
        if distribution == "normal":
            from scipy.stats import truncnorm
            cols.append(np.asarray(truncnorm((lo - 0) / std_dev, (hi - 0) / std_dev, loc=0,
                                             scale=std_dev).rvs(no_of_samples), np.float64))
        elif distribution == "uniform":
            cols.append(np.array([_pyrandom.uniform(lo, hi) for _ in range(no_of_samples)],
                                 np.float64))
        elif distribution == "random":
            arr = np.linspace(lo, hi, no_of_samples)
            np.random.shuffle(arr)
            cols.append(arr)
        else:
            raise ValueError(f"unknown distribution {distribution!r} "
                             "(normal, uniform or random)")
    return np.stack(cols, axis=1)
