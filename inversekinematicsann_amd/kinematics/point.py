"""3-D point value type and the two scalar helpers of kinematics/point.py.

These are host-side VALUE helpers kept for API compatibility (the reference's
tests/point_unit.py exercises them); no batched solve goes through them -- on
the GPU the same arithmetic runs inside the FABRIK kernel (csrc/ik_common.h
dist3 / point_between).
"""
from __future__ import annotations

from math import sqrt

import numpy as np


class Point(list):
    """3D point (kinematics/point.py:10-22): a list with .x .y .z; ValueError
    unless the input has shape (3,)."""

    def __init__(self, xyz):
        shape = np.shape(xyz)
        if shape != (3,):
            raise ValueError(f'3D Point input shape should be (3,) not {shape}')
        super().__init__(xyz)
        self.x, self.y, self.z = xyz

    def __str__(self):
        return f'Point{self.x, self.y, self.z}'

    def __repr__(self):
        return f'<Point at 0x{id(self):x}, x={self.x}, y={self.y}, z={self.z}>'


def get_distance_between(point_a, point_b):
    """|a - b|_2 summed left to right (kinematics/point.py:25-29)."""
    return sqrt((point_a.x - point_b.x) ** 2 + (point_a.y - point_b.y) ** 2
                + (point_a.z - point_b.z) ** 2)


def get_point_between(start_point, end_point, distance=None):
    """Point at `distance` from start towards end; the midpoint by default
    (kinematics/point.py:32-45).  ZeroDivisionError if the points coincide."""
    span = get_distance_between(start_point, end_point)
    if distance is None:
        distance = span / 2
    ratio = distance / span
    return Point([start_point.x + ratio * (end_point.x - start_point.x),
                  start_point.y + ratio * (end_point.y - start_point.y),
                  start_point.z + ratio * (end_point.z - start_point.z)])
