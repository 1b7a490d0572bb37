"""FABRIK on the GPU -- kinematics/fabrik.py of the reference.

Fabrik(joints_distances, err_margin, max_iter_num).calculate(init, goal)
returns the final joint positions as Points (fabrik.py:44-67); the loop runs in
libikhip's fabrik_calc kernel (float64, one goal per lane, reference operation
order).  calculate_batch() solves n goals in one launch.
"""
from __future__ import annotations

import numpy as np

from .. import _native
from .point import Point


class Fabrik:
    """Forward And Backward Reaching Inverse Kinematics (fabrik.py:9-16)."""

    def __init__(self, joints_distances, err_margin=0.001, max_iter_num=100):
        self.joints_distances = joints_distances
        self.err_margin = err_margin
        self.max_iter_num = max_iter_num
        self.last_iterations = None

    def calculate(self, init_joints_positions, goal_effector_position):
        """Joint positions after FABRIK iterations (fabrik.py:44-67)."""
        if not all(x == len(init_joints_positions)
                   for x in (len(init_joints_positions), len(self.joints_distances))):
            raise ValueError('Input vectors should have equal lengths!')
        goal = Point(goal_effector_position)
        out, it = self.calculate_batch(np.asarray([list(p) for p in init_joints_positions],
                                                  np.float64), np.asarray([list(goal)]))
        self.last_iterations = int(it[0])
        return [Point(list(map(float, q))) for q in out[0]]

    def calculate_batch(self, init, goals):
        """init: nj x 3 (shared) or n x nj x 3; goals n x 3 -> (joints n x nj x 3, iters)."""
        ctx = _native.context()
        out, it, st = ctx.fabrik_calc(self.joints_distances, init, goals, self.err_margin,
                                      self.max_iter_num)
        if st.first_err >= 0:
            raise ZeroDivisionError('float division by zero')
        return out, it
