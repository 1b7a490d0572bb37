"""Inverse kinematics API -- drop-in for the reference's kinematics/inverse.py.

Same class names, constructor signatures, defaults, return types and
exceptions as kinematics/inverse.py:18-155; the batch is solved on the GPU in
one call instead of a Python loop over points:

* FabrikInverseKinematics.ikine -> libikhip ik_fabrik_solve (float64, iteration
  counts bit-exact with the reference);
* AnnInverseKinematics.ikine    -> libikhip ik_ann_solve (fused fp32 MLP).

Errors follow the reference's sequential semantics: the workspace check covers
every point first (inverse.py:117,153) and raises OutOfRobotReachException for
the first point outside; otherwise the lowest-index point whose solve raised
decides the exception (ZeroDivisionError / ValueError), as the reference's loop
would have stopped there.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from math import atan2

import numpy as np

from .. import _native
from ..robot.robot import OutOfRobotReachException
from .ann import ANN, as_features as as_ann_points
from .forward import ForwardKinematics
from .fabrik import Fabrik

_ERR_EXC = {
    _native.IK_E_ZERODIV: (ZeroDivisionError, 'float division by zero'),
    _native.IK_E_DOMAIN: (ValueError, 'math domain error'),
    _native.IK_E_ANGLE_RANGE: (OutOfRobotReachException,
                               'Forward Kinematics exception, robot joints angles limits are '
                               '(-2pi, 2pi)'),
}


def limits_array(workspace_limits) -> np.ndarray:
    """{'x': [lo, hi], ...} in dict order -> [lo0, hi0, lo1, hi1, lo2, hi2];
    axes the dict does not name are unbounded (zip() in inverse.py:31 stops)."""
    lim = np.array([-np.inf, np.inf] * 3, np.float64)
    for i, (_, v) in enumerate(list(workspace_limits.items())[:3]):
        lim[2 * i], lim[2 * i + 1] = float(v[0]), float(v[1])
    return lim


def as_points(dest_points) -> np.ndarray:
    """The n x 3 float64 batch of destination points.  Every point must be 3D,
    as the reference's Point (point.py:12-14) requires; a wrong width raises its
    ValueError instead of being reinterpreted as other points."""
    pts = np.asarray(dest_points, dtype=np.float64)
    if pts.ndim == 2 and pts.shape[0] == 0:
        return np.empty((0, 3), np.float64)
    if pts.ndim == 1 and pts.shape[0] == 0:
        return np.empty((0, 3), np.float64)
    if pts.ndim != 2 or pts.shape[1] != 3:
        bad = pts.shape[1:] if pts.ndim >= 2 else pts.shape
        raise ValueError(f'3D Point input shape should be (3,) not {tuple(bad)}')
    return np.ascontiguousarray(pts)


class InverseKinematics(ABC):
    """Inverse kinematics base (inverse.py:18-40)."""

    def __init__(self, dh_matrix, joints_distances, workspace_limits):
        self.dh_matrix = dh_matrix
        self.joints_distances = joints_distances
        self.workspace_limits = workspace_limits
        self.fkine = ForwardKinematics(self.dh_matrix)
        self.last_stats = None

    def _ctx(self):
        """The process context holding this object's robot: uploaded when it
        differs from what the context holds (Context.set_robot compares), so
        objects with different robots can interleave and repeated calls of one
        object upload nothing."""
        ctx = _native.context()
        ctx.set_robot(np.asarray(self.dh_matrix, np.float64),
                      np.asarray(self.joints_distances, np.float64),
                      limits_array(self.workspace_limits))
        return ctx

    def _raise_out_of_reach(self, dest_points, idx):
        raise OutOfRobotReachException(
            f'Inverse Kinematics exception, point {dest_points[idx]} '
            'is out of manipulator reach area! '
            f'Limits: {self.workspace_limits}')

    def check_limits(self, dest_points):
        """Raise OutOfRobotReachException for the first point outside the
        (inclusive) workspace box (inverse.py:26-35), checked on the GPU."""
        pts = as_points(dest_points)
        st = self._ctx().check_limits(pts)
        if st.first_oob >= 0:
            self._raise_out_of_reach(dest_points, st.first_oob)

    @abstractmethod
    def ikine(self, dest_points):
        """Calculate inverse kinematics"""


class FabrikInverseKinematics(InverseKinematics):
    """Reaching inverse kinematics using the FABRIK method (inverse.py:45-139)."""

    def __init__(self, dh_matrix, joints_distances, workspace_limits,
                 max_err=0.001, max_iterations_num=100):
        super().__init__(dh_matrix, joints_distances, workspace_limits)
        self.fabrik = Fabrik(joints_distances, max_err, max_iterations_num)
        self.last_iterations = None

    def ikine(self, dest_points):
        """Joint angles [theta1..theta4] (float64) for every destination point."""
        pts = as_points(dest_points)
        if pts.shape[0] == 0:
            return []
        ang, iters, _, st = self._ctx().fabrik_solve(pts, self.fabrik.err_margin,
                                                     self.fabrik.max_iter_num)
        self.last_stats = st
        self.last_iterations = iters
        if st.first_oob >= 0:
            self._raise_out_of_reach(dest_points, st.first_oob)
        # inverse.py:125 writes each point's theta_1 into dh_matrix[0][0]; the
        # value left behind is the one of the last point processed.
        last = st.first_err if st.first_err >= 0 else pts.shape[0] - 1
        self.dh_matrix[0][0] = float(atan2(pts[last, 1], pts[last, 0]))
        if st.first_err >= 0:
            exc, msg = _ERR_EXC.get(st.first_err_code, (RuntimeError, 'ikine failed'))
            raise exc(msg)
        return ang.tolist()


class AnnInverseKinematics(InverseKinematics):
    """Reaching inverse kinematics using the ANN method (inverse.py:142-155)."""

    def __init__(self, dh_matrix, joints_distances, workspace_limits):
        super().__init__(dh_matrix, joints_distances, workspace_limits)
        self.ann = ANN(workspace_limits, dh_matrix)

    def load_model(self, model_name):
        """Load a model (.h5 + _scaler_{x,y}.bin, or .npz) onto the GPU."""
        self.ann.load_model(model_name)

    def ikine(self, dest_points):
        """Predicted joint angles (float32 values as Python floats)."""
        pts = as_ann_points(dest_points)
        if pts.shape[0] == 0:
            return []
        self._ctx()
        ang, st = self.ann.predict_checked(pts)
        self.last_stats = st
        if st.first_oob >= 0:
            self._raise_out_of_reach(dest_points, st.first_oob)
        return ang.tolist()
