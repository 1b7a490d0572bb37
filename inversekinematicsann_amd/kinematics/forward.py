"""Forward kinematics on the GPU -- kinematics/forward.py of the reference.

ForwardKinematics(dh).fkine(angles) returns (M_4, [M_1, M_2, M_3, M_4]) like
the reference (forward.py:73-94), computed by libikhip's fk kernel (one point
per lane, float64 DH chain).  fkine_batch(angles) is the batched entry point
(effector xyz n x 3), used for the CLI's --verbose round trip (cli.py:54-61).
"""
from __future__ import annotations

import numpy as np

from .. import _native
from ..robot.robot import OutOfRobotReachException

_ANGLE_MSG = 'Forward Kinematics exception, robot joints angles limits are (-2pi, 2pi)'


class ForwardKinematics:
    """Robotic arm forward kinematics (forward.py:11-19)."""

    def __init__(self, dh_matrix):
        assert all(len(x) == len(dh_matrix[0]) for x in dh_matrix)
        self.dh_matrix = dh_matrix
        self.thetas, self.epsilons, self.ais, self.alphas = self.dh_matrix
        self.no_of_features = len(self.thetas)
        assert self.no_of_features >= 3
        if self.no_of_features != 4:
            raise NotImplementedError('the HIP FK kernel implements 4-joint DH chains')

    def _ctx(self):
        """The process context with this object's DH table; the link lengths and
        workspace limits it holds (another object's) are left as they are."""
        ctx = _native.context()
        ctx.set_robot(np.asarray(self.dh_matrix, np.float64))
        return ctx

    def fkine(self, angles):
        """(end transform, [all four cumulative transforms]) for one angle vector."""
        self.thetas = angles
        _, mats, st = self._ctx().fk(np.asarray([angles], np.float64), with_mats=True)
        if st.first_err >= 0:
            raise OutOfRobotReachException(_ANGLE_MSG)
        ms = [mats[0, k].copy() for k in range(4)]
        return ms[-1], ms

    def fkine_batch(self, angles) -> np.ndarray:
        """Effector positions (n x 3 float64) of n angle vectors."""
        xyz, _, st = self._ctx().fk(angles)
        if st.first_err >= 0:
            raise OutOfRobotReachException(_ANGLE_MSG)
        return xyz
