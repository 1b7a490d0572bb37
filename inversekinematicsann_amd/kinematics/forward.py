"""Forward kinematics on the GPU -- kinematics/forward.py of the reference.

ForwardKinematics(dh).fkine(angles) returns (M_4, [M_1, M_2, M_3, M_4]) like
the reference (forward.py:73-94), computed by libikhip's fk kernel (one point
per lane, float64 DH chain).  fkine_batch(angles) is the batched entry point
(effector xyz n x 3), used for the CLI's --verbose round trip (cli.py:54-61).
"""
from __future__ import annotations

from math import pi

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
        if self.no_of_features > 1024:
            raise NotImplementedError('the HIP FK kernels take DH chains of 3 to 1024 joints')

    def _ctx(self):
        """The process context with this object's DH table; the link lengths and
        workspace limits it holds (another object's) are left as they are."""
        ctx = _native.context()
        ctx.set_robot(np.asarray(self.dh_matrix, np.float64))
        return ctx

    def _three_features(self, angles):
        # forward.py with 3 features: __rotation_matrix checks the angle, then
        # returns the axis name (its matrix is already 3 x 3, :42-43), and
        # __translation_matrix writes column 3 of a 3 x 3 identity (:56-59)
        if angles[0] < -2 * pi or angles[0] > 2 * pi:
            raise OutOfRobotReachException(_ANGLE_MSG)
        raise IndexError('index 3 is out of bounds for axis 1 with size 3')

    def fkine(self, angles):
        """(end transform, [all cumulative transforms]) for one angle vector:
        no_of_features x no_of_features matrices, as the reference builds them."""
        self.thetas = angles
        nf = self.no_of_features
        if nf == 3:
            self._three_features(angles)
        if nf == 4:
            _, mats, st = self._ctx().fk(np.asarray([angles], np.float64), with_mats=True)
        else:
            _, mats, st = _native.context().fk_chain(np.asarray(self.dh_matrix, np.float64),
                                                     np.asarray([angles], np.float64),
                                                     with_mats=True)
        if st.first_err >= 0:
            raise OutOfRobotReachException(_ANGLE_MSG)
        ms = []
        for k in range(nf):
            m = np.identity(nf)
            m[:4, :4] = mats[0, k]  # the 4 x 4 DH block; the rest is the identity
            ms.append(m)
        return ms[-1], ms

    def fkine_batch(self, angles) -> np.ndarray:
        """Effector positions (n x 3 float64) of n angle vectors."""
        nf = self.no_of_features
        if nf == 4:
            xyz, _, st = self._ctx().fk(angles)
        else:
            a = np.asarray(angles, np.float64).reshape(-1, nf)
            if nf == 3 and len(a):
                self._three_features(a[0])
            xyz, _, st = _native.context().fk_chain(np.asarray(self.dh_matrix, np.float64), a)
        if st.first_err >= 0:
            raise OutOfRobotReachException(_ANGLE_MSG)
        return xyz
