"""Robot constants -- the reference's robot/robot.py:38-46, restated.

SixDOFRobot is a 4-revolute-joint arm (the name is the reference's): DH rows
thetas / d / a / alpha, the inclusive effector workspace box and the four link
lengths.  These are the constants the kernels are parameterised with.
"""
from math import pi


class SixDOFRobot():
    """6 DOF robot math description (robot/robot.py:38-42)."""
    dh_matrix = [[0, pi/2, 0, 0], [2, 0, 0, 0], [0, 2, 2, 2], [pi/2, 0, 0, 0]]
    effector_workspace_limits = {'x': [0, 6], 'y': [-6, 6], 'z': [-3, 6]}
    links_lengths = [2, 2, 2, 2]


class OutOfRobotReachException(Exception):
    """Robot manipulator exception class (robot/robot.py:45-46)."""
