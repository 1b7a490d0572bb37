"""inversekinematicsann_amd -- MI355X-native batched inverse kinematics.

Drop-in for the kinematics.inverse API of lstar93/InverseKinematicsANN
(FabrikInverseKinematics / AnnInverseKinematics .ikine), backed by hand-written
HIP kernels for gfx950 in libikhip.so (see include/ikhip.h).
"""
__version__ = "0.1.0"
