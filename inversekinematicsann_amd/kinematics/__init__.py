"""kinematics package mirroring the reference's kinematics/ modules."""
