"""Hash of one ANN solve's outputs, for bit-identity checks between library
builds (IKHIP_LIB=... python tools/ann_bitcmp.py MODE): the reference architecture
(3 -> 12 x 500 tanh -> 4, Glorot seed 0) on 65 536 random_dist seed-1 points, plus a
ragged model.  Two builds that claim the same arithmetic print the same lines."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    from inversekinematicsann_amd.robot.position_generator import random_dist
    mode = sys.argv[1] if len(sys.argv) > 1 else "fp16x3"
    ctx = _native.Context(0)
    pts = random_dist(65536, seed=1)
    for dims in ((3,) + (500,) * 12 + (4,), (3, 100, 37, 250, 4), (3, 512, 256, 512, 4)):
        m = glorot_model(dims, seed=len(dims))
        ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
        ctx.ann_set_mode(mode)
        ang, err, _ = ctx.ann_solve(pts, want_fk_err=True, check_limits=False)
        h = hashlib.sha256(ang.tobytes() + err.tobytes()).hexdigest()[:16]
        print(mode, dims[1:-1][:3], len(dims) - 2, h)


if __name__ == "__main__":
    main()
