"""Command line front-end -- the reference's `cli.py --inverse-kine` contract.

    python -m inversekinematicsann_amd.cli --inverse-kine --method fabrik --points P.csv \
        [--to-file OUT.csv] [--verbose] [--tol 1e-3] [--max-iter 100]
    python -m inversekinematicsann_amd.cli --inverse-kine --method ann --model M.h5 \
        --points P.csv [--to-file OUT.csv] [--verbose]

Same flags, outputs and error behaviour as cli.py:232-388 of the reference:
the points CSV is read with pandas (header row, x,y,z columns), angles are
written as theta1..theta4 (index=False); OutOfRobotReachException and
ValueError are printed and the command still exits 0 (cli.py:250-252, 300),
a ZeroDivisionError propagates.  Plotting (plot/plot.py) is out of scope:
--verbose prints the angles and the FK round-trip error instead of plotting.
Extra flags: --tol / --max-iter (FABRIK, defaults 1e-3 / 100 as the
reference's constructor) and --device.
`--generate-data` supports the two shapes the benchmarks use (spring,
random_dist normal); the other generators are out of scope.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

EXAMPLES = {
    "ann": "--inverse-kine --method ann --model model_filename.h5 --points filename.csv",
    "fabrik": "--inverse-kine --method fabrik --points filename.csv",
    "spring": "--generate-data --shape spring --samples 50 --dim 2,3,6",
    "random_dist": "--generate-data --shape random_dist --dist normal --samples 100 "
                   "--std_dev 0.35 --limits 0,3;0,4;0,5",
}


def _parser():
    p = argparse.ArgumentParser(prog="cli")
    g = p.add_mutually_exclusive_group()
    g.add_argument("--inverse-kine", action="store_true")
    g.add_argument("--generate-data", action="store_true")
    p.add_argument("--method", choices=["ann", "fabrik"])
    p.add_argument("--shape", choices=["spring", "random_dist"])
    p.add_argument("--example", action="store_true")
    p.add_argument("--points", type=str, help=".csv file name with stored trajectory points")
    p.add_argument("--model", type=str, help="select saved model .h5 (or .npz) filename")
    p.add_argument("--to-file", type=str)
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--show-path", action="store_true")
    p.add_argument("--separate-plots", action="store_true")
    p.add_argument("--tol", type=float, default=0.001, help="FABRIK error margin")
    p.add_argument("--max-iter", type=int, default=100, help="FABRIK iteration cap")
    p.add_argument("--device", type=int, default=None, help="GPU index")
    # data generators
    p.add_argument("--samples", type=int)
    p.add_argument("--dim", type=str)
    p.add_argument("--dist", type=str, choices=["normal"])
    p.add_argument("--std_dev", type=float)
    p.add_argument("--limits", type=str)
    return p


def _read_points(path):
    import pandas as pd
    return pd.read_csv(path).values.tolist()


def _save_angles(data, filename):
    import pandas as pd
    pd.DataFrame(data, columns=['theta1', 'theta2', 'theta3', 'theta4']).to_csv(filename,
                                                                                index=False)


def _verbose(points, joint_angles):
    from .kinematics.forward import ForwardKinematics
    from .robot.robot import SixDOFRobot as Robot
    fk = ForwardKinematics([list(r) for r in Robot.dh_matrix])
    xyz = fk.fkine_batch(np.asarray(joint_angles, np.float64))
    err = np.linalg.norm(xyz - np.asarray(points, np.float64), axis=1)
    print(joint_angles)
    print(f"FK round trip: max |FK(theta) - p| = {err.max():.6g}, mean = {err.mean():.6g} "
          f"over {len(err)} points")


def _ikine(args, parser):
    from .robot.robot import OutOfRobotReachException
    from .robot.robot import SixDOFRobot as Robot
    if args.method is None:
        parser.error("the following arguments are required: --method")
    if args.example:
        print(EXAMPLES[args.method])
        return 0
    if args.points is None:
        parser.error("the following arguments are required: --points")
    if args.method == "ann" and args.model is None:
        parser.error("the following arguments are required: --model")
    from .kinematics.inverse import AnnInverseKinematics, FabrikInverseKinematics
    points = _read_points(args.points)
    dh = [list(r) for r in Robot.dh_matrix]
    if args.method == "ann":
        ik = AnnInverseKinematics(dh, Robot.links_lengths, Robot.effector_workspace_limits)
        ik.load_model(args.model)
    else:
        ik = FabrikInverseKinematics(dh, Robot.links_lengths, Robot.effector_workspace_limits,
                                     args.tol, args.max_iter)
    try:
        joint_angles = ik.ikine(points)
    except (OutOfRobotReachException, ValueError) as kine_exception:
        print(str(kine_exception))
        return 0
    if args.verbose:
        _verbose(points, joint_angles)
    if args.to_file is not None:
        _save_angles(joint_angles, args.to_file)
    return 0


def _generate(args, parser):
    import pandas as pd
    from .robot.position_generator import random_dist, spring
    if args.shape is None:
        parser.error("the following arguments are required: --shape")
    if args.example:
        print(EXAMPLES[args.shape])
        return 0
    if args.shape == "spring":
        if args.samples is None or args.dim is None:
            parser.error("the following arguments are required: --samples, --dim")
        pts = spring(args.samples, *[float(v) for v in args.dim.split(",")])
    else:
        if None in (args.samples, args.std_dev, args.limits, args.dist):
            parser.error("the following arguments are required: --dist, --samples, --std_dev, "
                         "--limits")
        lim = [[float(v) for v in ax.split(",")] for ax in args.limits.split(";")]
        pts = random_dist(args.samples, seed=0, std_dev=args.std_dev,
                          limits={"x": lim[0], "y": lim[1], "z": lim[2]})
    if args.verbose:
        print(pts.tolist())
    if args.to_file is not None:
        pd.DataFrame(pts.tolist(), columns=["x", "y", "z"]).to_csv(args.to_file, index=False)
    return 0


def main(argv=None):
    parser = _parser()
    args = parser.parse_args(sys.argv[1:] if argv is None else argv)
    if args.device is not None:
        os.environ["IKHIP_DEVICE"] = str(args.device)
    if not args.inverse_kine and not args.generate_data:
        parser.error('Operation --inverse-kine or --generate-data must be choosed')
    if args.inverse_kine:
        return _ikine(args, parser)
    return _generate(args, parser)


if __name__ == "__main__":
    sys.exit(main())
