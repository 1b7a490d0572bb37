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
`--generate-data --shape {circle,cube,cube_random,random,spring,random_dist}` runs
the reference's generators (robot/position_generator.py, cli.py:80-229) with the
same arguments: --to-file writes the x,y,z CSV, --verbose prints the shape's
parameters as the reference does (its 3-D plot is out of scope).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

EXAMPLES = {
    "ann": "--inverse-kine --method ann --model model_filename.h5 --points filename.csv",
    "fabrik": "--inverse-kine --method fabrik --points filename.csv",
    "circle": "--generate-data --shape circle --radius 3 --samples 20 --center 1,5,2",
    "cube": "--generate-data --shape cube --step 0.75 --dim 2,3,4 --start 1,2,3",
    "cube_random": "--generate-data --shape cube_random --step 0.75 --dim 2,3,4 --start 1,2,3",
    "random": "--generate-data --shape random --limits 0,3;0,4;0,5 --samples 20",
    "spring": "--generate-data --shape spring --samples 50 --dim 2,3,6",
    "random_dist": "--generate-data --shape random_dist --dist normal --samples 100 "
                   "--std_dev 0.35 --limits 0,3;0,4;0,5",
}
# each shape's required arguments (cli.py:91-94, 117-119, 155-157, 182-184, 206-211)
SHAPE_ARGS = {"circle": ("radius", "samples", "center"), "cube": ("step", "dim", "start"),
              "cube_random": ("step", "dim", "start"), "random": ("samples", "limits"),
              "spring": ("samples", "dim"),
              "random_dist": ("dist", "samples", "std_dev", "limits")}


def _parser():
    p = argparse.ArgumentParser(prog="cli")
    g = p.add_mutually_exclusive_group()
    g.add_argument("--inverse-kine", action="store_true")
    g.add_argument("--generate-data", action="store_true")
    p.add_argument("--method", choices=["ann", "fabrik"])
    p.add_argument("--shape", choices=list(SHAPE_ARGS))
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
    p.add_argument("--dist", type=str, choices=["normal", "uniform", "random"])
    p.add_argument("--std_dev", type=float)
    p.add_argument("--limits", type=str)
    p.add_argument("--radius", type=float)
    p.add_argument("--center", type=str)
    p.add_argument("--step", type=float)
    p.add_argument("--start", type=str)
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


def _floats(text):
    return [float(v) for v in text.split(",")]


def _limits(text):
    lim = text.split(";")
    return {"x": _floats(lim[0]), "y": _floats(lim[1]), "z": _floats(lim[2])}


def _generate(args, parser):
    """cli.py:80-229: the shape's generator on its arguments; --verbose prints the
    arguments tuple (the reference's ShapeCommand.verbose, before its plot),
    --to-file the points as an x,y,z CSV."""
    import pandas as pd
    from .robot import position_generator as G
    if args.shape is None:
        parser.error("the following arguments are required: --shape")
    if args.example:
        print(EXAMPLES[args.shape])
        return 0
    missing = [a for a in SHAPE_ARGS[args.shape] if getattr(args, a) is None]
    if missing:
        parser.error("the following arguments are required: " +
                     ", ".join("--" + a for a in missing))
    sh = args.shape
    if sh == "circle":
        center = _floats(args.center)
        params = (args.radius, args.samples, center)
        pts = G.circle(args.radius, args.samples, center)
    elif sh in ("cube", "cube_random"):
        dim, start = _floats(args.dim), _floats(args.start)
        params = (args.step, dim, start)
        pts = (G.cube if sh == "cube" else G.cube_random)(args.step, *dim, start)
    elif sh == "random":
        lim = _limits(args.limits)
        params = (args.samples, lim)
        pts = G.random(args.samples, lim)
    elif sh == "spring":
        dim = _floats(args.dim)
        params = (args.samples, *dim)
        pts = G.spring(args.samples, *dim)
    else:
        lim = _limits(args.limits)
        params = (args.samples, lim, args.dist, args.std_dev)
        pts = G.random_distribution(args.samples, lim, args.dist, args.std_dev)
    if args.verbose:
        print(params)
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
