"""Generate the golden fixtures in tests/golden/ by importing the reference.

Run in the build container only (the reference is mounted read-only at
/root/reference and never travels to the GPU box):

    python tests/golden/make_golden.py

The reference's kinematics/inverse.py imports kinematics/ann.py, which imports
keras; keras is not installed, so a stub module with the imported names is put
in sys.modules first (the FABRIK/FK path never touches it).  Iteration counts
are read by wrapping Fabrik's name-mangled __backward (one call per iteration,
fabrik.py:57-60).  Nothing from the reference is copied into the repo: only
inputs and the reference's outputs, as .npz / .json data.
"""
from __future__ import annotations

import json
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    keras = types.ModuleType("keras")
    for sub, names in {"models": ["load_model", "Sequential"], "optimizers": ["Adam"],
                       "layers": ["Dense", "Input"], "callbacks": ["EarlyStopping"]}.items():
        m = types.ModuleType("keras." + sub)
        for n in names:
            setattr(m, n, None)
        sys.modules["keras." + sub] = m
        setattr(keras, sub, m)
    keras.activations = types.SimpleNamespace(tanh=None)
    sys.modules["keras"] = keras
    sys.path.insert(0, REF)
    import kinematics.fabrik as fabrik  # noqa: E402
    import kinematics.forward as forward  # noqa: E402
    import kinematics.inverse as inverse  # noqa: E402
    import robot.position_generator as pg  # noqa: E402
    import robot.robot as robot  # noqa: E402
    return fabrik, forward, inverse, pg, robot


fabrik, forward, inverse, pg, robot = _import_reference()
R = robot.SixDOFRobot

_count = {"n": 0}
_orig_backward = fabrik.Fabrik._Fabrik__backward


def _counting_backward(self, *a, **k):
    _count["n"] += 1
    return _orig_backward(self, *a, **k)


fabrik.Fabrik._Fabrik__backward = _counting_backward


def fresh_dh():
    return [list(r) for r in R.dh_matrix]


def ref_ikine_with_iters(points, tol, max_iter):
    """Reference FabrikInverseKinematics.ikine point by point, recording the
    iteration count and the final FABRIK joint positions of each point."""
    dh = fresh_dh()
    ik = inverse.FabrikInverseKinematics(dh, R.links_lengths, R.effector_workspace_limits,
                                         tol, max_iter)
    fk = forward.ForwardKinematics(dh)
    fab = fabrik.Fabrik(R.links_lengths, tol, max_iter)
    angles, iters, joints, status = [], [], [], []
    for p in points:
        try:
            _count["n"] = 0
            a = ik.ikine([list(p)])[0]
            it = _count["n"]
            # final joint positions: rerun the same seed through Fabrik.calculate
            th = [math.atan2(p[1], p[0])] + dh[0][1:]
            _, fk_all = fk.fkine(th)
            init = [inverse.Point([m[0][3], m[1][3], m[2][3]]) for m in fk_all]
            fin = fab.calculate(init, list(p))
            angles.append(a); iters.append(it); joints.append([list(q) for q in fin])
            status.append(0)
        except ZeroDivisionError:
            angles.append([np.nan] * 4); iters.append(-1); joints.append([[np.nan] * 3] * 4)
            status.append(3)
        except ValueError:
            angles.append([np.nan] * 4); iters.append(-1); joints.append([[np.nan] * 3] * 4)
            status.append(2)
    return (np.array(angles, np.float64), np.array(iters, np.int32),
            np.array(joints, np.float64), np.array(status, np.int32))


def save_fabrik(name, pts, tol, max_iter, note):
    pts = np.ascontiguousarray(np.asarray(pts, np.float64).reshape(-1, 3))
    a, it, jo, st = ref_ikine_with_iters(pts.tolist(), tol, max_iter)
    np.savez_compressed(os.path.join(OUT, name), points=pts, angles=a, iters=it, joints=jo,
                        status=st, tol=np.float64(tol), max_iter=np.int32(max_iter),
                        note=np.array(note))
    print(f"{name}: n={len(pts)} mean iters={it[it >= 0].mean():.2f} "
          f"capped={(it == max_iter).sum()} errors={(st != 0).sum()}")


def main():
    rng_note = "reference TrainingDataGenerator.random_distribution(n, limits, 'normal', 0.5)"
    # 1. random_dist std 0.5, reference generator seeded through numpy/scipy.
    np.random.seed(1234)
    pts = pg.TrainingDataGenerator.random_distribution(4000, R.effector_workspace_limits,
                                                       "normal", 0.5)
    save_fabrik("fabrik_random_dist_tol1e-3.npz", pts, 1e-3, 100, rng_note + " seed 1234")
    np.random.seed(4321)
    pts = pg.TrainingDataGenerator.random_distribution(2000, R.effector_workspace_limits,
                                                       "normal", 0.5)
    save_fabrik("fabrik_random_dist_tol1e-5_it200.npz", pts, 1e-5, 200,
                rng_note + " seed 4321")
    # 2. uniform over the workspace box: ~37% unreachable -> iteration cap.
    rng = np.random.default_rng(7)
    lim = R.effector_workspace_limits
    pts = np.stack([rng.uniform(*lim["x"], 2000), rng.uniform(*lim["y"], 2000),
                    rng.uniform(*lim["z"], 2000)], axis=1)
    save_fabrik("fabrik_uniform_box.npz", pts, 1e-3, 100, "uniform box, numpy default_rng(7)")
    # 3. spring(20, 2, 3, 6) -- the CLI example shape (cli.py:195, position_generator.py:73-78)
    pts = pg.TrainingDataGenerator.spring(20, 2, 3, 6)
    save_fabrik("fabrik_spring20.npz", pts, 1e-3, 100, "spring(20, 2, 3, 6)")

    # 4. edge cases, each through the full reference ikine (limits included).
    edge_pts = [[0.0, 0.0, 0.0], [0.0, 0.0, 4.0], [6.0, 0.0, 2.0], [1e-9, 0.0, 5.0],
                [0.0, 0.0, 2.0], [1.0, 2.1, -3.123], [6.0, 6.0, 6.0], [0.0, -6.0, -3.0],
                [1e-300, 1e-300, 2.0], [2.0, 0.0, 10.0 / 3.0], [8.0 / 3, 0.0, 2.0],
                [0.5, 0.0, 2.0], [4.0, 0.0, 2.0], [1.0, 1.0, 1.0], [5.9, 0.1, 2.0],
                [0.0, 0.0, 8.0 / 1.0 - 1e-12]]
    edge = []
    for p in edge_pts:
        dh = fresh_dh()
        ik = inverse.FabrikInverseKinematics(dh, R.links_lengths, R.effector_workspace_limits)
        rec = {"point": p}
        try:
            _count["n"] = 0
            rec["angles"] = ik.ikine([p])[0]
            rec["iters"] = _count["n"]
            rec["exception"] = None
        except Exception as e:  # noqa: BLE001 -- record the reference's exception
            rec["exception"] = type(e).__name__
            rec["message"] = str(e)
        edge.append(rec)
    # batch error precedence: limits are checked for every point before any solve
    dh = fresh_dh()
    ik = inverse.FabrikInverseKinematics(dh, R.links_lengths, R.effector_workspace_limits)
    batch = [[1.0, 2.0, 3.0], [0.0, 0.0, 2.0], [1.0, 2.1, -3.123], [1.0, 2.0, 7.0]]
    try:
        ik.ikine(batch)
        batch_exc = None
    except Exception as e:  # noqa: BLE001
        batch_exc = {"exception": type(e).__name__, "message": str(e)}
    dh_after = None
    dh = fresh_dh()
    ik = inverse.FabrikInverseKinematics(dh, R.links_lengths, R.effector_workspace_limits)
    ik.ikine([[1.0, 2.0, 3.0], [2.0, -1.0, 1.0]])
    dh_after = dh[0][0]
    with open(os.path.join(OUT, "fabrik_edge.json"), "w") as f:
        json.dump({"edge": edge, "batch": batch, "batch_exception": batch_exc,
                   "dh00_after_ikine": dh_after}, f, indent=1)
    print("fabrik_edge.json:", [(r["point"], r["exception"]) for r in edge if r["exception"]])

    # 5. FK: random angles through ForwardKinematics.fkine, all four joints.
    rng = np.random.default_rng(11)
    ang = rng.uniform(-2 * math.pi, 2 * math.pi, (2000, 4))
    fk = forward.ForwardKinematics(fresh_dh())
    jo = np.array([[m[:3, 3] for m in fk.fkine(list(a))[1]] for a in ang])
    exc = []
    for bad in ([7.0, 0, 0, 0], [0, 0, 0, -6.3], [0, 2 * math.pi, 0, 0]):
        try:
            fk.fkine(bad)
            exc.append([bad, None, None])
        except Exception as e:  # noqa: BLE001
            exc.append([bad, type(e).__name__, str(e)])
    np.savez_compressed(os.path.join(OUT, "fk_random.npz"), angles=ang, joints=jo)
    with open(os.path.join(OUT, "fk_exceptions.json"), "w") as f:
        json.dump(exc, f, indent=1)
    print("fk_random.npz:", jo.shape, "fk exceptions:", exc)

    # 6. Fabrik.calculate with a generic 5-joint chain and unequal links
    #    (pins the dists[:-1] / dists[1:] indexing of fabrik.py:24,37).
    rng = np.random.default_rng(13)
    links5 = [1.0, 1.5, 2.0, 1.0, 0.5]
    n5 = 500
    init5 = np.zeros((n5, 5, 3))
    for k in range(1, 5):
        init5[:, k, 2] = init5[:, k - 1, 2] + links5[k - 1]
    init5[:, 1:, :2] += rng.normal(0, 0.05, (n5, 4, 2))
    goals5 = rng.normal(0, 1.5, (n5, 3)) + np.array([0.0, 0.0, 2.0])
    out5, it5 = [], []
    fab = fabrik.Fabrik(links5, 1e-4, 150)
    for i in range(n5):
        _count["n"] = 0
        r = fab.calculate([inverse.Point(list(q)) for q in init5[i]], list(goals5[i]))
        out5.append([list(q) for q in r]); it5.append(_count["n"])
    np.savez_compressed(os.path.join(OUT, "fabrik_calc_5joint.npz"), links=np.array(links5),
                        init=init5, goals=goals5, joints=np.array(out5),
                        iters=np.array(it5, np.int32), tol=np.float64(1e-4),
                        max_iter=np.int32(150))
    print("fabrik_calc_5joint.npz: mean iters", np.mean(it5))

    # 7. CPython round(v, 8), including values on and around half-way decimals.
    rng = np.random.default_rng(17)
    v = np.concatenate([rng.uniform(-1.2, 1.2, 20000), rng.normal(0, 1e-6, 2000),
                        (np.arange(-3000, 3000) + 0.5) / 1e8,
                        np.nextafter((np.arange(-500, 500) + 0.5) / 1e8, 1),
                        np.nextafter((np.arange(-500, 500) + 0.5) / 1e8, -1),
                        np.array([1 / 512, -1 / 512, 3 / 512, 0.99999999500000, 1.0, -1.0,
                                  0.0, -0.0, 5e-9, -5e-9, 1 - 1e-16])])
    r = np.array([round(float(x), 8) for x in v])
    np.savez_compressed(os.path.join(OUT, "round8.npz"), v=v, r=r)
    print("round8.npz:", v.shape)


if __name__ == "__main__":
    main()


# --------------------------------------------------------------------- CLI ----
_CLI_WRAPPER = r'''
import runpy, sys, types
keras = types.ModuleType("keras")
for sub, names in {"models": ["load_model", "Sequential"], "optimizers": ["Adam"],
                   "layers": ["Dense", "Input"], "callbacks": ["EarlyStopping"]}.items():
    m = types.ModuleType("keras." + sub)
    for n in names:
        setattr(m, n, None)
    sys.modules["keras." + sub] = m
    setattr(keras, sub, m)
keras.activations = types.SimpleNamespace(tanh=None)
sys.modules["keras"] = keras
sys.path.insert(0, "/root/reference")
sys.argv = ["cli.py"] + sys.argv[1:]
runpy.run_path("/root/reference/cli.py", run_name="__main__")
'''


def cli_goldens():
    """Run the reference CLI (FABRIK method) on two CSVs; record stdout, exit
    code and the output CSV text."""
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp()
    wrapper = os.path.join(tmp, "run_ref_cli.py")
    with open(wrapper, "w") as f:
        f.write(_CLI_WRAPPER)
    spring_csv = os.path.join(OUT, "cli_spring20_points.csv")
    oor_csv = os.path.join(OUT, "cli_out_of_reach_points.csv")
    import pandas as pd
    pd.DataFrame(pg.TrainingDataGenerator.spring(20, 2, 3, 6),
                 columns=["x", "y", "z"]).to_csv(spring_csv, index=False)
    pd.DataFrame([[1.0, 2.1, 3.0], [1.567, 2.22, -3.123]],
                 columns=["x", "y", "z"]).to_csv(oor_csv, index=False)
    env = dict(os.environ, MPLBACKEND="Agg")
    rec = {}
    for name, csvp in (("spring20", spring_csv), ("out_of_reach", oor_csv)):
        outp = os.path.join(tmp, name + "_angles.csv")
        r = subprocess.run([sys.executable, wrapper, "--inverse-kine", "--method", "fabrik",
                            "--points", csvp, "--to-file", outp], cwd="/root/reference",
                           env=env, capture_output=True, text=True)
        rec[name] = {"returncode": r.returncode, "stdout": r.stdout,
                     "angles_csv": open(outp).read() if os.path.exists(outp) else None}
    r = subprocess.run([sys.executable, wrapper, "--inverse-kine", "--method", "fabrik",
                        "--example"], cwd="/root/reference", env=env, capture_output=True,
                       text=True)
    rec["example"] = {"returncode": r.returncode, "stdout": r.stdout}
    with open(os.path.join(OUT, "cli_fabrik.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("cli_fabrik.json:", {k: v["returncode"] for k, v in rec.items()})


if __name__ == "__main__" and "--cli" in sys.argv:
    cli_goldens()
