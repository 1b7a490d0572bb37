"""Pin the CPU oracle (oracle/ik_oracle.c) to the reference's own outputs.

The fixtures were produced by importing the reference (tests/golden/make_golden.py);
the reference's unit-test goldens are restated inline below with their file:line.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("name", ["fabrik_random_dist_tol1e-3.npz",
                                  "fabrik_random_dist_tol1e-5_it200.npz",
                                  "fabrik_uniform_box.npz", "fabrik_spring20.npz"])
def test_oracle_fabrik_ikine_bit_exact(name):
    g = _load(name)
    ang, it, jo, st = O.fabrik_ikine(g["points"], float(g["tol"]), int(g["max_iter"]))
    assert np.array_equal(st, g["status"])
    assert np.array_equal(it, g["iters"])
    assert np.array_equal(ang, g["angles"])  # bit-exact (same glibc, same op order)
    assert np.array_equal(jo, g["joints"])


def test_oracle_fk_bit_exact():
    g = _load("fk_random.npz")
    xyz, jo, st = O.fk(g["angles"])
    assert (st == 0).all()
    assert np.array_equal(jo, g["joints"])
    assert np.array_equal(xyz, g["joints"][:, 3])


def test_oracle_fk_angle_range():
    with open(os.path.join(GOLDEN, "fk_exceptions.json")) as f:
        exc = json.load(f)
    for ang, name, _msg in exc:
        _, _, st = O.fk(np.array([ang], np.float64))
        assert (st[0] == O.E_ANGLE_RANGE) == (name == "OutOfRobotReachException")


def test_oracle_fabrik_calc_generic_chain():
    g = _load("fabrik_calc_5joint.npz")
    out, it, st = O.fabrik_calc(g["init"], g["goals"], g["links"], float(g["tol"]),
                                int(g["max_iter"]))
    assert (st == 0).all()
    assert np.array_equal(it, g["iters"])
    assert np.array_equal(out, g["joints"])


@pytest.mark.parametrize("nj", [1, 9, 13, 24])
def test_oracle_fabrik_calc_any_length(nj):
    """Chains outside 2..8 joints (make_golden_chains.py: the reference's own
    outputs), bit-exact: fabrik.py:44-67 takes any len(init) == len(dists)."""
    g = _load("fabrik_calc_chains.npz")
    out, it, st = O.fabrik_calc(g[f"init_{nj}"], g[f"goals_{nj}"], g[f"links_{nj}"],
                                float(g["tol"]), int(g["max_iter"]))
    assert (st == 0).all()
    assert np.array_equal(it, g[f"iters_{nj}"])
    assert np.array_equal(out, g[f"joints_{nj}"])


def test_oracle_round8():
    g = _load("round8.npz")
    r = np.array([O.round_nd(v, 8) for v in g["v"]])
    assert np.array_equal(r.view(np.uint64), g["r"].view(np.uint64))


def test_oracle_edge_cases():
    with open(os.path.join(GOLDEN, "fabrik_edge.json")) as f:
        d = json.load(f)
    for rec in d["edge"]:
        p = np.array([rec["point"]], np.float64)
        bad = O.check_limits(p)
        if rec["exception"] == "OutOfRobotReachException":
            assert bad == 0
            continue
        assert bad == -1
        ang, it, _, st = O.fabrik_ikine(p)
        if rec["exception"] == "ZeroDivisionError":
            assert st[0] == O.E_ZERODIV
        elif rec["exception"] == "ValueError":
            assert st[0] == O.E_DOMAIN
        else:
            assert st[0] == 0
            assert it[0] == rec["iters"]
            assert np.array_equal(ang[0], np.array(rec["angles"]))


# Reference unit-test goldens, restated as data.
def test_reference_unit_goldens():
    # tests/inverse_unit.py:23-28
    pts = [[1.0, 2.1, 3.0], [1.567, 2.22, -2.123], [1.02, 3.33, 4.99]]
    out = [[1.1263771168937977, 1.95663870779144, -1.581170282866297, -1.2914981807424972],
           [0.9561510602151175, -0.1334947854494175, -1.441291844752837, 0.38467252287989595],
           [1.2735640189772053, 1.4953811089376177, -0.6880936114216039, -1.03376967052818]]
    ang, _, _, st = O.fabrik_ikine(np.array(pts))
    assert (st == 0).all()
    np.testing.assert_almost_equal(ang, out, decimal=6)
    # tests/inverse_unit.py:32-34: z = -3.123 < -3 is out of reach, first bad index 1
    assert O.check_limits(np.array([[1.0, 2.1, 3.0], [1.567, 2.22, -3.123],
                                    [1.02, 3.33, 4.99]])) == 1
    # tests/fabrik_unit.py:24-35: seed FK([0, pi/2, 0, 0]), goal (1, 2, 3), effector only
    _, seed, _ = O.fk(np.array([[0.0, math.pi / 2, 0.0, 0.0]]))
    jo, _, st = O.fabrik_calc(seed, np.array([[1.0, 2.0, 3.0]]))
    np.testing.assert_array_almost_equal(
        jo[0, 3], [1.0000000035582093, 2.0000000071394073, 2.999999989135574])
    # tests/forward_unit.py:18-31 (4 decimals)
    dest = [[1.34542, 2.99821, 3.67401], [0.01333, -3.72111, -1.09902],
            [3.95444, -1.00112, 1.00378]]
    angs = [[1.1489898108341745, 1.6426609377538854, -1.2027772444264693, -1.0663073873609727],
            [-1.5672140776862065, 0.2433182869870163, -1.3760689820099818, 0.0465569704233757],
            [-0.24795388218721454, 0.9644220067435634, -1.5389903144536021,
             -0.3143083371860276]]
    xyz, _, _ = O.fk(np.array(angs))
    np.testing.assert_array_almost_equal(xyz, dest, decimal=4)
    # tests/point_unit.py:22,34-37: |(0,0,0)-(-2.22,3.123,0.002)| = 3.831649
    assert abs(math.sqrt(2.22 ** 2 + 3.123 ** 2 + 0.002 ** 2) - 3.831649) < 1e-6


def test_oracle_fk_n_pinned_to_reference_fk():
    """oracle.fk_n (forward.py's nf x nf matrices in numpy, the checker of the
    5..8-joint FK kernels) reproduces the reference's own 4-joint FK outputs."""
    g = _load("fk_random.npz")
    for a, jo in zip(g["angles"][:200], g["joints"][:200]):
        mats = O.fk_n(O.DH, a)
        got = np.array([m[:3, 3] for m in mats])
        assert np.abs(got - jo).max() <= 1e-12
