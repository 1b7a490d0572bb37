"""GPU parity: libikhip (HIP, gfx950) against the CPU oracle and the reference's
golden fixtures.  Tolerances (north_star: 1e-5 absolute on angles, bit-exact
FABRIK iteration counts) are written next to each assert; where the kernels do
better than the contract the tighter bound is asserted too.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

NS_TOL = 1e-5  # north_star angle tolerance (float), absolute


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="module", params=[1, 0, 2], ids=["split", "simple", "split_refill1"])
def ctx(request):
    from inversekinematicsann_amd import _native
    os.environ["IKHIP_FABRIK_VARIANT"] = str(request.param)
    c = _native.Context(0)
    os.environ.pop("IKHIP_FABRIK_VARIANT", None)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx1():
    from inversekinematicsann_amd import _native
    c = _native.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", ["fabrik_random_dist_tol1e-3.npz",
                                  "fabrik_random_dist_tol1e-5_it200.npz",
                                  "fabrik_uniform_box.npz", "fabrik_spring20.npz"])
def test_fabrik_vs_reference_golden(ctx, name):
    g = _load(name)
    ang, it, jo, st = ctx.fabrik_solve(g["points"], float(g["tol"]), int(g["max_iter"]),
                                       want_joints=True)
    assert st.first_oob == -1 and st.first_err == -1
    assert np.array_equal(it, g["iters"])                       # bit-exact counts
    assert np.abs(ang - g["angles"]).max() <= NS_TOL            # contract
    assert np.abs(ang - g["angles"]).max() <= 1e-9              # achieved
    assert np.abs(jo - g["joints"]).max() <= 1e-9
    assert st.sum_iters == int(g["iters"].sum())
    assert st.max_iters == int(g["iters"].max())
    assert st.n_capped == int((g["iters"] >= int(g["max_iter"])).sum())


def test_fabrik_vs_oracle_random(ctx):
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(50_000, seed=3)
    for tol, mi in ((1e-3, 100), (1e-5, 200)):
        ang, it, jo, st = ctx.fabrik_solve(pts, tol, mi, want_joints=True)
        rang, rit, rjo, rst = O.fabrik_ikine(pts, tol, mi)
        assert np.array_equal(it, rit)
        assert np.abs(ang - rang).max() <= 1e-9
        assert np.abs(jo - rjo).max() <= 1e-9


def test_fabrik_vs_oracle_tight_tolerances(ctx):
    """Deeper convergence than the BASELINE configs (tol 1e-7 / 300 and 1e-9 / 400):
    more iterations per goal, errors near the band's width (D ~ 1e-12), and the
    closed-form seed's last-bit difference from the reference's chain given the most
    iterations to show: iteration counts still bit-exact with the C oracle, angles
    and joints within 1e-9, on random_dist and uniform-box goals."""
    from inversekinematicsann_amd.robot.position_generator import random_dist
    rng = np.random.default_rng(17)
    pts = np.concatenate([random_dist(12_000, seed=17),
                          rng.uniform([0.0, -6.0, -3.0], [6.0, 6.0, 6.0], size=(4_000, 3))])
    for tol, mi in ((1e-7, 300), (1e-9, 400)):
        ang, it, jo, st = ctx.fabrik_solve(pts, tol, mi, want_joints=True)
        rang, rit, rjo, rst = O.fabrik_ikine(pts, tol, mi)
        assert np.array_equal(it, rit), (tol, int((it != rit).sum()))
        for a_, r_ in ((ang, rang), (jo, rjo)):  # (NaN where the reference raises)
            a_, r_ = np.asarray(a_).reshape(len(pts), -1), np.asarray(r_).reshape(len(pts), -1)
            assert np.array_equal(np.isnan(a_), np.isnan(r_))
            ok = ~np.isnan(r_)
            assert np.abs(a_[ok] - r_[ok]).max() <= 1e-9


def test_fabrik_tol_zero_and_negative():
    """tol = 0 (and tols whose threshold rounds to 0, or below it) is accepted by
    the reference (fabrik.py:57: the loop then stops only where both errors are
    exactly 0, i.e. on an exact fixed point of the chain).  The kernels' error
    band must decide nothing there: the band-deciding kernel (split,
    CORE 2) gives the same iteration counts and the same bits as the kernel that
    compares every error exactly (simple), on every point.  Against the oracle the
    counts cannot be bit-exact at tol 0 alone: whether a chain lands on an exact
    fixed point depends on every bit of its trajectory, and the closed-form seed
    (Rz(theta_1) P_k) differs from the reference's chain in the last
    bits of x / y; so there
    the angles are checked (<= 1e-9) and the points whose counts differ must be
    few and must have converged in one of the two runs."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(20_000, seed=11)
    ctxs = {}
    try:
        for name, v in (("simple", 0), ("split", 1)):
            os.environ["IKHIP_FABRIK_VARIANT"] = str(v)
            ctxs[name] = _native.Context(0)
        os.environ.pop("IKHIP_FABRIK_VARIANT", None)
        for tol, mi in ((0.0, 100), (1e-300, 100), (-1.0, 5)):
            out = {k: c.fabrik_solve(pts, tol, mi, want_joints=True) for k, c in ctxs.items()}
            (a0, i0, j0, _), (a1, i1, j1, _) = out["simple"], out["split"]
            assert np.array_equal(i0, i1), (tol, int((i0 != i1).sum()))
            assert np.array_equal(a0, a1, equal_nan=True) and np.array_equal(j0, j1)
            rang, rit, rjo, rst = O.fabrik_ikine(pts, tol, mi)
            assert np.abs(a1 - rang).max() <= 1e-9, tol
            assert np.abs(j1 - rjo).max() <= 1e-9, tol
            bad = i1 != rit
            assert bad.sum() <= 0.01 * len(pts), (tol, int(bad.sum()))
            assert ((i1[bad] < mi) | (rit[bad] < mi)).all(), tol
            if tol < 0:
                assert (i1 == mi).all() and (rit == mi).all()
    finally:
        os.environ.pop("IKHIP_FABRIK_VARIANT", None)
        for c in ctxs.values():
            c.close()


def test_fabrik_ragged_sizes(ctx):
    from inversekinematicsann_amd.robot.position_generator import random_dist
    for n in (1, 63, 64, 65, 255, 257, 1000, 4097):
        pts = random_dist(n, seed=n)
        ang, it, _, st = ctx.fabrik_solve(pts, 1e-3, 100)
        rang, rit, _, _ = O.fabrik_ikine(pts, 1e-3, 100)
        assert np.array_equal(it, rit), n
        assert np.abs(ang - rang).max() <= 1e-9, n
    ang, it, _, st = ctx.fabrik_solve(np.zeros((0, 3)), 1e-3, 100)
    assert ang.shape == (0, 4)


def test_fabrik_fk_err_equals_standalone_fk(ctx):
    """The --verbose round trip (cli.py:54-72) fused into the FABRIK launch equals
    |FK(theta) - p| from the standalone FK kernel on the same angles (1e-12),
    and its batch stats are the reductions of the per-point errors."""
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(20_000, seed=17)
    pts[5] = (0.0, 0.0, 2.0)  # ZeroDivisionError: NaN error, left out of the stats
    for tol, mi in ((1e-3, 100), (1e-5, 200)):
        ang, it, err, st = ctx.fabrik_solve_fk(pts, tol, mi)
        ang2, it2, _, _ = ctx.fabrik_solve(pts, tol, mi)
        assert np.array_equal(ang, ang2, equal_nan=True) and np.array_equal(it, it2)
        assert st.first_err == 5 and st.first_err_code == 3 and math.isnan(err[5])
        ok = np.ones(len(pts), bool)
        ok[5] = False
        xyz, _, _ = ctx.fk(ang[ok])
        ref = np.sqrt(((xyz - pts[ok]) ** 2).sum(axis=1))
        assert np.abs(err[ok] - ref).max() <= 1e-12
        assert st.max_fk_err == err[ok].max()
        assert abs(st.sum_fk_err - err[ok].sum()) <= 1e-9 * max(1.0, err[ok].sum())


def test_fabrik_zero_iteration_solves(ctx):
    """tol >= 1 (the loop's initial errors of 1.0 pass) and max_iter = 0 return the
    seed pose's angles with 0 iterations, as the reference does (fabrik.py:53-59)."""
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(3000, seed=21)
    for tol, mi in ((1.0, 100), (5.0, 100), (1e-3, 0)):
        ang, it, _, st = ctx.fabrik_solve(pts, tol, mi)
        rang, rit, _, _ = O.fabrik_ikine(pts, tol, mi)
        assert np.array_equal(it, rit) and not it.any()
        assert np.abs(ang - rang).max() <= 1e-9


def test_fabrik_edge_cases_and_errors(ctx):
    with open(os.path.join(GOLDEN, "fabrik_edge.json")) as f:
        d = json.load(f)
    for rec in d["edge"]:
        p = np.array([rec["point"]])
        ang, it, _, st = ctx.fabrik_solve(p, 1e-3, 100)
        exc = rec["exception"]
        if exc == "OutOfRobotReachException":
            assert st.first_oob == 0
        elif exc == "ZeroDivisionError":
            assert st.first_err == 0 and st.first_err_code == 3
        elif exc == "ValueError":
            assert st.first_err == 0 and st.first_err_code == 2
        else:
            assert st.first_err == -1 and st.first_oob == -1
            assert it[0] == rec["iters"]
            assert np.abs(ang[0] - np.array(rec["angles"])).max() <= 1e-9


def test_fabrik_error_precedence(ctx):
    # a ZeroDivision point (index 1) before an out-of-reach point (index 2):
    # the reference checks limits for the whole batch first.
    pts = np.array([[1.0, 2.0, 3.0], [0.0, 0.0, 2.0], [1.0, 2.1, -3.123], [1.0, 2.0, 7.0]])
    _, _, _, st = ctx.fabrik_solve(pts, 1e-3, 100)
    assert st.first_oob == 2
    _, _, _, st = ctx.fabrik_solve(pts[:2], 1e-3, 100)
    assert st.first_oob == -1 and st.first_err == 1 and st.first_err_code == 3


def test_fabrik_api_dropin():
    """kinematics.inverse-style usage, mirroring tests/inverse_unit.py:15-34."""
    from inversekinematicsann_amd.kinematics.inverse import FabrikInverseKinematics
    from inversekinematicsann_amd.robot.robot import SixDOFRobot, OutOfRobotReachException
    robot = SixDOFRobot()
    dh = [list(r) for r in robot.dh_matrix]
    ik = FabrikInverseKinematics(dh, robot.links_lengths, robot.effector_workspace_limits)
    points = [[1.0, 2.1, 3.0], [1.567, 2.22, -2.123], [1.02, 3.33, 4.99]]
    output = [[1.1263771168937977, 1.95663870779144, -1.581170282866297, -1.2914981807424972],
              [0.9561510602151175, -0.1334947854494175, -1.441291844752837,
               0.38467252287989595],
              [1.2735640189772053, 1.4953811089376177, -0.6880936114216039, -1.03376967052818]]
    predicted = ik.ikine(points)
    assert isinstance(predicted, list) and isinstance(predicted[0][0], float)
    np.testing.assert_almost_equal(predicted, output, decimal=6)
    with open(os.path.join(GOLDEN, "fabrik_edge.json")) as f:
        d = json.load(f)
    assert dh[0][0] == math.atan2(3.33, 1.02)  # last point's theta_1
    with pytest.raises(OutOfRobotReachException) as ei:
        ik.ikine(d["batch"])
    assert str(ei.value) == d["batch_exception"]["message"]
    with pytest.raises(ZeroDivisionError):
        ik.ikine([[1.0, 2.0, 3.0], [0.0, 0.0, 2.0]])


def test_fabrik_calc_generic_chain(ctx1):
    g = _load("fabrik_calc_5joint.npz")
    out, it, st = ctx1.fabrik_calc(g["links"], g["init"], g["goals"], float(g["tol"]),
                                   int(g["max_iter"]))
    assert np.array_equal(it, g["iters"])
    assert np.abs(out - g["joints"]).max() <= 1e-9


@pytest.mark.parametrize("nj", [1, 9, 13, 24])
def test_fabrik_calc_any_length(ctx1, nj):
    """fabrik_calc_any_kernel (chains outside the unrolled 2..8 joints) against the
    reference's outputs (make_golden_chains.py) and the oracle: bit-exact iteration
    counts; joints within 1e-9 (the kernels square with v * v where CPython's
    pow(v, 2) differs in the last ulp on ~0.1 % of inputs, DESIGN.md "Numerics")."""
    g = _load("fabrik_calc_chains.npz")
    links, init, goals = g[f"links_{nj}"], g[f"init_{nj}"], g[f"goals_{nj}"]
    out, it, st = ctx1.fabrik_calc(links, init, goals, float(g["tol"]), int(g["max_iter"]))
    assert st.first_err == -1
    assert np.array_equal(it, g[f"iters_{nj}"])
    assert np.abs(out - g[f"joints_{nj}"]).max() <= 1e-9
    # one init chain shared by every goal (init_shared), against the oracle
    out2, it2, _ = ctx1.fabrik_calc(links, init[0], goals, 1e-3, 60)
    rout, rit, rst = O.fabrik_calc(np.broadcast_to(init[0], init.shape), goals, links, 1e-3, 60)
    assert np.array_equal(it2, rit) and np.abs(out2 - rout).max() <= 1e-9


def test_fabrik_calc_longest_chain(ctx1):
    """the documented upper length (4096 joints, ikhip.h) runs in
    well under a second for a handful of goals at 100 iterations and matches the
    oracle (bit-exact iteration counts, joints within 1e-9); 4097 joints are refused
    with IK_E_BADARG instead of becoming a multi-second kernel."""
    import time
    from inversekinematicsann_amd import _native
    nj = 4096
    links = np.full(nj, 0.01)
    init = np.zeros((nj, 3))
    init[:, 2] = np.arange(nj) * 0.01
    goals = np.array([[5.0, 3.0, 20.0], [-4.0, 2.0, 30.0], [0.5, 0.5, 40.0], [30.0, 0.0, 1.0]])
    t0 = time.perf_counter()
    out, it, st = ctx1.fabrik_calc(links, init, goals, 1e-3, 100)
    secs = time.perf_counter() - t0
    rout, rit, rst = O.fabrik_calc(np.broadcast_to(init, (len(goals), nj, 3)), goals, links,
                                   1e-3, 100)
    assert st.first_err == -1 and (rst == O.OK).all()
    assert np.array_equal(it, rit) and it.max() > 1
    assert np.abs(out - rout).max() <= 1e-9
    assert secs < 5.0, secs
    with pytest.raises(_native.NativeError) as ei:
        ctx1.fabrik_calc(np.full(nj + 1, 0.01), np.zeros((nj + 1, 3)), goals[:1], 1e-3, 10)
    assert ei.value.code == _native.IK_E_BADARG


def test_fabrik_calc_any_length_zero_division(ctx1):
    """A zero-length segment raises ZeroDivisionError in the reference
    (point.py:40-43): a goal on the chain's second-to-last joint makes the first
    backward step's |goal - joint| zero.  Status IK_E_ZERODIV at the lowest failing
    goal (index 1 here: goal 0 is an ordinary one)."""
    nj = 10
    links = np.full(nj, 0.5)
    init = np.zeros((nj, 3))
    init[:, 2] = np.arange(nj) * 0.5
    goals = np.array([[0.2, 0.1, 2.0], init[nj - 2], init[nj - 2]])
    _, _, st = ctx1.fabrik_calc(links, init, goals, 1e-3, 100)
    _, _, rst = O.fabrik_calc(np.broadcast_to(init, (3, nj, 3)), goals, links, 1e-3, 100)
    assert rst[0] == O.OK and rst[1] == O.E_ZERODIV and rst[2] == O.E_ZERODIV
    assert st.first_err == 1 and st.first_err_code == 3


def test_fabrik_calculate_dropin():
    """tests/fabrik_unit.py:17-41 through the GPU Fabrik class."""
    from inversekinematicsann_amd.kinematics.fabrik import Fabrik
    from inversekinematicsann_amd.kinematics.forward import ForwardKinematics
    from inversekinematicsann_amd.kinematics.point import Point
    from inversekinematicsann_amd.robot.robot import SixDOFRobot
    robot = SixDOFRobot()
    fab = Fabrik(robot.links_lengths)
    fk = ForwardKinematics([list(r) for r in robot.dh_matrix])
    _, fkall = fk.fkine([0, math.pi / 2, 0, 0])
    start = [Point([m[0, 3], m[1, 3], m[2, 3]]) for m in fkall]
    calc = fab.calculate(start, [1, 2, 3])
    np.testing.assert_array_almost_equal(
        calc[3], [1.0000000035582093, 2.0000000071394073, 2.999999989135574])
    with pytest.raises(ValueError):
        fab.calculate(start[:3], [1, 2, 3])


def test_fk_vs_reference_golden(ctx1):
    g = _load("fk_random.npz")
    xyz, mats, st = ctx1.fk(g["angles"], with_mats=True)
    assert st.first_err == -1
    assert np.abs(xyz - g["joints"][:, 3]).max() <= 1e-12
    assert np.abs(mats[:, :, :3, 3] - g["joints"]).max() <= 1e-12
    # forward_unit.py:18-31
    dest = [[1.34542, 2.99821, 3.67401], [0.01333, -3.72111, -1.09902],
            [3.95444, -1.00112, 1.00378]]
    angs = [[1.1489898108341745, 1.6426609377538854, -1.2027772444264693, -1.0663073873609727],
            [-1.5672140776862065, 0.2433182869870163, -1.3760689820099818, 0.0465569704233757],
            [-0.24795388218721454, 0.9644220067435634, -1.5389903144536021,
             -0.3143083371860276]]
    xyz, _, _ = ctx1.fk(np.array(angs))
    np.testing.assert_array_almost_equal(xyz, dest, decimal=4)
    _, _, st = ctx1.fk(np.array([[0.0, 0.0, 0.0, 0.0], [7.0, 0, 0, 0]]))
    assert st.first_err == 1 and st.first_err_code == 4


# ------------------------------------------------------------------ ANN ----
def _ann_case(ctx, dims, acts_hidden, n, seed, check_limits=False, fk=False):
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    from inversekinematicsann_amd.robot.position_generator import random_dist
    m = glorot_model(dims=dims, seed=seed, hidden_act=acts_hidden)
    rng = np.random.default_rng(seed)
    for b in m.biases:
        b[:] = rng.normal(0, 0.1, b.shape).astype(np.float32)
    ctx.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    pts = random_dist(n, seed=seed)
    ang, err, st = ctx.ann_solve(pts, check_limits=check_limits, want_fk_err=fk)
    ref64 = O.ann_forward(pts, m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean,
                          YS.scale, compute=np.float64)
    return m, pts, ang, err, st, ref64


@pytest.mark.parametrize("dims,act", [
    ((3,) + (500,) * 12 + (4,), "tanh"),       # the reference architecture, ann.py:46-56
    ((3, 64, 4), "tanh"),
    ((3, 100, 37, 250, 4), "tanh"),             # ragged widths: every NR path
    ((3, 512, 512, 4), "relu"),
    ((3, 96, 96, 4), "sigmoid"),
    ((3, 4), "linear"),
    # full-width layers whose K is padded to 64 past what the layer before wrote
    ((3, 450, 500, 4), "tanh"),
    ((3, 70, 512, 4), "sigmoid"),
    # wider than 512: the wide build (1028-float LDS rows, 32-point tiles)
    ((3, 1024, 1024, 4), "tanh"),
    ((3, 768, 500, 4), "tanh"),
    ((3, 600, 1000, 37, 4), "relu"),
    # past the fused kernel's caps (> 24 layers, or wider than 1024): the layered
    # path (ik_ann_big.hip), activations through HBM
    ((3, 2048, 2048, 4), "tanh"),
    ((3,) + (64,) * 29 + (4,), "tanh"),         # 30 layers
    ((3, 1100, 37, 4), "relu"),
    ((3,) + (40,) * 25 + (4,), "sigmoid"),
])
def test_ann_vs_oracle(ctx1, dims, act):
    n = 4099  # not a multiple of the 64-point tile
    m, pts, ang, _, st, ref64 = _ann_case(ctx1, dims, act, n, seed=len(dims))
    assert ang.dtype == np.float32 and ang.shape == (n, 4)
    d = np.abs(ang.astype(np.float64) - ref64).max()
    assert d <= NS_TOL, d  # north_star: 1e-5 absolute


def test_ann_layered_chunks_and_stats(ctx1, monkeypatch):
    """The layered path over many chunks (a 1 MiB activation budget: 128-row
    chunks of a 1100-wide model) equals one chunk bit for bit, and its limits
    check and FK round-trip stats match the fused kernel's semantics."""
    dims = (3, 1100, 4)
    _, pts, ang1, err1, st1, ref64 = _ann_case(ctx1, dims, "tanh", 5000, seed=8,
                                               check_limits=True, fk=True)
    monkeypatch.setenv("IKHIP_ANN_ACT_MB", "1")
    ang2, err2, st2 = ctx1.ann_solve(pts, check_limits=True, want_fk_err=True)
    assert np.array_equal(ang1, ang2) and np.array_equal(err1, err2)
    assert np.abs(ang2.astype(np.float64) - ref64).max() <= NS_TOL
    assert st2.first_oob == st1.first_oob
    assert st2.max_fk_err == err2.max()
    assert abs(st2.sum_fk_err - err2.sum()) <= 1e-9 * err2.sum()
    xyz, _, _ = ctx1.fk(ang2.astype(np.float64))
    assert np.abs(err2 - np.sqrt(((xyz - pts) ** 2).sum(axis=1))).max() <= 1e-9
    bad = pts.copy()
    bad[77] = (0.0, 0.0, 50.0)
    _, _, st3 = ctx1.ann_solve(bad, check_limits=True)
    assert st3.first_oob == 77


@pytest.mark.parametrize("hidden", [True, False])
def test_ann_tanh_accuracy(ctx1, hidden):
    """The kernels' tanh (1 - 2 / (1 + exp2(2 log2(e) v)), hardware exp2 and
    reciprocal) against float64 tanh: absolute error <= 3e-7 (2.5 fp32 ulps at
    |tanh| in [0.5, 1)) over [-12, 12], exact +-1 in saturation, for the hidden-layer
    epilogue (3 -> 32 tanh -> 4 linear, identity weights) and the 4-wide output layer
    (3 -> 4 tanh).  Scalers are the identity, so the outputs are tanh(f32(p))."""
    rng = np.random.default_rng(3)
    n = 20_000
    pts = np.concatenate([rng.uniform(-12, 12, (n, 3)), rng.uniform(-1e-3, 1e-3, (2000, 3)),
                          np.array([[0.0, -0.0, 30.0], [1e30, -1e30, 9.1], [-9.1, 1e-30, 1.0]])])
    if hidden:
        W1 = np.zeros((3, 32), np.float32)
        W1[0, 0] = W1[1, 1] = W1[2, 2] = 1.0
        W2 = np.zeros((32, 4), np.float32)
        W2[0, 0] = W2[1, 1] = W2[2, 2] = 1.0
        Ws, bs, acts = [W1, W2], [np.zeros(32, np.float32), np.zeros(4, np.float32)], \
            ["tanh", "linear"]
    else:
        W = np.zeros((3, 4), np.float32)
        W[0, 0] = W[1, 1] = W[2, 2] = 1.0
        Ws, bs, acts = [W], [np.zeros(4, np.float32)], ["tanh"]
    ctx1.ann_load(Ws, bs, acts, np.zeros(3), np.ones(3), np.zeros(4), np.ones(4))
    ang, _, _ = ctx1.ann_solve(pts, check_limits=False)
    ref = np.tanh(pts.astype(np.float32).astype(np.float64))
    err = np.abs(ang[:, :3].astype(np.float64) - ref)
    assert err.max() <= 3e-7, float(err.max())
    big = np.abs(pts) >= 9.1
    assert np.array_equal(ang[:, :3][big], np.sign(pts[big]).astype(np.float32))


@pytest.mark.parametrize("hidden", [True, False])
def test_ann_sigmoid_accuracy(ctx1, hidden):
    """The kernels' sigmoid (1 / (1 + exp2(-log2(e) v)), hardware exp2 and
    reciprocal) against float64: absolute error <= 2e-7 everywhere over [-90, 90];
    relative error <= 4 fp32 ulps (4.8e-7) plus the exponent argument's own fp32
    rounding, which exp2 turns into a relative error of up to |v| log2(e) 2^-24 ln 2
    (bounded here by 9e-8 |v|), wherever the value is >= 1e-30; exactly 0.5 at 0 and 1
    in saturation.  Same identity-weight models as the tanh test."""
    rng = np.random.default_rng(5)
    n = 20_000
    pts = np.concatenate([rng.uniform(-90, 90, (n, 3)), rng.uniform(-20, 20, (n, 3)),
                          np.array([[0.0, -0.0, 200.0], [-200.0, 1e-30, 17.0]])])
    if hidden:
        W1 = np.zeros((3, 32), np.float32)
        W1[0, 0] = W1[1, 1] = W1[2, 2] = 1.0
        W2 = np.zeros((32, 4), np.float32)
        W2[0, 0] = W2[1, 1] = W2[2, 2] = 1.0
        Ws, bs, acts = [W1, W2], [np.zeros(32, np.float32), np.zeros(4, np.float32)], \
            ["sigmoid", "linear"]
    else:
        W = np.zeros((3, 4), np.float32)
        W[0, 0] = W[1, 1] = W[2, 2] = 1.0
        Ws, bs, acts = [W], [np.zeros(4, np.float32)], ["sigmoid"]
    ctx1.ann_load(Ws, bs, acts, np.zeros(3), np.ones(3), np.zeros(4), np.ones(4))
    ang, _, _ = ctx1.ann_solve(pts, check_limits=False)
    x = pts.astype(np.float32).astype(np.float64)
    ref = 1.0 / (1.0 + np.exp(-x))
    got = ang[:, :3].astype(np.float64)
    assert np.abs(got - ref).max() <= 2e-7, float(np.abs(got - ref).max())
    big = ref >= 1e-30
    rel = np.abs(got[big] - ref[big]) / ref[big]
    bound = 4.8e-7 + 9e-8 * np.abs(x[big])
    assert np.all(rel <= bound), float((rel / bound).max())
    assert got[pts[:, :3] == 0.0].tolist() == [0.5] * int((pts[:, :3] == 0.0).sum())
    assert np.all(got[pts[:, :3] >= 200.0] == 1.0)


def test_ann_width_cap(ctx1):
    """ik_ann_load takes widths up to 16384 (past 1024 through the layered path)
    and refuses only wider layers."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    m = glorot_model(dims=(3, 16385, 4), seed=1)
    with pytest.raises(_native.NativeError, match="1..16384"):
        ctx1.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    for w in (1024, 1025, 16384):
        m = glorot_model(dims=(3, w, 4), seed=1)
        ctx1.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)


@pytest.mark.parametrize("mode", ["bf16x6", "fp16x3"])
@pytest.mark.parametrize("dims,act", [
    ((3,) + (500,) * 12 + (4,), "tanh"),
    ((3, 100, 37, 250, 4), "tanh"),             # ragged: K not a multiple of 16, NR 1..4
    ((3, 512, 512, 4), "relu"),                 # fp16x3: unbounded input -> fp32 layer
    ((3, 96, 96, 4), "sigmoid"),
    ((3, 64, 32, 64, 4), "tanh"),               # a split-K (32-wide) layer feeds a split one
    # the layered path (annb_gemm_x6_kernel; fp16x3 runs bf16x6 there)
    ((3, 2048, 2048, 4), "tanh"),
    ((3,) + (64,) * 29 + (4,), "tanh"),
    ((3, 1100, 200, 37, 4), "relu"),            # partial 128-feature tiles, K of 1120 / 224
])
def test_ann_split_modes(ctx1, dims, act, mode):
    """IK_ANN_BF16X6 / IK_ANN_FP16X3: split hidden GEMMs stay within the
    north_star 1e-5 and within a small factor of the fp32 mode's own distance to
    a float64 forward."""
    n = 4099
    try:
        ctx1.ann_set_mode(mode)
        assert ctx1.ann_mode() == mode
        _, pts, ang_x, _, _, ref64 = _ann_case(ctx1, dims, act, n, seed=len(dims))
    finally:
        ctx1.ann_set_mode("fp32")
    ang_f, _, _ = ctx1.ann_solve(pts, check_limits=False)
    d_x = np.abs(ang_x.astype(np.float64) - ref64).max()
    d_f = np.abs(ang_f.astype(np.float64) - ref64).max()
    print(f"{mode} {dims[:3]}.. {act}: max|d| {d_x:.3e} (fp32 mode {d_f:.3e})")
    assert d_x <= NS_TOL, d_x             # north_star: 1e-5 absolute
    assert d_x <= 4 * d_f + 2e-7, (d_x, d_f)


def test_ann_layered_bf16x6_kernel_runs(ctx1):
    """In a split mode the layered path's hidden layers after the first run the
    bf16x6 GEMM (annb_gemm_x6_kernel) and the first / output layers the fp32 one;
    in fp32 mode only the fp32 one runs."""
    dims = (3, 1100, 300, 4)
    names = {}
    for mode in ("fp32", "bf16x6"):
        try:
            ctx1.ann_set_mode(mode)
            ctx1.set_timing(True)
            _ann_case(ctx1, dims, "tanh", 1000, seed=2)
            names[mode] = [k for k, _ in ctx1.kernel_times()]
        finally:
            ctx1.set_timing(False)
            ctx1.ann_set_mode("fp32")
    assert names["fp32"].count("annb_gemm_kernel") == 3
    assert "annb_gemm_x6_kernel" not in names["fp32"]
    assert names["bf16x6"].count("annb_gemm_x6_kernel") == 1
    assert names["bf16x6"].count("annb_gemm_kernel") == 2


def test_ann_layered_bf16x6_chunks(ctx1, monkeypatch):
    """bf16x6 through the layered path over many chunks (a 1 MiB activation budget;
    the activation buffers hold fp32 rows, which annb_gemm_x6_kernel splits into
    three bf16 parts in LDS as it stages them) equals one chunk bit for bit and
    stays within 1e-5 of a float64 forward."""
    dims = (3, 1100, 300, 200, 4)
    try:
        ctx1.ann_set_mode("bf16x6")
        _, pts, ang1, _, _, ref64 = _ann_case(ctx1, dims, "tanh", 3000, seed=9)
        monkeypatch.setenv("IKHIP_ANN_ACT_MB", "1")
        ang2, _, _ = ctx1.ann_solve(pts, check_limits=False)
    finally:
        ctx1.ann_set_mode("fp32")
    assert np.array_equal(ang1, ang2)
    assert np.abs(ang2.astype(np.float64) - ref64).max() <= NS_TOL


def test_ann_fp16x3_layer_mix(ctx1):
    """fp16x3 on a model whose layers switch between the split GEMM (input bounded:
    after tanh / sigmoid) and fp32 (after relu / linear, or 32-wide split-K layers),
    so the activations go out as split fp16 planes exactly where the next layer reads
    them that way: within 1e-5 of a float64 forward and of the fp32 mode's distance."""
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    from inversekinematicsann_amd.robot.position_generator import random_dist
    dims = (3, 200, 160, 32, 96, 128, 64, 4)
    m = glorot_model(dims=dims, seed=31)
    m.activations[:] = ["tanh", "relu", "tanh", "sigmoid", "linear", "tanh", "linear"]
    rng = np.random.default_rng(31)
    for b in m.biases:
        b[:] = rng.normal(0, 0.1, b.shape).astype(np.float32)
    pts = random_dist(3001, seed=31)
    ref64 = O.ann_forward(pts, m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean,
                          YS.scale, compute=np.float64)
    ctx1.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    try:
        ctx1.ann_set_mode("fp16x3")
        ang_x, _, _ = ctx1.ann_solve(pts, check_limits=False)
    finally:
        ctx1.ann_set_mode("fp32")
    ang_f, _, _ = ctx1.ann_solve(pts, check_limits=False)
    d_x = np.abs(ang_x.astype(np.float64) - ref64).max()
    d_f = np.abs(ang_f.astype(np.float64) - ref64).max()
    assert d_x <= NS_TOL, d_x
    assert d_x <= 4 * d_f + 2e-7, (d_x, d_f)


def test_ann_fk_roundtrip_and_limits(ctx1):
    dims = (3, 128, 128, 4)
    m, pts, ang, err, st, ref64 = _ann_case(ctx1, dims, "tanh", 2000, seed=9, fk=True)
    xyz = O.fk_closed_form(ang.astype(np.float64))
    ref_err = np.linalg.norm(xyz - pts, axis=1)
    assert np.abs(err - ref_err).max() <= 1e-9
    assert st.max_fk_err == pytest.approx(ref_err.max(), rel=1e-12)
    assert st.sum_fk_err == pytest.approx(ref_err.sum(), rel=1e-9)
    bad = pts.copy()
    bad[777, 2] = -3.5
    bad[1500, 0] = 6.01
    _, _, st = ctx1.ann_solve(bad, check_limits=True)
    assert st.first_oob == 777


def test_ann_dropin_api():
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER, \
        REFERENCE_Y_SCALER
    from inversekinematicsann_amd.kinematics.inverse import AnnInverseKinematics
    from inversekinematicsann_amd.robot.robot import SixDOFRobot, OutOfRobotReachException
    robot = SixDOFRobot()
    ik = AnnInverseKinematics(robot.dh_matrix, robot.links_lengths,
                              robot.effector_workspace_limits)
    m = glorot_model(dims=(3, 50, 50, 4), seed=2)
    ik.ann.set_model(m, REFERENCE_X_SCALER, REFERENCE_Y_SCALER)
    pts = [[1.0, 2.1, 3.0], [1.567, 2.22, -2.123], [1.02, 3.33, 4.99]]
    out = ik.ikine(pts)
    ref = O.ann_forward(pts, m.weights, m.biases, m.activations, REFERENCE_X_SCALER.mean,
                        REFERENCE_X_SCALER.scale, REFERENCE_Y_SCALER.mean,
                        REFERENCE_Y_SCALER.scale)
    assert np.abs(np.array(out) - ref).max() <= NS_TOL
    assert all(float(np.float32(v)) == v for row in out for v in row)  # fp32 values
    with pytest.raises(OutOfRobotReachException):
        ik.ikine([[1.0, 2.1, 3.0], [1.567, 2.22, -3.123], [1.02, 3.33, 4.99]])
    # ANN.predict has no limit check (ann_unit.py:40 uses an out-of-box point)
    p = ik.ann.predict([[-1.567, 2.22, -3.123]])
    assert p.shape == (1, 4) and p.dtype == np.float32


def test_fabrik_work_order_is_invisible():
    """The hard-first work order (ik_fabrik.hip "Work order") only changes which
    point a lane takes when: results are bit-identical from call to call while
    the cost table learns, across batch sizes with different histogram segment
    counts, and iteration counts stay equal to the oracle's."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    c = _native.Context(0)
    try:
        big = random_dist(60_000, seed=5)
        first = None
        for n in (60_000, 9_000, 60_000, 300, 60_000):
            ang, it, _, _ = c.fabrik_solve(big[:n], 1e-3, 100)
            if n == 60_000:
                if first is None:
                    first = (ang.copy(), it.copy())
                else:
                    assert np.array_equal(ang, first[0], equal_nan=True)
                    assert np.array_equal(it, first[1])
        # a forgotten table (ik_fabrik_reset_order: the built-in one again) and an
        # empty one (point order) change nothing
        c.fabrik_reset_order()
        ang, it, _, _ = c.fabrik_solve(big, 1e-3, 100)
        assert np.array_equal(ang, first[0], equal_nan=True) and np.array_equal(it, first[1])
        c.fabrik_order_set(None)
        ang, it, _, _ = c.fabrik_solve(big, 1e-3, 100)
        assert np.array_equal(ang, first[0], equal_nan=True) and np.array_equal(it, first[1])
        ref_ang, ref_it, _, _ = O.fabrik_ikine(big[:8192], 1e-3, 100)
        assert np.array_equal(first[1][:8192], ref_it)  # bit-exact iteration counts
        assert np.abs(first[0][:8192] - ref_ang).max() <= 1e-9
    finally:
        c.close()


def test_fabrik_prior_gate_first_call_other_distributions():
    """a fresh context's first call on a batch the built-in table
    was not learned on (uniform workspace box, a spring trajectory; most goals in
    cells the prior has never seen) keeps the empty table's order (the scatter's
    gate, ik_fabrik.hip) -- and, gated or not, the results are the oracle's bit for
    bit in the counts, identical to an empty-table solve, and the call teaches
    the table as usual."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist, spring
    rng = np.random.default_rng(5)
    box = np.stack([rng.uniform(0, 6, 40_000), rng.uniform(-6, 6, 40_000),
                    rng.uniform(-3, 6, 40_000)], axis=1)
    for pts in (box, spring(40_000, 2, 3, 6), random_dist(40_000, seed=6)):
        c = _native.Context(0)
        try:
            prior = c.fabrik_order_get().copy()
            ang, it, _, _ = c.fabrik_solve(pts, 1e-3, 100)
            assert not np.array_equal(c.fabrik_order_get(), prior)  # learned
            c.fabrik_order_set(None)
            ang2, it2, _, _ = c.fabrik_solve(pts, 1e-3, 100)
            assert np.array_equal(it, it2) and np.array_equal(ang, ang2, equal_nan=True)
            rang, rit, _, _ = O.fabrik_ikine(pts[:8192], 1e-3, 100)
            assert np.array_equal(it[:8192], rit)
            assert np.array_equal(np.isnan(ang[:8192]), np.isnan(rang))
            assert np.nanmax(np.abs(ang[:8192] - rang)) <= 1e-9
        finally:
            c.close()


def test_fabrik_builtin_work_order_table():
    """a fresh context of SixDOFRobot's chain starts from the
    library's built-in cost table (the tol 1e-3 / 100 one); its first solve at
    tol 1e-5 / 200 swaps in that tolerance's table before it learns; reset
    restores the built-in one; another chain starts empty (point order) and
    going back to SixDOFRobot's restores the built-in table."""
    import json
    import os
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "r04", "fabrik_prior_tables.json")) as f:
        tabs = {k: np.array(v, np.uint32) for k, v in json.load(f)["tables"].items()}
    c = _native.Context(0)
    try:
        assert np.array_equal(c.fabrik_order_get(), tabs["0.001/100"])
        pts = random_dist(300, seed=8)
        c.fabrik_solve(pts, 1e-5, 200)
        t = c.fabrik_order_get()  # the 1e-5 table with this call's records folded in
        assert np.all(t >= tabs["1e-05/200"] - (tabs["1e-05/200"] >> 3))
        assert not np.array_equal(t, tabs["0.001/100"])
        c.fabrik_reset_order()
        assert np.array_equal(c.fabrik_order_get(), tabs["0.001/100"])
        c.fabrik_order_set(None)
        assert not c.fabrik_order_get().any()
        c.set_robot(np.array([[0.0, np.pi / 2, 0, 0], [2, 0, 0, 0], [0, 2, 2, 1.5],
                              [np.pi / 2, 0, 0, 0]]), links=[2, 2, 2, 1.5])
        assert not c.fabrik_order_get().any()
        c.set_robot(np.array([[0.0, np.pi / 2, 0, 0], [2, 0, 0, 0], [0, 2, 2, 2],
                              [np.pi / 2, 0, 0, 0]]), links=[2, 2, 2, 2])
        assert np.array_equal(c.fabrik_order_get(), tabs["0.001/100"])
    finally:
        c.close()


def test_device_pointer_path(ctx1):
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(10_000, seed=21)
    dpts = torch.from_numpy(pts).cuda()
    dang = torch.empty((10_000, 4), dtype=torch.float64, device="cuda")
    dit = torch.empty(10_000, dtype=torch.int32, device="cuda")
    ctx1.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx1.fabrik_solve_device(dpts, dang, dit, None, 1e-3, 100,
                             flags=_native.IK_F_DEVICE | _native.IK_F_ASYNC)
    st = ctx1.stats_fetch()
    ctx1.set_stream(None)
    rang, rit, _, _ = O.fabrik_ikine(pts)
    assert np.array_equal(dit.cpu().numpy(), rit)
    assert np.abs(dang.cpu().numpy() - rang).max() <= 1e-9
    assert st.sum_iters == int(rit.sum())


def test_fabrik_core_sequences_bit_identical():
    """The iteration kernel's sqrt_core / div_core path (ik_common.h), alone (1) and
    with the repeated distances taken once (2, fabrik_step4_reuse), claims the
    same bits as the general sqrt / division wherever its domain check passes,
    and falls back per wave elsewhere: final joints and iteration counts of the
    two paths are compared bit for bit on reachable, unreachable (capped),
    near-singular and degenerate goals.  Path 2 also decides the loop condition
    from the step's radicands through the launch's error band (fabrik_step4_lazy):
    goals past the band's reach (exact comparisons) and tolerances of 1e-11 and
    2e-12, where many errors fall inside the band, are in the set."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    rng = np.random.default_rng(11)
    box = rng.uniform([0.0, -6.0, -3.0], [6.0, 6.0, 6.0], size=(100_000, 3))
    near = np.array([0.0, 0.0, 2.0]) + rng.normal(0.0, 1e-6, size=(2_000, 3))
    near[:, 0] = np.abs(near[:, 0])
    far = rng.normal(0.0, 1.0, size=(3_000, 3)) * rng.choice([50.0, 700.0, 1e3, 1e5], (3_000, 1))
    pts = np.concatenate([random_dist(200_000, seed=12), box, near, far,
                          [[0.0, 0.0, 2.0], [1e-300, 0.0, 2.0], [0.0, 0.0, 4.0]]])
    out = {}
    for core in ("0", "1", "2"):
        os.environ["IKHIP_FABRIK_CORE"] = core
        c = _native.Context(0)
        os.environ.pop("IKHIP_FABRIK_CORE", None)
        try:
            out[core] = [c.fabrik_solve(pts, tol, mi, want_joints=True)
                         for tol, mi in ((1e-3, 100), (1e-5, 200), (1e-11, 60), (2e-12, 60))]
        finally:
            c.close()
    pairs = list(zip(out["0"], out["1"])) + list(zip(out["0"], out["2"]))
    for (a0, i0, j0, s0), (a1, i1, j1, s1) in pairs:
        assert np.array_equal(i0, i1)
        assert np.array_equal(j0.view(np.uint64), j1.view(np.uint64))
        assert np.array_equal(a0.view(np.uint64), a1.view(np.uint64))
        assert (s0.first_oob, s0.first_err, s0.first_err_code) == \
            (s1.first_oob, s1.first_err, s1.first_err_code)


@pytest.mark.parametrize("links", [(2.0, 2.0, 2.0, 2.5),     # L2 != L3: no carried distance
                                   (2.5, 2.0, 2.0, 2.0),     # L0 != L1: no shared distance
                                   (1.5, 1.5, 2.5, 2.5),     # both equal pairs, not 2
                                   (1.7, 1.7, 1.7, 1.7),     # equal, not 2: converges
                                   (0.7, 1.9, 1.3, 2.2)])    # nothing shared
def test_fabrik_custom_links_match_oracle(links):
    """FABRIK ikine with joints_distances other than the robot's [2, 2, 2, 2]
    (InverseKinematics takes them separately from the DH table, inverse.py:20):
    every iteration path the library picks from the links (distance reuse when
    L0 == L1 and L2 == L3, the plain core sequences otherwise) gives the oracle's
    iteration counts bit for bit, its angles to 1e-9 and its first error.  With
    unequal links the reference never converges (its backward pass uses links
    0-2 and its forward pass links 1-3, fabrik.py:24,37), so those cases run every
    point to the iteration cap."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(20_000, seed=21)
    links = np.array(links, dtype=np.float64)
    c = _native.Context(0)
    try:
        c.set_robot(O.DH, links, O.LIMITS)
        for tol, mi in ((1e-3, 100), (1e-5, 200)):
            for _ in range(2):  # the second call runs in the learned work order
                ang, it, _, st = c.fabrik_solve(pts, tol, mi)
            rang, rit, _, rst = O.fabrik_ikine(pts, tol, mi, links=links)
            ok = rst == 0
            assert ok.sum() > len(pts) // 2
            assert np.array_equal(it[ok], rit[ok]), int((it[ok] != rit[ok]).sum())
            assert np.abs(ang[ok] - rang[ok]).max() <= 1e-9
            bad = np.nonzero(~ok)[0]
            want = (int(bad[0]), int(rst[bad[0]])) if len(bad) else (-1, 0)
            assert (st.first_err, st.first_err_code) == want
    finally:
        c.close()


def test_fk_full_angle_range_vs_oracle():
    """The FK kernel's closed-form DH matrices and range-limited sincos over the
    whole legal angle range [-2 pi, 2 pi] (forward.py:23-25), its edges, and a few
    out-of-range angles (IK_E_ANGLE_RANGE at the first one): effector positions
    within 1e-12 of the oracle's DH-product restatement, with a custom DH table too."""
    rng = np.random.default_rng(31)
    ang = rng.uniform(-2 * math.pi, 2 * math.pi, size=(200_000, 4))
    ang[:8] = [[2 * math.pi] * 4, [-2 * math.pi] * 4, [0.0] * 4, [math.pi / 2] * 4,
               [-math.pi / 2] * 4, [math.pi] * 4, [1e-300, -1e-300, 5e-324, 0.0],
               [math.pi / 4, 3 * math.pi / 4, -3 * math.pi / 4, 7 * math.pi / 4]]
    from inversekinematicsann_amd import _native
    c = _native.Context(0)
    for dh in (O.DH, np.array([[0.3, -1.1, 0.2, 0.0], [1.5, 0.25, 0.0, -0.5],
                               [0.0, 1.7, 2.3, 0.9], [math.pi / 2, -0.4, 0.0, 1.2]])):
        c.set_robot(dh, O.LINKS, O.LIMITS)
        xyz, _, st = c.fk(ang)
        rxyz, _, rst = O.fk(ang, dh=dh)
        assert st.first_err == -1 and not rst.any()
        assert np.abs(xyz - rxyz).max() <= 1e-12
    c.set_robot(O.DH, O.LINKS, O.LIMITS)
    bad = ang[:100].copy()
    bad[37, 2] = 2 * math.pi + 1e-9
    bad[60, 0] = -7.0
    xyz, _, st = c.fk(bad)
    assert (st.first_err, st.first_err_code) == (37, 4)
    assert np.isnan(xyz[37]).all() and np.isnan(xyz[60]).all()
    rxyz, _, _ = O.fk(bad)
    ok = np.ones(100, bool)
    ok[[37, 60]] = False
    assert np.abs(xyz[ok] - rxyz[ok]).max() <= 1e-12
    c.close()


def test_robot_state_per_object_interleaved():
    """Objects with different robots interleave on the one process context:
    FABRIK with custom links, then fkine of another object, then FABRIK again --
    every result equals the oracle for its own robot, and fkine leaves the links
    and limits alone (it uploads only its DH table)."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.forward import ForwardKinematics
    from inversekinematicsann_amd.kinematics.inverse import FabrikInverseKinematics
    from inversekinematicsann_amd.robot.position_generator import random_dist
    from inversekinematicsann_amd.robot.robot import SixDOFRobot
    robot = SixDOFRobot()
    dh = [list(r) for r in robot.dh_matrix]
    links = [2.0, 2.0, 2.5, 2.5]
    lim = robot.effector_workspace_limits
    pts = random_dist(2000, seed=31)
    ik_a = FabrikInverseKinematics([list(r) for r in dh], links, lim)
    ik_b = FabrikInverseKinematics([list(r) for r in dh], robot.links_lengths, lim)
    ra, rit_a, _, _ = O.fabrik_ikine(pts, 1e-3, 100, links=np.array(links))
    rb, rit_b, _, _ = O.fabrik_ikine(pts, 1e-3, 100)
    a1 = np.array(ik_a.ikine(pts))
    m4, _ = ForwardKinematics([list(r) for r in dh]).fkine([0.1, 0.2, 0.3, 0.4])
    rxyz, _, _ = O.fk(np.array([[0.1, 0.2, 0.3, 0.4]]))
    assert np.abs(m4[:3, 3] - rxyz[0]).max() <= 1e-12
    a2 = np.array(ik_a.ikine(pts))  # the links must still be ik_a's
    b1 = np.array(ik_b.ikine(pts))
    a3 = np.array(ik_a.ikine(pts))
    for got, ref in ((a1, ra), (a2, ra), (b1, rb), (a3, ra)):
        assert np.abs(got - ref).max() <= 1e-9
    assert np.array_equal(ik_a.last_iterations, rit_a)
    assert np.array_equal(ik_b.last_iterations, rit_b)
    ctx = _native.context()
    n0 = ctx.robot_uploads
    ik_a.ikine(pts)
    ik_a.ikine(pts)  # the context holds ik_a's robot (dh[0][0] moves, unread): no upload
    assert ctx.robot_uploads == n0
    ik_b.ikine(pts)
    assert ctx.robot_uploads == n0 + 1


def test_cli_call_uploads_the_robot_at_most_once():
    """A 20-point CLI call (cli.py --inverse-kine --method fabrik) makes at most one
    ik_set_robot in the process (none when the context already holds the robot)."""
    import subprocess
    import sys
    code = ("import sys; sys.argv=['ik_cli','--inverse-kine','--method','fabrik','--points',"
            f"{os.path.join(GOLDEN, 'cli_spring20_points.csv')!r},'--verbose'];"
            "from inversekinematicsann_amd.cli import main; rc=main(sys.argv[1:]);"
            "from inversekinematicsann_amd import _native;"
            "print('UPLOADS', _native.context().robot_uploads)")
    from tests.conftest import ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=120, cwd=ROOT)
    line = [l for l in out.stdout.splitlines() if l.startswith("UPLOADS")]
    assert line, out.stdout + out.stderr
    assert int(line[0].split()[1]) <= 1


@pytest.mark.parametrize("mode", ["fp32", "bf16x6", "fp16x3"])
def test_ann_tile_variants_agree(ctx1, tmp_path, mode):
    """fp32 runs 32-point tiles by default (MR = 1), the split modes 64 (MR = 2);
    IKHIP_ANN_MR forces either.  The other tile size, in a fresh process, gives
    the same bits (per point the same K order and the same fixed split-K sum) --
    for fp16x3 also through the 16x16x32 sub-tiles of a 32-point tile."""
    import subprocess
    import sys
    from tests.conftest import ROOT
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    from inversekinematicsann_amd.robot.position_generator import random_dist
    dims = (3, 200, 300, 4)
    m = glorot_model(dims=dims, seed=9)
    pts = random_dist(5000, seed=9)
    ctx1.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    ctx1.ann_set_mode(mode)
    try:
        mine, err, _ = ctx1.ann_solve(pts, want_fk_err=True)
    finally:
        ctx1.ann_set_mode("fp32")
    out = tmp_path / "other.npz"
    code = (
        "import numpy as np\n"
        "from inversekinematicsann_amd import _native\n"
        "from inversekinematicsann_amd.kinematics.ann import glorot_model, "
        "REFERENCE_X_SCALER as XS, REFERENCE_Y_SCALER as YS\n"
        "from inversekinematicsann_amd.robot.position_generator import random_dist\n"
        f"m = glorot_model(dims={dims!r}, seed=9); pts = random_dist(5000, seed=9)\n"
        "c = _native.Context(0)\n"
        "c.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)\n"
        f"c.ann_set_mode({mode!r})\n"
        "a, e, _ = c.ann_solve(pts, want_fk_err=True)\n"
        f"np.savez({str(out)!r}, a=a, e=e)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=120,
                       env=dict(os.environ, IKHIP_ANN_MR="2" if mode == "fp32" else "1"))
    assert r.returncode == 0, r.stderr[-2000:]
    other = np.load(out)
    assert np.array_equal(mine, other["a"]) and np.array_equal(err, other["e"])


@pytest.mark.parametrize("nj", [5, 6, 8, 9, 13])
def test_fk_chains_of_other_lengths(nj):
    """ForwardKinematics accepts any number of features >= 3 (forward.py:13-19):
    5..8-joint DH tables (unrolled kernels) and 9 / 13 joints (the run-time joint
    loop, fk_any_kernel) on the GPU (ik_fk_chain) against the numpy restatement
    of forward.py's nf x nf matrices (oracle.fk_n), and 3 features fail like
    the reference (IndexError, after the angle check)."""
    from inversekinematicsann_amd.kinematics.forward import ForwardKinematics
    from inversekinematicsann_amd.robot.robot import OutOfRobotReachException
    rng = np.random.default_rng(nj)
    dh = np.vstack([np.zeros(nj), rng.uniform(0, 2, nj), rng.uniform(0, 2, nj),
                    rng.uniform(-np.pi, np.pi, nj)])
    fk = ForwardKinematics([list(r) for r in dh])
    angs = rng.uniform(-np.pi, np.pi, (64, nj))
    xyz = fk.fkine_batch(angs)
    for a, p in zip(angs[:8], xyz[:8]):
        end, mats = fk.fkine(list(a))
        ref = O.fk_n(dh, a)
        assert len(mats) == nj and end.shape == (nj, nj)
        for m, r in zip(mats, ref):
            assert np.abs(m - r).max() <= 1e-12
        assert np.abs(p - ref[-1][:3, 3]).max() <= 1e-12
    bad = angs[0].copy()
    bad[nj - 1] = 7.0
    with pytest.raises(OutOfRobotReachException):
        fk.fkine(list(bad))
    fk3 = ForwardKinematics([[0.0, 0.0, 0.0], [2.0, 0.0, 0.0], [0.0, 2.0, 2.0],
                             [np.pi / 2, 0.0, 0.0]])
    with pytest.raises(IndexError, match="index 3 is out of bounds"):
        fk3.fkine([0.1, 0.2, 0.3])
    with pytest.raises(OutOfRobotReachException):
        fk3.fkine([7.0, 0.2, 0.3])


def test_pinned_host_pipeline_equals_device_path(ctx1):
    """Host arrays in pinned memory (ik_host_alloc) take the chunked copy / solve /
    copy pipeline: the same bits as the one-shot pageable path, and the stats of
    the chunks merge with global indices (an out-of-reach point and a
    ZeroDivisionError point in different chunks)."""
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd.kinematics.ann import glorot_model, REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    from inversekinematicsann_amd.robot.position_generator import random_dist
    n = 300_001  # 2 chunks, ragged
    pts = random_dist(n, seed=41)
    pts[200_123] = (0.0, 0.0, 2.0)    # ZeroDivisionError, chunk 1
    pts[250_000] = (1.0, 2.0, -3.5)   # out of reach, chunk 1
    pts[70_000] = (0.0, 0.0, 2.0)     # ZeroDivisionError, chunk 0
    pp = _native.pinned_empty((n, 3))
    pp[:] = pts
    ang = _native.pinned_empty((n, 4))
    it = _native.pinned_empty((n,), np.int32)
    err = _native.pinned_empty((n,), np.float64)
    s = _native.IkStats()
    import ctypes
    rc = ctx1.lib.ik_fabrik_solve_fk(ctx1.handle, pp.ctypes.data, n, 1e-3, 100, ang.ctypes.data,
                                     it.ctypes.data, None, err.ctypes.data, 0, ctypes.byref(s))
    assert rc == 0
    r_ang, r_it, r_err, r_st = ctx1.fabrik_solve_fk(pts, 1e-3, 100)  # pageable: one shot
    assert np.array_equal(ang, r_ang, equal_nan=True) and np.array_equal(it, r_it)
    assert np.array_equal(err, r_err, equal_nan=True)
    for k in ("first_oob", "first_err", "first_err_code", "max_iters", "sum_iters", "n_capped",
              "max_fk_err"):
        assert getattr(s, k) == getattr(r_st, k), k
    assert (s.first_oob, s.first_err) == (250_000, 70_000)
    m = glorot_model(dims=(3, 64, 64, 4), seed=4)  # ANN on pinned arrays: one shot
    ctx1.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)
    fa = _native.pinned_empty((n, 4), np.float32)
    rc = ctx1.lib.ik_ann_solve(ctx1.handle, pp.ctypes.data, n, fa.ctypes.data, err.ctypes.data,
                               0, ctypes.byref(s))
    assert rc == 0
    r_a, r_e, r_s = ctx1.ann_solve(pts, want_fk_err=True)
    assert np.array_equal(fa, r_a) and np.array_equal(err, r_e, equal_nan=True)
    assert s.first_oob == r_s.first_oob == 250_000


def test_device_tensors_from_pending_torch_ops():
    """Points produced by a torch kernel still in flight: the device wrappers run
    the library on torch's current stream, so the solve reads finished inputs;
    a float32 / non-contiguous / wrong-shape tensor is refused, not misread."""
    import torch
    from inversekinematicsann_amd import _native
    ctx = _native.Context(0)
    n = 200_000
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        base = torch.rand((n, 3), generator=g, dtype=torch.float64, device="cuda")
        pts = base * torch.tensor([1.5, 2.0, 2.0], dtype=torch.float64, device="cuda") \
            + torch.tensor([0.2, -1.0, 0.5], dtype=torch.float64, device="cuda")
        for _ in range(20):  # keep the stream busy so a racing solve would read zeros
            pts = pts * 1.0
        ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
        it = torch.empty(n, dtype=torch.int32, device="cuda")
        st = ctx.fabrik_solve_device(pts, ang, it, None, 1e-3, 100)
        host = pts.cpu().numpy()
    ref, rit, _, _ = ctx.fabrik_solve(host, 1e-3, 100)
    assert np.array_equal(ang.cpu().numpy(), ref, equal_nan=True)
    assert np.array_equal(it.cpu().numpy(), rit) and st.sum_iters == int(rit.sum())
    with pytest.raises(ValueError, match="dtype"):
        ctx.fabrik_solve_device(pts.float(), ang)
    with pytest.raises(ValueError, match="contiguous"):
        ctx.fabrik_solve_device(pts.t().contiguous().t(), ang)
    with pytest.raises(ValueError, match="shape"):
        ctx.fabrik_solve_device(pts, ang[:10])
    ctx.close()
