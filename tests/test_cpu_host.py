"""CPU-only checks: the C-ABI library loads and exports every symbol declared in
include/ikhip.h; host-side logic (scaler decoding, limits, inputs)."""
import os
import re

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "ikhip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|double|const char \*|void \*)\s*(ik_\w+)\s*\(",
                                 src, re.M)))


def test_header_matches_binding_list():
    from inversekinematicsann_amd import _native
    assert _declared_symbols() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    from inversekinematicsann_amd import _native
    lib = _native.load_library()
    for sym in _declared_symbols():
        assert hasattr(lib, sym), sym
    assert lib.ik_version().decode().startswith("ikhip")


def test_library_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from inversekinematicsann_amd import _native
    with pytest.raises(_native.NativeUnavailable):
        _native.Context(0)


def test_scaler_bin_decoder():
    from inversekinematicsann_amd.kinematics.ann import REFERENCE_X_SCALER, REFERENCE_Y_SCALER
    from inversekinematicsann_amd.models.scaler_bin import load_scaler
    base = os.path.join(GOLDEN, "roboarm_model_1674153800-982793")
    sx = load_scaler(base + "_scaler_x.bin")
    sy = load_scaler(base + "_scaler_y.bin")
    # SURVEY.md 8(a6) values, and scale == sqrt(var)
    assert sx.mean.tolist() == REFERENCE_X_SCALER.mean.tolist()
    assert sx.scale.tolist() == REFERENCE_X_SCALER.scale.tolist()
    assert sy.mean.tolist() == REFERENCE_Y_SCALER.mean.tolist()
    assert sy.scale.tolist() == REFERENCE_Y_SCALER.scale.tolist()
    assert np.array_equal(np.sqrt(sx.var), sx.scale) and np.array_equal(np.sqrt(sy.var), sy.scale)
    assert sx.n_samples_seen == 67000 and sx.sklearn_version == "1.0.2"
    assert sx.with_mean and sx.with_std


def test_scaler_transform_semantics():
    from inversekinematicsann_amd.kinematics.ann import REFERENCE_Y_SCALER as YS
    y = np.array([[0.1, -0.2, 0.3, 0.4]], np.float32)
    out = YS.inverse_transform(y)
    assert out.dtype == np.float32
    exp = (y.astype(np.float64) * YS.scale).astype(np.float32)
    exp = (exp.astype(np.float64) + YS.mean).astype(np.float32)
    assert np.array_equal(out, exp)


def test_limits_array_and_points():
    from inversekinematicsann_amd.kinematics.inverse import as_points, limits_array
    lim = limits_array({'x': [0, 6], 'y': [-6, 6], 'z': [-3, 6]})
    assert lim.tolist() == [0, 6, -6, 6, -3, 6]
    lim2 = limits_array({'x': [0, 1]})
    assert lim2[2] == -np.inf and lim2[5] == np.inf
    p = as_points([[1, 2, 3], [4, 5, 6]])
    assert p.dtype == np.float64 and p.flags.c_contiguous and p.shape == (2, 3)


def test_random_dist_generator():
    from inversekinematicsann_amd.robot.position_generator import random_dist, spring
    p = random_dist(100_000, seed=0)
    assert p.shape == (100_000, 3)
    assert (p[:, 0] >= 0).all() and (p[:, 0] <= 6).all()
    assert (p[:, 2] >= -3).all()
    assert np.array_equal(p, random_dist(100_000, seed=0))
    s = spring(20, 2, 3, 6)
    g = np.load(os.path.join(GOLDEN, "fabrik_spring20.npz"))["points"]
    assert np.array_equal(s, g)


def test_point_helpers():
    """tests/point_unit.py:16-51 against the API helpers."""
    from inversekinematicsann_amd.kinematics.point import (Point, get_distance_between,
                                                           get_point_between)
    p0, p1 = Point([0, 0, 0]), Point([-2.22, 3.123, 0.002])
    with pytest.raises(ValueError):
        Point([0, 0, 0, 1])
    assert [-2.22, 3.123, 0.002] == p1
    np.testing.assert_almost_equal(3.831649, get_distance_between(p0, p1))
    np.testing.assert_almost_equal((np.array(p0) + np.array(p1)) / 2, get_point_between(p0, p1))


def test_points_of_the_wrong_width_raise(tmp_path, capsys):
    """A 4-column CSV (e.g. written with pandas index=True) is not reinterpreted as
    other points: FABRIK raises the reference Point's ValueError (point.py:12-14),
    ANN the StandardScaler's feature-count error, and the CLI prints it and exits 0
    (cli.py:250-252).  Host-side checks: nothing reaches the GPU."""
    import pandas as pd
    from inversekinematicsann_amd.cli import main
    from inversekinematicsann_amd.kinematics.ann import as_features
    from inversekinematicsann_amd.kinematics.inverse import as_points
    with pytest.raises(ValueError, match=r"3D Point input shape should be \(3,\) not \(4,\)"):
        as_points(np.ones((3, 4)))
    with pytest.raises(ValueError, match=r"not \(2,\)"):
        as_points([[1.0, 2.0], [3.0, 4.0]])
    with pytest.raises(ValueError, match="X has 4 features, but StandardScaler is expecting 3"):
        as_features(np.ones((3, 4)))
    assert as_points([]).shape == (0, 3) and as_features([1.0, 2.0, 3.0]).shape == (1, 3)
    csv = tmp_path / "pts4.csv"
    pd.DataFrame([[1.0, 2.0, 3.0], [1.5, 2.5, 3.5], [1.0, 1.0, 1.0]],
                 columns=["x", "y", "z"]).to_csv(csv, index=True)
    rc = main(["--inverse-kine", "--method", "fabrik", "--points", str(csv)])
    assert rc == 0
    assert capsys.readouterr().out.strip() == "3D Point input shape should be (3,) not (4,)"


def test_scaler_flags_reach_the_kernel_constants():
    """with_mean / with_std off: the kernels get mean 0 / scale 1, so the fused
    (x - mean) / scale and y * scale + mean equal sklearn's skipped steps."""
    from inversekinematicsann_amd.models.scaler_bin import ScalerParams
    sp = ScalerParams(mean=np.array([1.0, 2.0, 3.0]), scale=np.array([2.0, 4.0, 8.0]), var=None,
                      with_mean=False, with_std=True)
    m, s = sp.effective()
    assert m.tolist() == [0.0, 0.0, 0.0] and s.tolist() == [2.0, 4.0, 8.0]
    x = np.array([[1.0, 2.0, 3.0]])
    assert np.array_equal((x - m) / s, sp.transform(x))
    sp = ScalerParams(mean=np.array([1.0, 2.0, 3.0]), scale=np.array([2.0, 4.0, 8.0]), var=None,
                      with_mean=True, with_std=False)
    m, s = sp.effective()
    assert m.tolist() == [1.0, 2.0, 3.0] and s.tolist() == [1.0, 1.0, 1.0]
    assert np.array_equal((x - m) / s, sp.transform(x))
