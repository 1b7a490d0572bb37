"""C-ABI argument checking on a live context (include/ikhip.h): every entry
point refuses bad arguments with IK_E_BADARG / IK_E_NOMODEL and a message in
ik_last_error(), leaves the context usable, and never launches a kernel on a
rejected call.  The Python wrappers surface these as NativeError."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from inversekinematicsann_amd import _native
    c = _native.Context(0)
    yield c
    c.close()


def _rc_msg(ctx, rc):
    return rc, ctx.lib.ik_last_error().decode()


def test_bad_arguments_are_refused(ctx):
    from inversekinematicsann_amd import _native as N
    L, h = ctx.lib, ctx.handle
    st = N.IkStats()
    pts = np.zeros((4, 3))
    ang = np.zeros((4, 4))
    # negative sizes / null pointers
    rc, msg = _rc_msg(ctx, L.ik_fabrik_solve(h, pts.ctypes.data, -1, 1e-3, 100, ang.ctypes.data,
                                             None, None, 0, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG and "ik_fabrik_solve" in msg
    rc, msg = _rc_msg(ctx, L.ik_fabrik_solve(h, None, 4, 1e-3, 100, ang.ctypes.data, None, None,
                                             0, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG
    rc, msg = _rc_msg(ctx, L.ik_fk(h, ang.ctypes.data, 4, None, None, 0, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG and "ik_fk" in msg
    rc, msg = _rc_msg(ctx, L.ik_check_limits(h, None, 3, 0, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG
    # async without device pointers
    rc, msg = _rc_msg(ctx, L.ik_fabrik_solve(h, pts.ctypes.data, 4, 1e-3, 100, ang.ctypes.data,
                                             None, None, N.IK_F_ASYNC, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG and "IK_F_ASYNC" in msg
    # device outputs the kernels store 16 bytes at a time must be 16-byte aligned
    import torch
    dp = torch.zeros((4, 3), dtype=torch.float64, device="cuda")
    da = torch.zeros(17, dtype=torch.float64, device="cuda")
    rc, msg = _rc_msg(ctx, L.ik_fabrik_solve(h, dp.data_ptr(), 4, 1e-3, 100,
                                             da.data_ptr() + 8, None, None, N.IK_F_DEVICE,
                                             ctypes.byref(st)))
    assert rc == N.IK_E_BADARG and "aligned" in msg
    # generic chains: at least one joint
    rc, msg = _rc_msg(ctx, L.ik_fabrik_calc(h, 0, pts.ctypes.data, pts.ctypes.data, 1,
                                            pts.ctypes.data, 4, 1e-3, 100, ang.ctypes.data,
                                            None, 0, ctypes.byref(st)))
    assert rc == N.IK_E_BADARG and "nj" in msg
    # unknown ANN mode
    rc, msg = _rc_msg(ctx, L.ik_ann_set_mode(h, 7))
    assert rc == N.IK_E_BADARG and "mode" in msg
    # the context still works
    p = np.array([[1.0, 2.1, 3.0]])
    a, it, _, s = ctx.fabrik_solve(p)
    ra, rit, _, _ = O.fabrik_ikine(p)
    assert np.array_equal(it, rit) and np.abs(a - ra).max() <= 1e-9


def test_ann_without_model_and_bad_models():
    from inversekinematicsann_amd import _native as N
    from inversekinematicsann_amd.kinematics.ann import REFERENCE_X_SCALER as XS, \
        REFERENCE_Y_SCALER as YS
    c = N.Context(0)
    try:
        with pytest.raises(N.NativeError) as ei:
            c.ann_solve(np.zeros((3, 3)))
        assert ei.value.code == N.IK_E_NOMODEL
        rng = np.random.default_rng(0)

        def dense(i, o):
            return rng.standard_normal((i, o)).astype(np.float32), np.zeros(o, np.float32)

        # wider than the layered path takes (16384), wrong input / output widths
        for dims in ((3, 16385, 4), (4, 16, 4), (3, 16, 5)):
            ws, bs = zip(*[dense(dims[k], dims[k + 1]) for k in range(len(dims) - 1)])
            with pytest.raises(N.NativeError) as ei:
                c.ann_load(list(ws), list(bs), ["tanh"] * (len(dims) - 2) + ["linear"], XS.mean,
                           XS.scale, YS.mean, YS.scale)
            assert ei.value.code == N.IK_E_BADARG
        # after the refusals a valid model loads and solves
        ws, bs = zip(*[dense(3, 32), dense(32, 4)])
        c.ann_load(list(ws), list(bs), ["tanh", "linear"], XS.mean, XS.scale, YS.mean, YS.scale)
        pts = np.array([[1.0, 0.5, 2.0], [0.3, -0.2, 1.0]])
        ang, _, _ = c.ann_solve(pts)
        ref = O.ann_forward(pts, list(ws), list(bs), ["tanh", "linear"], XS.mean, XS.scale,
                            YS.mean, YS.scale)
        assert np.abs(ang.astype(np.float64) - ref).max() <= 1e-5
    finally:
        c.close()


def test_bad_device_index():
    from inversekinematicsann_amd import _native as N
    L = N.load_library()
    h = ctypes.c_void_p()
    rc = L.ik_ctx_create(4096, ctypes.byref(h))
    assert rc == N.IK_E_BADARG and not h.value
    assert b"out of range" in L.ik_last_error()


def test_ann_effective_mode_reports_the_arithmetic_run():
    """ik_ann_effective_mode: the set mode when the model has layers
    that take it, fp32 for a fused model wider than 512 (with a RuntimeWarning from
    the Python wrapper), bf16x6 for fp16x3 on the layered path; -IK_E_NOMODEL
    before a model is loaded."""
    import warnings
    from inversekinematicsann_amd import _native as N
    from inversekinematicsann_amd.kinematics.ann import (REFERENCE_X_SCALER as XS,
                                                         REFERENCE_Y_SCALER as YS, glorot_model)
    c = N.Context(0)
    try:
        assert c.lib.ik_ann_effective_mode(c.handle) == -N.IK_E_NOMODEL

        def load(dims):
            m = glorot_model(dims, seed=1)
            c.ann_load(m.weights, m.biases, m.activations, XS.mean, XS.scale, YS.mean, YS.scale)

        load((3, 64, 64, 4))
        for mode in ("fp32", "bf16x6", "fp16x3"):
            c.ann_set_mode(mode)
            assert c.ann_effective_mode() == mode
        c.ann_set_mode("bf16x6")
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            load((3, 600, 600, 4))          # fused, wider than 512: fp32 build
        assert c.ann_effective_mode() == "fp32"
        assert any("ik_ann_effective_mode" in str(x.message) for x in w)
        c.ann_set_mode("fp16x3")
        load((3,) + (64,) * 30 + (4,))      # past the fused kernel's 24 layers: layered
        assert c.ann_effective_mode() == "bf16x6"
        pts = np.array([[1.0, 0.5, 2.0], [0.3, -0.2, 1.0]])
        ang, _ = c.ann_solve(pts)[:2]
        assert np.isfinite(ang).all()
    finally:
        c.close()


def test_kernel_timing_per_call_and_accumulated(ctx):
    """ik_ctx_set_timing: on = 1 keeps the last call's kernels, on = 2 accumulates
    the calls' kernels in launch order (what bench.timed uses to time back-to-back
    steps with no host sync between them); every duration is positive and the
    accumulated run repeats the one-call sequence."""
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(50_000, seed=5)
    ctx.set_timing(True)
    ctx.fabrik_solve(pts, 1e-3, 100)
    ctx.fabrik_solve(pts, 1e-3, 100)
    one = ctx.kernel_times()
    ctx.set_timing(2)
    for _ in range(3):
        ctx.fabrik_solve(pts, 1e-3, 100)
    acc = ctx.kernel_times()
    ctx.set_timing(False)
    assert ctx.kernel_times() == []
    names = [k for k, _ in one]
    assert "fabrik_iter_kernel" in names
    assert [k for k, _ in acc] == names * 3
    assert all(ms > 0.0 for _, ms in one + acc)
