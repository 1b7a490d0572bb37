"""ctypes binding of libikhip.so (the C ABI in include/ikhip.h).

The product path has no CPU fallback: if the shared library is missing or no
HIP device can be opened, every solve raises (NativeUnavailable).  Arrays may be
numpy host arrays (staged by the library) or torch CUDA tensors on the
context's device (passed as device pointers, computed in place on the
context's stream).
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
from typing import Optional, Sequence

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# IKHIP_LIB selects another build of the same ABI (e.g. libikhip_diag.so, the
# diagnostic build with in-kernel stamps); the default is the production build.
LIB_PATH = os.environ.get("IKHIP_LIB") or os.path.join(_PKG, "libikhip.so")

IK_OK, IK_E_OUT_OF_REACH, IK_E_DOMAIN, IK_E_ZERODIV, IK_E_ANGLE_RANGE = 0, 1, 2, 3, 4
IK_E_BADARG, IK_E_HIP, IK_E_NOMODEL, IK_E_RCCL = 16, 17, 18, 19
IK_METHOD_ANN, IK_METHOD_FABRIK = 0, 1
IK_COMM_ID_BYTES = 128
IK_MAX_GATHER_CHUNKS = 8
IK_FKHIST_BINS = 2048
IK_F_DEVICE, IK_F_ASYNC, IK_F_NO_LIMITS = 1, 2, 4
ACTS = {"linear": 0, "tanh": 1, "relu": 2, "sigmoid": 3}

EXPORTED_SYMBOLS = ("ik_ctx_create", "ik_ctx_destroy", "ik_ctx_set_stream", "ik_ctx_get_stream",
                    "ik_last_error", "ik_version", "ik_set_robot", "ik_check_limits", "ik_fk", "ik_fk_chain",
                    "ik_fabrik_solve", "ik_fabrik_solve_fk", "ik_fabrik_calc", "ik_fabrik_reset_order", "ik_ann_load", "ik_ann_solve",
                    "ik_stats_fetch", "ik_ctx_set_timing", "ik_kernel_times",
                    "ik_ctx_set_debug", "ik_debug_read", "ik_ann_set_mode", "ik_ann_get_mode",
                    "ik_ann_effective_mode",
                    "ik_comm_unique_id", "ik_comm_init", "ik_comm_init_loopback",
                    "ik_loopback_byte", "ik_comm_destroy", "ik_comm_info",
                    "ik_comm_set_chunks", "ik_shard_plan_of", "ik_shard_part", "ik_shard_range",
                    "ik_tail_reduce", "ik_fkhist_bin", "ik_fkhist_upper", "ik_fk_err_quantile",
                    "ik_ann_solve_sharded", "ik_fabrik_solve_sharded", "ik_host_alloc",
                    "ik_host_free", "ik_ctx_sync", "ik_comm_set_timeout",
                    "ik_comm_loopback_stall", "ik_fabrik_order_get", "ik_fabrik_order_set")
ANN_MODES = {"fp32": 0, "bf16x6": 1, "fp16x3": 2}


class NativeUnavailable(RuntimeError):
    """libikhip.so is not built or no gfx950 device is usable."""


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libikhip error {code}: {msg}")
        self.code = code


class IkStats(ctypes.Structure):
    _fields_ = [("first_oob", ctypes.c_int64), ("first_err", ctypes.c_int64),
                ("first_err_code", ctypes.c_int32), ("max_iters", ctypes.c_int32),
                ("sum_iters", ctypes.c_int64), ("n_capped", ctypes.c_int64),
                ("max_fk_err", ctypes.c_double), ("sum_fk_err", ctypes.c_double),
                ("gather_ms", ctypes.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class ShardTail(ctypes.Structure):
    """ik_shard_tail: one rank's batch stats as gathered (64 bytes)."""
    _fields_ = [("first_oob", ctypes.c_int64), ("first_err", ctypes.c_int64),
                ("first_err_code", ctypes.c_int32), ("max_iters", ctypes.c_int32),
                ("sum_iters", ctypes.c_int64), ("n_capped", ctypes.c_int64),
                ("max_fk_err", ctypes.c_double), ("sum_fk_err", ctypes.c_double),
                ("rows", ctypes.c_int64)]


class ShardPlan(ctypes.Structure):
    """ik_shard_plan: a batch split over the ranks in chunks (include/ikhip.h)."""
    _fields_ = [("n", ctypes.c_int64), ("nranks", ctypes.c_int32), ("chunks", ctypes.c_int32),
                ("part_rows", ctypes.c_int64), ("full_rows", ctypes.c_int64)]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load libikhip.so.  torch (if installed) is imported first so that the
    process has exactly one HIP runtime (torch ships its own libamdhip64)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"{path} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C inversekinematicsann_amd/csrc`)")
        if "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except Exception:  # noqa: BLE001 -- torch is optional plumbing
                pass
        L = ctypes.CDLL(path)
        vp, dp, ip = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p
        i64, i32 = ctypes.c_int64, ctypes.c_int32
        st = ctypes.POINTER(IkStats)
        L.ik_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.ik_ctx_destroy.argtypes = [vp]
        L.ik_ctx_set_stream.argtypes = [vp, vp]
        L.ik_ctx_get_stream.argtypes = [vp]
        L.ik_ctx_get_stream.restype = vp
        L.ik_last_error.restype = ctypes.c_char_p
        L.ik_version.restype = ctypes.c_char_p
        L.ik_set_robot.argtypes = [vp, dp, dp, dp]
        L.ik_check_limits.argtypes = [vp, dp, i64, ctypes.c_int, st]
        L.ik_fk.argtypes = [vp, dp, i64, dp, dp, ctypes.c_int, st]
        L.ik_fk_chain.argtypes = [vp, ctypes.c_int, dp, dp, i64, dp, dp, ctypes.c_int, st]
        L.ik_fabrik_solve.argtypes = [vp, dp, i64, ctypes.c_double, i32, dp, ip, dp, ctypes.c_int,
                                      st]
        L.ik_fabrik_solve_fk.argtypes = [vp, dp, i64, ctypes.c_double, i32, dp, ip, dp, dp,
                                         ctypes.c_int, st]
        L.ik_fabrik_reset_order.argtypes = [vp]
        L.ik_fabrik_order_get.argtypes = [vp, vp, ctypes.c_int]
        L.ik_fabrik_order_set.argtypes = [vp, vp, ctypes.c_int]
        L.ik_fabrik_calc.argtypes = [vp, ctypes.c_int, dp, dp, ctypes.c_int, dp, i64,
                                     ctypes.c_double, i32, dp, ip, ctypes.c_int, st]
        L.ik_ann_load.argtypes = [vp, ctypes.c_int, ip, ip, ctypes.POINTER(ctypes.c_void_p),
                                  ctypes.POINTER(ctypes.c_void_p), dp, dp, dp, dp]
        L.ik_ann_solve.argtypes = [vp, dp, i64, dp, dp, ctypes.c_int, st]
        L.ik_stats_fetch.argtypes = [vp, st]
        L.ik_ctx_sync.argtypes = [vp]
        L.ik_comm_set_timeout.argtypes = [vp, ctypes.c_double]
        L.ik_comm_loopback_stall.argtypes = [vp, ctypes.c_int]
        L.ik_ctx_set_timing.argtypes = [vp, ctypes.c_int]
        L.ik_kernel_times.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int]
        L.ik_ctx_set_debug.argtypes = [vp, ctypes.c_int]
        L.ik_debug_read.argtypes = [vp, vp, ctypes.c_int]
        L.ik_ann_set_mode.argtypes = [vp, ctypes.c_int]
        L.ik_ann_get_mode.argtypes = [vp]
        L.ik_ann_effective_mode.argtypes = [vp]
        L.ik_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        L.ik_host_free.argtypes = [vp]
        L.ik_comm_unique_id.argtypes = [vp]
        L.ik_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.ik_comm_init_loopback.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.ik_loopback_byte.argtypes = [ctypes.c_int, i64]
        L.ik_comm_destroy.argtypes = [vp]
        ipt = ctypes.POINTER(ctypes.c_int)
        L.ik_comm_info.argtypes = [vp, ipt, ipt, ipt]
        L.ik_comm_set_chunks.argtypes = [vp, ctypes.c_int]
        L.ik_shard_plan_of.argtypes = [i64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ShardPlan)]
        L.ik_shard_part.argtypes = [ctypes.POINTER(ShardPlan), ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.ik_shard_range.argtypes = [i64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(i64),
                                     ctypes.POINTER(i64)]
        L.ik_tail_reduce.argtypes = [vp, ctypes.c_int, st]
        L.ik_fkhist_bin.argtypes = [ctypes.c_double]
        L.ik_fkhist_upper.argtypes = [ctypes.c_int]
        L.ik_fkhist_upper.restype = ctypes.c_double
        L.ik_fk_err_quantile.argtypes = [vp, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
        L.ik_ann_solve_sharded.argtypes = [vp, dp, i64, dp, dp, ctypes.c_int, st]
        L.ik_fabrik_solve_sharded.argtypes = [vp, dp, i64, ctypes.c_double, i32, dp, ip, dp,
                                              ctypes.c_int, st]
        _lib = L
        return L


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def _is_device(a) -> bool:
    return hasattr(a, "is_cuda") and bool(a.is_cuda)


def _host(a, dtype, shape_last=None):
    arr = np.ascontiguousarray(a, dtype=dtype)
    if shape_last is not None:
        arr = arr.reshape(-1, shape_last)
    return arr


class Context:
    """One libikhip context (device, stream, scratch, ANN weights)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.ik_ctx_create(int(device), ctypes.byref(h))
        if rc != IK_OK:
            raise NativeUnavailable(f"ik_ctx_create(device={device}) failed: "
                                    f"{self.lib.ik_last_error().decode()}")
        self.handle = h
        self.device = int(device)
        # what ik_ctx_create installed (SixDOFRobot, robot/robot.py:38-42)
        self._robot = (np.array([0.0, np.pi / 2, 0.0, 0.0, 2.0, 0.0, 0.0, 0.0,
                                 0.0, 2.0, 2.0, 2.0, np.pi / 2, 0.0, 0.0, 0.0]),
                       np.array([2.0, 2.0, 2.0, 2.0]), np.array([0.0, 6.0, -6.0, 6.0, -3.0, 6.0]))
        self.robot_uploads = 0

    def close(self):
        if getattr(self, "handle", None):
            self.lib.ik_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def _check(self, rc: int):
        if rc != IK_OK:
            raise NativeError(rc, self.lib.ik_last_error().decode())

    # -- configuration ------------------------------------------------------
    def set_stream(self, stream_handle: Optional[int]):
        self._check(self.lib.ik_ctx_set_stream(self.handle, stream_handle))

    def set_robot(self, dh, links=None, limits=None) -> bool:
        """Upload a robot (None keeps the context's links / limits).  Skipped when
        nothing the device reads changes: dh[0][0] (theta_1) is not read there --
        every solve takes the point's own azimuth -- so the reference's per-call
        write of the last point's theta_1 into the table (inverse.py:125) costs no
        upload.  Returns whether ik_set_robot was called."""
        dh = _host(dh, np.float64).reshape(16)
        links = self._robot[1] if links is None else _host(links, np.float64).reshape(4)
        limits = self._robot[2] if limits is None else _host(limits, np.float64).reshape(6)
        if (np.array_equal(dh[1:], self._robot[0][1:]) and np.array_equal(links, self._robot[1])
                and np.array_equal(limits, self._robot[2])):
            return False
        self._check(self.lib.ik_set_robot(self.handle, _ptr(dh), _ptr(links), _ptr(limits)))
        self._robot = (dh.copy(), links.copy(), limits.copy())
        self.robot_uploads += 1
        return True

    # -- solves ---------------------------------------------------------------
    def check_limits(self, pts) -> IkStats:
        s = IkStats()
        if _is_device(pts):
            self._check(self.lib.ik_check_limits(self.handle, _ptr(pts), pts.shape[0],
                                                 IK_F_DEVICE, ctypes.byref(s)))
        else:
            p = _host(pts, np.float64, 3)
            self._check(self.lib.ik_check_limits(self.handle, _ptr(p), p.shape[0], 0,
                                                 ctypes.byref(s)))
        return s

    def fk(self, ang, with_mats: bool = False):
        """Batched FK: returns (xyz n x 3, mats n x 4 x 4 x 4 or None, stats)."""
        s = IkStats()
        a = _host(ang, np.float64, 4)
        n = a.shape[0]
        xyz = np.empty((n, 3), np.float64)
        mats = np.empty((n, 4, 4, 4), np.float64) if with_mats else None
        self._check(self.lib.ik_fk(self.handle, _ptr(a), n, _ptr(xyz), _ptr(mats), 0,
                                   ctypes.byref(s)))
        return xyz, mats, s

    def fk_chain(self, dh, ang, with_mats: bool = False):
        """FK of an nj-joint DH table (4 x nj): returns (xyz n x 3, mats n x nj x 4 x 4
        or None, stats)."""
        d = _host(dh, np.float64)
        if d.ndim != 2 or d.shape[0] != 4:
            raise ValueError("dh must be 4 x nj")
        nj = d.shape[1]
        a = _host(ang, np.float64, nj)
        n = a.shape[0]
        xyz = np.empty((n, 3), np.float64)
        mats = np.empty((n, nj, 4, 4), np.float64) if with_mats else None
        s = IkStats()
        self._check(self.lib.ik_fk_chain(self.handle, nj, _ptr(d), _ptr(a), n, _ptr(xyz),
                                         _ptr(mats), 0, ctypes.byref(s)))
        return xyz, mats, s

    def fk_device(self, ang, xyz, flags: int = IK_F_DEVICE):
        s = IkStats()
        n = int(ang.shape[0])
        args = (self._dev(ang, "float64", (n, 4), "ang"), self._dev(xyz, "float64", (n, 3), "xyz"))
        self._on_torch_stream(lambda: self._check(self.lib.ik_fk(
            self.handle, args[0], n, args[1], None, flags, ctypes.byref(s))))
        return s

    def fabrik_solve(self, pts, tol=1e-3, max_iter=100, check_limits=True,
                     want_iters=True, want_joints=False):
        """Host arrays in/out: returns (angles n x 4 f64, iters, joints, stats)."""
        s = IkStats()
        p = _host(pts, np.float64, 3)
        n = p.shape[0]
        ang = np.empty((n, 4), np.float64)
        it = np.empty(n, np.int32) if want_iters else None
        jo = np.empty((n, 4, 3), np.float64) if want_joints else None
        flags = 0 if check_limits else IK_F_NO_LIMITS
        self._check(self.lib.ik_fabrik_solve(self.handle, _ptr(p), n, float(tol), int(max_iter),
                                             _ptr(ang), _ptr(it), _ptr(jo), flags,
                                             ctypes.byref(s)))
        return ang, it, jo, s

    def fabrik_solve_fk(self, pts, tol=1e-3, max_iter=100, check_limits=True):
        """FABRIK with the FK round trip in the same launch (ik_fabrik_solve_fk):
        returns (angles n x 4 f64, iters, fk_err n f64, stats)."""
        s = IkStats()
        p = _host(pts, np.float64, 3)
        n = p.shape[0]
        ang = np.empty((n, 4), np.float64)
        it = np.empty(n, np.int32)
        err = np.empty(n, np.float64)
        flags = 0 if check_limits else IK_F_NO_LIMITS
        self._check(self.lib.ik_fabrik_solve_fk(self.handle, _ptr(p), n, float(tol),
                                                int(max_iter), _ptr(ang), _ptr(it), None,
                                                _ptr(err), flags, ctypes.byref(s)))
        return ang, it, err, s

    def _on_torch_stream(self, fn):
        """Run fn with the library on torch's current stream of this device, so a
        call on tensors that pending torch kernels produce orders after them (the
        context's own stream does not wait for torch's); the previous stream is
        restored after.  A caller that pinned a stream with set_stream (bench.py
        uses one shared stream) gets the same ordering either way."""
        import torch
        cur = torch.cuda.current_stream(self.device).cuda_stream
        prev = self.lib.ik_ctx_get_stream(self.handle)
        self._check(self.lib.ik_ctx_set_stream(self.handle, cur))
        try:
            return fn()
        finally:
            self.lib.ik_ctx_set_stream(self.handle, prev)

    def _dev(self, t, dtype: str, shape, name: str):
        """Checks a device tensor argument before its pointer goes to the library:
        the kernels read raw memory of a fixed dtype and layout."""
        if t is None:
            return None
        if not _is_device(t):
            raise ValueError(f"{name}: expected a device tensor on cuda:{self.device}")
        if str(t.dtype) != f"torch.{dtype}":
            raise ValueError(f"{name}: dtype {t.dtype}, expected torch.{dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name}: must be contiguous")
        if t.device.index != self.device:
            raise ValueError(f"{name}: on {t.device}, the context is on cuda:{self.device}")
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
        return _ptr(t)

    def fabrik_solve_device(self, pts, ang, iters=None, joints=None, tol=1e-3, max_iter=100,
                            flags: int = IK_F_DEVICE, fk_err=None):
        s = IkStats()
        n = int(pts.shape[0])
        args = (self._dev(pts, "float64", (n, 3), "pts"),
                self._dev(ang, "float64", (n, 4), "ang"),
                self._dev(iters, "int32", (n,), "iters"),
                self._dev(joints, "float64", (n, 4, 3), "joints"),
                self._dev(fk_err, "float64", (n,), "fk_err"))
        self._on_torch_stream(lambda: self._check(self.lib.ik_fabrik_solve_fk(
            self.handle, args[0], n, float(tol), int(max_iter), args[1], args[2], args[3],
            args[4], flags, ctypes.byref(s))))
        return s

    def fabrik_reset_order(self):
        """Forget the learned FABRIK work order (ik_fabrik_reset_order): the table
        a fresh context starts with (SixDOFRobot: the built-in prior; other chains:
        empty, point order), on the context's current stream."""
        self._on_torch_stream(lambda: self._check(self.lib.ik_fabrik_reset_order(self.handle)))

    def fabrik_order_get(self) -> np.ndarray:
        """The work-order table (1024 uint32: 1 + largest recorded iterations per cell)."""
        out = np.zeros(1024, np.uint32)
        n = self.lib.ik_fabrik_order_get(self.handle, out.ctypes.data, out.size)
        if n < 0:
            raise NativeError(-n, self.lib.ik_last_error().decode())
        return out

    def fabrik_order_set(self, key=None):
        """Replace the work-order table (None: empty, point order)."""
        k = None if key is None else np.ascontiguousarray(key, np.uint32).reshape(1024)
        self._check(self.lib.ik_fabrik_order_set(self.handle, _ptr(k), 0 if k is None else 1024))

    def fabrik_calc(self, dists, init, goals, tol=1e-3, max_iter=100):
        """Batched Fabrik.calculate; init n x nj x 3 or nj x 3 (shared)."""
        s = IkStats()
        d = _host(dists, np.float64).reshape(-1)
        nj = d.shape[0]
        ini = np.ascontiguousarray(init, dtype=np.float64)
        shared = 1 if ini.ndim == 2 else 0
        g = _host(goals, np.float64, 3)
        n = g.shape[0]
        if ini.shape[-2:] != (nj, 3) or (not shared and ini.shape[0] != n):
            raise ValueError("init must be n x nj x 3 or nj x 3")
        out = np.empty((n, nj, 3), np.float64)
        it = np.empty(n, np.int32)
        self._check(self.lib.ik_fabrik_calc(self.handle, nj, _ptr(d), _ptr(ini), shared, _ptr(g),
                                            n, float(tol), int(max_iter), _ptr(out), _ptr(it),
                                            0, ctypes.byref(s)))
        return out, it, s

    def ann_load(self, weights: Sequence, biases: Sequence, acts: Sequence[str], x_mean,
                 x_scale, y_mean, y_scale):
        Ws = [np.ascontiguousarray(w, dtype=np.float32) for w in weights]
        bs = [np.ascontiguousarray(b, dtype=np.float32).reshape(-1) for b in biases]
        nl = len(Ws)
        dims = [Ws[0].shape[0]] + [w.shape[1] for w in Ws]
        for l in range(nl):
            if Ws[l].shape != (dims[l], dims[l + 1]) or bs[l].shape != (dims[l + 1],):
                raise ValueError(f"layer {l}: kernel {Ws[l].shape} / bias {bs[l].shape} mismatch")
        dims_a = np.array(dims, np.int32)
        acts_a = np.array([ACTS[a] for a in acts], np.int32)
        wp = (ctypes.c_void_p * nl)(*[w.ctypes.data for w in Ws])
        bp = (ctypes.c_void_p * nl)(*[b.ctypes.data for b in bs])
        sc = [_host(v, np.float64).reshape(-1) for v in (x_mean, x_scale, y_mean, y_scale)]
        self._check(self.lib.ik_ann_load(self.handle, nl, _ptr(dims_a), _ptr(acts_a), wp, bp,
                                         *[_ptr(v) for v in sc]))
        self._warn_mode()

    def ann_set_mode(self, mode: str):
        """Hidden-layer GEMM arithmetic: "fp32" (default), "bf16x6" or "fp16x3" (ikhip.h)."""
        if mode not in ANN_MODES:
            raise ValueError(f"unknown ANN mode {mode!r}; expected one of {sorted(ANN_MODES)}")
        self._check(self.lib.ik_ann_set_mode(self.handle, ANN_MODES[mode]))
        self._warn_mode()

    def ann_effective_mode(self) -> str:
        """The arithmetic the next ANN solve runs for the loaded model
        (ik_ann_effective_mode): the set mode, or "fp32" when no layer can take it
        (a fused model wider than 512, or split planes left out at load because
        the device had room only for the fp32 operands), or "bf16x6" for
        "fp16x3" on the layered path."""
        m = self.lib.ik_ann_effective_mode(self.handle)
        if m < 0:
            raise NativeError(-m, self.lib.ik_last_error().decode())
        return {v: k for k, v in ANN_MODES.items()}[m]

    def _warn_mode(self):
        """Say so when a loaded model runs another arithmetic than the set mode."""
        want = self.ann_mode()
        if want == "fp32" or self.lib.ik_ann_effective_mode(self.handle) < 0:
            return
        got = self.ann_effective_mode()
        if got != want:
            import warnings
            warnings.warn(f"ANN mode {want!r} is not available for the loaded model; its "
                          f"solves run {got!r} (ik_ann_effective_mode)", RuntimeWarning,
                          stacklevel=3)

    def ann_mode(self) -> str:
        m = self.lib.ik_ann_get_mode(self.handle)
        if m < 0:
            raise NativeError(-m, self.lib.ik_last_error().decode())
        return {v: k for k, v in ANN_MODES.items()}[m]

    def ann_solve(self, pts, check_limits=True, want_fk_err=False):
        s = IkStats()
        p = _host(pts, np.float64, 3)
        n = p.shape[0]
        ang = np.empty((n, 4), np.float32)
        err = np.empty(n, np.float64) if want_fk_err else None
        flags = 0 if check_limits else IK_F_NO_LIMITS
        self._check(self.lib.ik_ann_solve(self.handle, _ptr(p), n, _ptr(ang), _ptr(err), flags,
                                          ctypes.byref(s)))
        return ang, err, s

    def ann_solve_device(self, pts, ang, fk_err=None, flags: int = IK_F_DEVICE):
        s = IkStats()
        n = int(pts.shape[0])
        args = (self._dev(pts, "float64", (n, 3), "pts"), self._dev(ang, "float32", (n, 4), "ang"),
                self._dev(fk_err, "float64", (n,), "fk_err"))
        self._on_torch_stream(lambda: self._check(self.lib.ik_ann_solve(
            self.handle, args[0], n, args[1], args[2], flags, ctypes.byref(s))))
        return s

    # -- multi-GPU (RCCL over xGMI; include/ikhip.h "multi-GPU") -------------
    def comm_init(self, nranks: int, rank: int, uid: bytes):
        """Collective over the ranks: binds this context to an RCCL communicator."""
        if len(uid) != IK_COMM_ID_BYTES:
            raise ValueError(f"unique id must be {IK_COMM_ID_BYTES} bytes")
        buf = ctypes.create_string_buffer(bytes(uid), IK_COMM_ID_BYTES)
        self._check(self.lib.ik_comm_init(self.handle, int(nranks), int(rank), buf))

    def comm_init_loopback(self, nranks: int, rank: int):
        """TEST-ONLY (ik_comm_init_loopback): rank `rank` of `nranks` on this one GPU,
        no RCCL; the other ranks' gathered rows come back as loopback_byte patterns."""
        self._check(self.lib.ik_comm_init_loopback(self.handle, int(nranks), int(rank)))

    def comm_destroy(self):
        self._check(self.lib.ik_comm_destroy(self.handle))

    def comm_set_timeout(self, seconds: float):
        """Deadline of the communicator's host waits (0: IKHIP_RCCL_TIMEOUT_S or 120 s)."""
        self._check(self.lib.ik_comm_set_timeout(self.handle, float(seconds)))

    def comm_loopback_stall(self, on: bool = True):
        """TEST-ONLY (ik_comm_loopback_stall): the loopback all-gathers wait for a
        peer that never comes, until the deadline's abort releases them."""
        self._check(self.lib.ik_comm_loopback_stall(self.handle, 1 if on else 0))

    def sync(self):
        """Wait for the last call (ik_ctx_sync): bounded by the communicator's
        deadline when one is bound; raises NativeError(IK_E_RCCL) on abort."""
        self._check(self.lib.ik_ctx_sync(self.handle))

    def comm_info(self):
        """(ranks of the library's communicator, this rank, chunks of the last sharded call)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.ik_comm_info(self.handle, ctypes.byref(a), ctypes.byref(b),
                                          ctypes.byref(c)))
        return a.value, b.value, c.value

    def comm_set_chunks(self, chunks: int):
        """Chunks of the sharded solves' in-place all-gathers (0 = automatic)."""
        self._check(self.lib.ik_comm_set_chunks(self.handle, int(chunks)))

    def fk_err_quantile(self, q: float) -> float:
        """q-quantile (upper bound, 1/16 octave) of the last sharded call's FK errors,
        from every rank's gathered histogram."""
        out = ctypes.c_double()
        self._check(self.lib.ik_fk_err_quantile(self.handle, float(q), ctypes.byref(out)))
        return out.value

    def ann_solve_sharded(self, pts, check_limits=True, want_fk_err=False):
        """Host arrays: every rank passes the whole batch and gets the whole batch's
        angles (float32) and stats back; it solves only its own shard."""
        s = IkStats()
        p = _host(pts, np.float64, 3)
        n = p.shape[0]
        ang = np.empty((n, 4), np.float32)
        # only this rank's rows of fk_err are written (ikhip.h): the rest stay NaN
        err = np.full(n, np.nan) if want_fk_err else None
        flags = 0 if check_limits else IK_F_NO_LIMITS
        self._check(self.lib.ik_ann_solve_sharded(self.handle, _ptr(p), n, _ptr(ang), _ptr(err),
                                                  flags, ctypes.byref(s)))
        return ang, err, s

    def fabrik_solve_sharded(self, pts, tol=1e-3, max_iter=100, check_limits=True,
                             want_fk_err=False):
        s = IkStats()
        p = _host(pts, np.float64, 3)
        n = p.shape[0]
        ang = np.empty((n, 4), np.float64)
        it = np.empty(n, np.int32)
        # only this rank's rows of fk_err are written (ikhip.h): the rest stay NaN
        err = np.full(n, np.nan) if want_fk_err else None
        flags = 0 if check_limits else IK_F_NO_LIMITS
        self._check(self.lib.ik_fabrik_solve_sharded(self.handle, _ptr(p), n, float(tol),
                                                     int(max_iter), _ptr(ang), _ptr(it),
                                                     _ptr(err), flags, ctypes.byref(s)))
        return ang, it, err, s

    def ann_solve_sharded_device(self, pts, ang, fk_err=None, flags: int = IK_F_DEVICE):
        s = IkStats()
        n = int(pts.shape[0])
        args = (self._dev(pts, "float64", (n, 3), "pts"), self._dev(ang, "float32", (n, 4), "ang"),
                self._dev(fk_err, "float64", (n,), "fk_err"))
        self._on_torch_stream(lambda: self._check(self.lib.ik_ann_solve_sharded(
            self.handle, args[0], n, args[1], args[2], flags, ctypes.byref(s))))
        return s

    def fabrik_solve_sharded_device(self, pts, ang, iters=None, fk_err=None, tol=1e-3,
                                    max_iter=100, flags: int = IK_F_DEVICE):
        s = IkStats()
        n = int(pts.shape[0])
        args = (self._dev(pts, "float64", (n, 3), "pts"), self._dev(ang, "float64", (n, 4), "ang"),
                self._dev(iters, "int32", (n,), "iters"), self._dev(fk_err, "float64", (n,),
                                                                     "fk_err"))
        self._on_torch_stream(lambda: self._check(self.lib.ik_fabrik_solve_sharded(
            self.handle, args[0], n, float(tol), int(max_iter), args[1], args[2], args[3], flags,
            ctypes.byref(s))))
        return s

    def set_timing(self, on=True):
        """ik_ctx_set_timing: True / 1 each call's kernels, 2 accumulate across calls
        (up to 64 kernels, in launch order), False / 0 off."""
        self._check(self.lib.ik_ctx_set_timing(self.handle, 2 if on == 2 else (1 if on else 0)))

    def kernel_times(self):
        """[(kernel name, ms)] of the last call (after set_timing(True)), or of every
        call since set_timing(2), in launch order."""
        ms = np.zeros(64, np.float32)
        names = ctypes.create_string_buffer(64 * 48)
        n = self.lib.ik_kernel_times(self.handle, 64, ms.ctypes.data, ctypes.addressof(names), 48)
        if n < 0:
            raise NativeError(-n, self.lib.ik_last_error().decode())
        raw = names.raw
        return [(raw[i * 48:(i + 1) * 48].split(b"\0")[0].decode(), float(ms[i]))
                for i in range(n)]

    def set_debug(self, on: bool = True):
        self._check(self.lib.ik_ctx_set_debug(self.handle, 1 if on else 0))

    def debug_stamps(self) -> np.ndarray:
        """ANN diagnostic stamps as (tile, wave, slot) uint64 (see ikhip.h)."""
        out = np.zeros(4 * 4 * 32, np.uint64)
        n = self.lib.ik_debug_read(self.handle, out.ctypes.data, out.size)
        if n < 0:
            raise NativeError(-n, self.lib.ik_last_error().decode())
        return out[:n].reshape(4, 4, 32) if n == out.size else out[:n]

    def debug_words(self, n: int) -> np.ndarray:
        """The first n words of the diagnostic buffer (FABRIK counters, diag build)."""
        out = np.zeros(n, np.uint64)
        got = self.lib.ik_debug_read(self.handle, out.ctypes.data, out.size)
        if got < 0:
            raise NativeError(-got, self.lib.ik_last_error().decode())
        return out[:got]

    def stats_fetch(self) -> IkStats:
        s = IkStats()
        self._check(self.lib.ik_stats_fetch(self.handle, ctypes.byref(s)))
        return s


def _host_check(rc: int):
    if rc != IK_OK:
        raise NativeError(rc, load_library().ik_last_error().decode())


class _PinnedBlock:
    """Owner of one ik_host_alloc block; freed when the last array view goes."""

    def __init__(self, nbytes: int):
        self.lib = load_library()
        self.ptr = ctypes.c_void_p()
        _host_check(self.lib.ik_host_alloc(max(1, int(nbytes)), ctypes.byref(self.ptr)))
        self.nbytes = int(nbytes)

    def __del__(self):
        try:
            if self.ptr:
                self.lib.ik_host_free(self.ptr)
        except Exception:  # noqa: BLE001
            pass


def pinned_empty(shape, dtype=np.float64) -> np.ndarray:
    """A numpy array in pinned host memory (ik_host_alloc): host-pointer solves
    on such arrays overlap their PCIe copies with the kernels (ikhip.h).  The
    block is freed when the last view of it goes (the buffer numpy holds keeps
    its owner alive)."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape))
    blk = _PinnedBlock(n * dt.itemsize)
    buf = (ctypes.c_char * max(1, n * dt.itemsize)).from_address(blk.ptr.value)
    buf._owner = blk
    return np.frombuffer(buf, dtype=dt, count=n).reshape(shape)


def comm_unique_id() -> bytes:
    """ncclGetUniqueId through the library (one rank calls it and shares the bytes)."""
    L = load_library()
    buf = ctypes.create_string_buffer(IK_COMM_ID_BYTES)
    _host_check(L.ik_comm_unique_id(buf))
    return buf.raw


def shard_range(n: int, nranks: int, rank: int):
    """ik_shard_range (host only): rank's rows [begin, end) of an n-point batch."""
    b, e = ctypes.c_int64(), ctypes.c_int64()
    _host_check(load_library().ik_shard_range(int(n), int(nranks), int(rank), ctypes.byref(b),
                                              ctypes.byref(e)))
    return b.value, e.value


def shard_plan(n: int, nranks: int, chunks: int = 1) -> ShardPlan:
    """ik_shard_plan_of (host only): the batch in chunks of nranks parts."""
    p = ShardPlan()
    _host_check(load_library().ik_shard_plan_of(int(n), int(nranks), int(chunks),
                                                ctypes.byref(p)))
    return p


def shard_part(plan: ShardPlan, rank: int, chunk: int):
    """ik_shard_part (host only): rank's rows [begin, end) of the chunk."""
    b, e = ctypes.c_int64(), ctypes.c_int64()
    _host_check(load_library().ik_shard_part(ctypes.byref(plan), int(rank), int(chunk),
                                             ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def fkhist_bin(e: float) -> int:
    """ik_fkhist_bin: the FK-error histogram bin of e (-1: not counted)."""
    return int(load_library().ik_fkhist_bin(float(e)))


def fkhist_upper(b: int) -> float:
    """ik_fkhist_upper: the upper edge of histogram bin b."""
    return float(load_library().ik_fkhist_upper(int(b)))


def tail_reduce(tails: Sequence[ShardTail]) -> IkStats:
    """ik_tail_reduce (host only): the batch stats from every rank's tail."""
    arr = (ShardTail * len(tails))(*tails)
    s = IkStats()
    _host_check(load_library().ik_tail_reduce(arr, len(tails), ctypes.byref(s)))
    return s


_default_ctx: Optional[Context] = None
_default_lock = threading.Lock()


def default_device() -> int:
    for k in ("IKHIP_DEVICE", "LOCAL_RANK"):
        if os.environ.get(k):
            return int(os.environ[k])
    return 0


def context() -> Context:
    """The process-wide context on default_device()."""
    global _default_ctx
    with _default_lock:
        if _default_ctx is None:
            _default_ctx = Context(default_device())
        return _default_ctx
