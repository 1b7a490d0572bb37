"""The host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): libikhip_asan.so (`make -C
inversekinematicsann_amd/csrc asan`: the same sources, the host code
instrumented, the gfx950 code objects unchanged) loaded in a child Python with
the clang ASan runtime preloaded, running the CPU tests that drive the host
paths -- the shard plan / part / tail / histogram helpers against the gloo
mirror (test_dist_gloo.py), the exported-symbol and loader checks
(test_cpu_host.py) -- and the ABI's argument refusals below.  Any sanitizer
report aborts the child (halt_on_error), so a green run means no reports.  No
GPU: the calls that need a device fail cleanly before touching one."""
import ctypes
import glob
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

LIB = os.path.join(ROOT, "inversekinematicsann_amd", "libikhip_asan.so")


def _asan_runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def _ensure_lib():
    src = os.path.join(ROOT, "inversekinematicsann_amd", "csrc")
    r = subprocess.run(["make", "-q", "-C", src, "asan"], capture_output=True)
    if r.returncode != 0:  # missing or stale: build it (host + gfx950, ~1.5 min)
        subprocess.run(["make", "-j8", "-C", src, "asan"], check=True, capture_output=True)


def bad_args():
    """The ABI's refusals that need no device: every one returns IK_E_BADARG (or
    a negative status) with a message, never touches memory it was not given."""
    from inversekinematicsann_amd import _native
    L = _native.load_library()
    assert os.path.basename(_native.LIB_PATH) == "libikhip_asan.so"
    BAD = _native.IK_E_BADARG
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    out = vp()
    assert L.ik_ctx_create(-1, ctypes.byref(out)) != 0 and not out.value
    assert L.ik_ctx_create(0, None) == BAD
    for fn, args in (("ik_ctx_destroy", (None,)),):
        assert getattr(L, fn)(*args) == 0  # NULL is a no-op
    assert L.ik_ctx_set_stream(None, None) == BAD
    assert L.ik_set_robot(None, None, None, None) == BAD
    assert L.ik_ctx_sync(None) == BAD
    assert L.ik_stats_fetch(None, None) == BAD
    assert L.ik_check_limits(None, None, i64(0), 0, None) == BAD
    assert L.ik_fk(None, None, i64(0), None, None, 0, None) == BAD
    assert L.ik_fabrik_solve(None, None, i64(0), ctypes.c_double(1e-3), 100, None, None, None,
                             0, None) == BAD
    assert L.ik_ann_solve(None, None, i64(0), None, None, 0, None) == BAD
    assert L.ik_ann_load(None, 1, None, None, None, None, None, None, None, None) == BAD
    assert L.ik_ann_set_mode(None, 0) == BAD
    assert L.ik_comm_set_chunks(None, 1) == BAD
    assert L.ik_comm_set_timeout(None, ctypes.c_double(1.0)) == BAD
    assert L.ik_comm_info(None, None, None, None) == BAD
    assert L.ik_comm_destroy(None) == BAD
    assert L.ik_comm_unique_id(None) == BAD
    assert L.ik_fk_err_quantile(None, ctypes.c_double(0.5), None) == BAD
    assert L.ik_fabrik_order_get(None, None, 0) < 0
    assert L.ik_fabrik_order_set(None, None, 0) == BAD
    assert L.ik_fabrik_calc(None, 4, None, None, 0, None, i64(0), ctypes.c_double(1e-3), 10,
                            None, None, 0, None) == BAD
    assert L.ik_kernel_times(None, 0, None, None, 0) < 0
    plan = _native.IkShardPlan() if hasattr(_native, "IkShardPlan") else None
    assert L.ik_shard_plan_of(i64(-1), 2, 1, None) == BAD
    assert L.ik_shard_plan_of(i64(10), 0, 1, None) == BAD
    b, e = i64(), i64()
    assert L.ik_shard_part(None, 0, 0, ctypes.byref(b), ctypes.byref(e)) == BAD
    assert L.ik_shard_range(i64(10), 2, 5, ctypes.byref(b), ctypes.byref(e)) == BAD
    assert L.ik_shard_range(i64(10), 2, 1, ctypes.byref(b), ctypes.byref(e)) == 0
    assert (b.value, e.value) == (5, 10)
    assert L.ik_tail_reduce(None, 2, None) == BAD
    assert L.ik_fkhist_bin(ctypes.c_double(float("nan"))) == -1
    assert L.ik_fkhist_bin(ctypes.c_double(-1.0)) == -1
    assert L.ik_last_error()  # the last refusal's message
    del plan
    print("bad_args ok")


@pytest.mark.skipif(_asan_runtime() is None, reason="clang ASan runtime not found")
def test_host_code_under_asan_ubsan():
    _ensure_lib()
    env = dict(os.environ,
               LD_PRELOAD=_asan_runtime(), IKHIP_LIB=LIB,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "tests/test_cpu_host.py", "tests/test_dist_gloo.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail
    r = subprocess.run([sys.executable, "-c", "import tests.test_asan_host as t; t.bad_args()"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "bad_args ok" in out, out[-3000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-3000:]
