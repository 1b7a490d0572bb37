"""Why does the pinned host path vary from run to run?  In one process: the CPU
the process runs on, the GPU's NUMA node, pinned copy rates (torch pin_memory and
ik_host_alloc buffers) and five timed FABRIK host-pointer solves on pinned and
pageable arrays.  Diagnostic only."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inversekinematicsann_amd import _native  # noqa: E402
from inversekinematicsann_amd.robot.position_generator import random_dist  # noqa: E402

out = {"cpu": os.sched_getaffinity(0).__len__()}
libc = ctypes.CDLL(None)
out["sched_getcpu"] = libc.sched_getcpu()
try:
    bus = torch.cuda.get_device_properties(0).pci_bus_id if hasattr(
        torch.cuda.get_device_properties(0), "pci_bus_id") else None
except Exception:  # noqa: BLE001
    bus = None
out["gpu_bus"] = bus
nodes = {}
for d in sorted(os.listdir("/sys/bus/pci/devices")):
    try:
        cls = open(f"/sys/bus/pci/devices/{d}/class").read().strip()
        if cls.startswith("0x0380") or cls.startswith("0x0300") or cls.startswith("0x1200"):
            nodes[d] = open(f"/sys/bus/pci/devices/{d}/numa_node").read().strip()
    except OSError:
        pass
out["display_numa"] = nodes
try:
    out["cpu_node_of_this_cpu"] = [n for n in os.listdir("/sys/devices/system/cpu/cpu%d" % out["sched_getcpu"]) if n.startswith("node")]
except OSError:
    pass

n = 1_000_000
pts = random_dist(n, seed=0)
ctx = _native.Context(0)
pp = _native.pinned_empty(pts.shape, np.float64)
pp[:] = pts
ang_p = _native.pinned_empty((n, 4), np.float64)
d = torch.empty(24_000_000, dtype=torch.uint8, device="cuda")
hp = torch.empty(24_000_000, dtype=torch.uint8).pin_memory()


def rate(fn, nb, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round(nb * reps / (time.perf_counter() - t0) / 1e9, 2)


out["h2d_torch_pinned_GBps"] = rate(lambda: d.copy_(hp, non_blocking=True), 24_000_000)
ikbuf = torch.from_numpy(pp.view(np.uint8).reshape(-1))
out["h2d_ik_host_alloc_GBps"] = rate(lambda: d.copy_(ikbuf, non_blocking=True), 24_000_000)
times = {"pinned_pipeline": [], "pageable": []}
ang_q = np.empty((n, 4), np.float64)
L, h = ctx.lib, ctx.handle
for label, src, dst in (("pinned_pipeline", pp, ang_p),
                        ("pageable", np.ascontiguousarray(pts), ang_q)):
    for _ in range(int(os.environ.get("PROBE_CALLS", "10"))):
        s = _native.IkStats()
        t0 = time.perf_counter()
        ctx._check(L.ik_fabrik_solve_fk(h, src.ctypes.data, n, 1e-3, 100, dst.ctypes.data,
                                        None, None, None, 0, ctypes.byref(s)))
        times[label].append(round((time.perf_counter() - t0) * 1e3, 3))
out["solve_ms"] = times
print(json.dumps(out))
