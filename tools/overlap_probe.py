"""Does a sharded call's gather run under the next chunk's solve?  One GPU plays
rank 0 of 8 through the test-only loopback communicator (its gather is a kernel on
the library's comm stream, as RCCL's is), FABRIK on 8M points (1M per rank), chunk
counts 1 and 2; run it under `rocprofv3 --kernel-trace` and read the kernels'
start / end times:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/overlap -- \\
        python3 tools/overlap_probe.py
    python3 tools/overlap_probe.py --summary gpurun_out/overlap
"""
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run():
    import torch
    from inversekinematicsann_amd import _native
    from inversekinematicsann_amd import dist as D
    from inversekinematicsann_amd.robot.position_generator import random_dist
    g, n = 8, 8_000_000
    ctx = _native.Context(0)
    sc = D.ShardedContext.loopback(ctx, g, 0)
    pts = torch.from_numpy(random_dist(n, seed=1)).cuda()
    ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
    it = torch.empty(n, dtype=torch.int32, device="cuda")
    for chunks in (1, 2, 1, 2):
        sc.set_chunks(chunks)
        for _ in range(3):
            st = sc.fabrik_device(pts, ang, it, None, 1e-3, 100)
        torch.cuda.synchronize()
        print(f"chunks {chunks}: gather_ms {st.gather_ms:.3f}", flush=True)
    sc.close()


def summary(d):
    import csv
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    keep = [r for r in rows if any(k in r["Kernel_Name"] for k in
                                   ("fabrik_iter", "loopback_gather", "fabrik_classify",
                                    "fabrik_scatter", "pack_tail"))]
    t0 = int(keep[0]["Start_Timestamp"]) if keep else 0
    for r in keep[-40:]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].split("(")[0].split("::")[-1][:28]
        print(f"{name:30s} {s / 1e3:10.1f} {e / 1e3:10.1f} us  ({(e - s) / 1e3:7.1f})")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
