"""Copy one lease's outputs (tools/lease.sh, merged into gpurun_out/ or a saved copy)
into profiles/<dest>/: the profile summary (traffic.json, pmc/), the rocprof stats and
trace of the bench command, the default bench line, the traced bench line, the GPU test
log, the FABRIK diagnostic counters and the spread probe's summary and bench lines.

    python tools/save_lease.py SRC DEST     e.g. gpurun_out profiles/r04
"""
import glob
import os
import shutil
import sys


def cp(src, dst):
    if os.path.exists(src):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(src, dst)
        print(dst)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    p = os.path.join(src, "prof")
    for f in glob.glob(os.path.join(p, "summary", "**", "*.json"), recursive=True):
        cp(f, os.path.join(dst, os.path.relpath(f, os.path.join(p, "summary"))))
    for kind in ("kernel_stats", "kernel_trace", "domain_stats"):
        for f in glob.glob(os.path.join(p, "trace", "**", f"*_{kind}.csv"), recursive=True):
            cp(f, os.path.join(dst, "trace", f"{kind}.csv"))
    cp(os.path.join(p, "bench_default.log"), os.path.join(dst, "lease_bench_default.json"))
    cp(os.path.join(p, "trace.log"), os.path.join(dst, "trace", "traced_bench_line.json"))
    cp(os.path.join(p, "steps.txt"), os.path.join(dst, "lease_steps.txt"))
    cp(os.path.join(src, "pytest_gpu.txt"), os.path.join(dst, "pytest_gpu.txt"))
    cp(os.path.join(src, "fabrik_diag.json"), os.path.join(dst, "fabrik_diag.json"))
    s = os.path.join(src, "spread")
    cp(os.path.join(s, "summary.txt"), os.path.join(dst, "spread", "summary.txt"))
    for f in glob.glob(os.path.join(s, "p*.json")):
        cp(f, os.path.join(dst, "spread", os.path.basename(f)))


if __name__ == "__main__":
    main()
