"""Summary of tools/ab_split_r05.sh: per build and mode, the split-mode kernel's
rocprof average over each run's timed window (the last 20 dispatches), the
step time from HIP events, the kernel clock (GRBM_GUI_ACTIVE / 8 over the
dispatch) from the counter pass, and the angles digest."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import counters, durations  # noqa: E402


def main(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        tag = os.path.basename(f)[:-5]
        lib, mode, kind = tag.split("__")
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        kname = f"ann_fused_kernel_{mode}" if mode != "fp32" else "ann_fused_kernel"
        dur = durations(os.path.join(d, tag)).get(kname, [])
        win = [ms for _, ms in dur][-line["steps"]:]
        rec = {"lib": lib, "mode": mode, "run": kind, "event_ms": round(line["ms_per_step"], 4),
               "rocprof_avg_ms": round(sum(win) / len(win), 4) if win else None,
               "sha16": line["angles_sha16"]}
        if kind == "pmc":
            cs = counters(os.path.join(d, tag)).get(kname, {})
            ghz = []
            for did, ms in dur[-line["steps"]:]:
                v = cs.get(did, {}).get("GRBM_GUI_ACTIVE")
                if v:
                    ghz.append(v / 8 / (ms * 1e6))
            rec["clock_ghz"] = round(sum(ghz) / len(ghz), 3) if ghz else None
        rows.append(rec)
    for r in rows:
        print(json.dumps(r))
    for mode in sorted({r["mode"] for r in rows}):
        avg = {}
        for lib in sorted({r["lib"] for r in rows}):
            v = [r["rocprof_avg_ms"] for r in rows if r["lib"] == lib and r["mode"] == mode
                 and r["run"].startswith("t") and r["rocprof_avg_ms"]]
            if v:
                avg[lib] = sum(v) / len(v)
        print(mode, {k: round(v, 4) for k, v in avg.items()})


if __name__ == "__main__":
    main(sys.argv[1])
