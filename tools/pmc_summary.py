"""Per-kernel averages of every PMC counter found under the given rocprofv3
--pmc output directories (counter_collection.csv), plus derived ratios.

    python tools/pmc_summary.py DIR [DIR ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(dirs):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    short = name.split("(")[0].split("::")[-1]
                    c = row["Counter_Name"]
                    tot[short][c] += float(row["Counter_Value"])
                    disp[short][c].add(row.get("Dispatch_Id"))
    out = {}
    for k, cs in tot.items():
        avg = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: /8 is the kernel's cycles;
        # the SQ counters are summed over the 1024 SIMDs (MI355X_MICROARCH.md)
        simd_cycles = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
        if simd_cycles and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            avg["MfmaUtil_pct"] = 100 * avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if simd_cycles and "SQ_ACTIVE_INST_VALU" in avg:  # quad-cycles
            avg["ValuActive_pct"] = 100 * 4 * avg["SQ_ACTIVE_INST_VALU"] / simd_cycles
        f64 = [avg.get(f"SQ_INSTS_VALU_{o}_F64") for o in ("ADD", "MUL", "FMA")]
        if simd_cycles and all(v is not None for v in f64):
            # a wave64 fp64 add / mul / fma occupies the SIMD's fp64 pipe 4 cycles
            avg["Fp64PipeBusy_pct"] = 100 * 4 * sum(f64) / simd_cycles
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            avg["L2_hit_pct"] = 100 * avg["TCC_HIT_sum"] / max(1, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        if "TCC_REQ_sum" in avg:
            # L2 requests (128 B lines on gfx950): the L2 read rate is checked against
            # the ~34.5 TB/s the guide measures, with the kernel's duration from the
            # stats pass (tools/pmc_traffic.py) -- here the raw request count per launch
            avg["TCC_REQ_bytes_128B"] = 128 * avg["TCC_REQ_sum"]
        out[k] = avg
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
