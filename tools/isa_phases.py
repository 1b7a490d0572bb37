"""Instruction census of the FABRIK iteration kernel by phase:
an analysis build of ik_fabrik.hip with -DIKHIP_PHASE_MARKS carries an assembly
comment ';@phase <name>' at each phase boundary (IKHIP_MARK); this counts the
VALU / fp64 / SALU / LDS / VMEM instructions from each mark to the next one in
the kernel's assembly text, and the phase's out-of-line blocks (branch targets
between the two marks that lie elsewhere are not followed: the counts are the
straight-line path, which is what a phase runs when no lane leaves the core
sequences).  Development aid; the production build has no marks.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DIKHIP_PHASE_MARKS \\
          --cuda-device-only -S inversekinematicsann_amd/csrc/ik_fabrik.hip -o fab_marks.s
    python tools/isa_phases.py fab_marks.s [kernel-substring] [--json out.json]
"""
import json
import re
import sys

KERNEL = "_ZN5ikhip18fabrik_iter_kernelILi12ELb1ELi2EEEvNS_7FabArgsE"


def census(path, kern=KERNEL):
    s = open(path).read()
    k = s.index(kern + ":")
    e = s.index(".Lfunc_end", k)
    phases, cur = [], None
    for line in s[k:e].split("\n"):
        m = re.search(r";@phase (\S+)", line)
        if m:
            cur = {"phase": m.group(1), "n": 0, "valu": 0, "f64": 0, "salu": 0, "lds": 0,
                   "vmem": 0, "trans": 0}
            phases.append(cur)
            continue
        t = line.strip()
        if cur is None or not line.startswith("\t") or t.startswith(".") or t.startswith(";"):
            continue
        op = t.split()[0]
        cur["n"] += 1
        if op.startswith("v_"):
            cur["valu"] += 1
            if "f64" in op:
                cur["f64"] += 1
            if any(x in op for x in ("rsq", "rcp", "sqrt", "exp", "log", "sin", "cos")):
                cur["trans"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cur["vmem"] += 1
    return phases


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out in args:
        args.remove(out)
    ph = census(args[0], args[1] if len(args) > 1 else KERNEL)
    print(f"{'phase (text order)':22s} {'instr':>6s} {'valu':>6s} {'f64':>6s} {'trans':>6s} "
          f"{'salu':>6s} {'lds':>5s} {'vmem':>5s}")
    for p in ph:
        print(f"{p['phase']:22s} {p['n']:6d} {p['valu']:6d} {p['f64']:6d} {p['trans']:6d} "
              f"{p['salu']:6d} {p['lds']:5d} {p['vmem']:5d}")
    if out:
        with open(out, "w") as f:
            json.dump(ph, f, indent=1)


if __name__ == "__main__":
    main()
