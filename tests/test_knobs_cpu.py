"""the compile-time knobs are self-documenting.  Every
`#ifndef IKHIP_X` / `#define IKHIP_X v` pair in the library's sources has a row in
INTEGRATION.md's macro table with the same default, every row names a macro the
sources define, and no macro selecting a path documented as slower or wrong is
left (the r04 alternatives were deleted, their A/Bs kept in DESIGN_HISTORY.md)."""
import glob
import os
import re

from tests.conftest import ROOT

CSRC = os.path.join(ROOT, "inversekinematicsann_amd", "csrc")
# build-wide switches that are not tuning knobs: the diagnostic build and the two
# translation units that re-include ik_ann.hip
NOT_KNOBS = {"IKHIP_DIAG", "IKHIP_ANN_WIDE", "IKHIP_ANN_X_TU", "IKHIP_PHASE_MARKS"}
DELETED = {"IKHIP_EXP_L1W", "IKHIP_FAB_FUSED_SCATTER", "IKHIP_FAB_PREP_CARRY", "IKHIP_ANN_CLAIM",
           "IKHIP_ANN_H16", "IKHIP_ANN_X16", "IKHIP_ANN_DYN", "IKHIP_ANN_HSWZ",
           "IKHIP_ANN_BIAS_FIRST", "IKHIP_ANN_H16_PATTERN", "IKHIP_ANN_X16_PATTERN",
           "IKHIP_ANN_XRING", "IKHIP_FAB_INNER", "IKHIP_FAB_REFILL_PRIO", "IKHIP_FAB_FAST_ANGLES"}


def source_knobs():
    knobs = {}
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
                    + glob.glob(os.path.join(CSRC, "*.cpp"))):
        src = open(f).read()
        for name, val in re.findall(r"^#ifndef (IKHIP_\w+)[^\n]*\n#define \1 ([^\n/]+)", src, re.M):
            assert name not in knobs, f"{name} defined twice"
            knobs[name] = val.strip()
    return knobs


def doc_knobs():
    src = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = src.index("| Macro | Default | What it sets |")
    rows = {}
    for line in src[i:].splitlines()[2:]:
        if not line.startswith("|"):
            break
        cells = [c.strip() for c in line.strip("|").split("|")]
        rows[cells[0].strip("`")] = cells[1]
    return rows


def test_every_knob_documented_with_its_default():
    src, doc = source_knobs(), doc_knobs()
    assert src, "no knobs parsed"
    assert set(src) == set(doc), (sorted(set(src) ^ set(doc)))
    for k, v in src.items():
        assert doc[k] == v, (k, "source", v, "INTEGRATION.md", doc[k])


def test_no_dropped_alternative_left():
    text = ""
    for f in glob.glob(os.path.join(CSRC, "*")):
        if f.endswith((".hip", ".h", ".cpp")):
            text += open(f).read()
    used = set(re.findall(r"\bIKHIP_[A-Z0-9_]+", text))
    assert not (used & DELETED), sorted(used & DELETED)
    # every IKHIP_ name in the sources is a documented knob, a build switch, a
    # diagnostic macro or an environment variable documented in INTEGRATION.md
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for name in sorted(used - NOT_KNOBS - set(source_knobs())):
        if name in ("IKHIP_DG", "IKHIP_DT", "IKHIP_DT_ACC", "IKHIP_MARK"):  # diagnostic / census builds
            continue
        assert f"`{name}`" in doc, name
