"""bench.py's cpu_baseline leg on the CPU (no GPU): the oracle timed on a bounded
sample, its thread count, and the parity fields it computes against a GPU batch
(here the oracle's own output stands in for the GPU's)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class _Args:
    tol = 1e-3
    max_iter = 100
    cpu_seconds = 0.2


def test_fabrik_cpu_baseline_threads_and_parity():
    import bench
    from oracle import oracle as O
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(4096, seed=0)
    ang, it, _, _ = O.fabrik_ikine(pts, 1e-3, 100)
    r = bench.cpu_baseline("fabrik", _Args(), sample_pts=pts, gpu_out={"ang": ang, "iters": it})
    assert r["kind"] == "port" and r["unit"] == "IK solutions/s" and r["value"] > 0
    assert 1 <= r["cores"] <= (os.cpu_count() or 1)
    assert r["parity"]["ok"] and r["parity"]["iters_equal"] == 4096
    assert r["parity"]["max_abs_diff"] == 0.0
    bad = it.copy()
    bad[7] += 1
    r = bench.cpu_baseline("fabrik", _Args(), sample_pts=pts, gpu_out={"ang": ang, "iters": bad})
    assert not r["parity"]["ok"] and r["parity"]["iters_equal"] == 4095


def test_ann_cpu_baseline_parity_fields():
    import bench
    from inversekinematicsann_amd.robot.position_generator import random_dist
    pts = random_dist(8192, seed=0)
    r = bench.cpu_baseline("ann", _Args(), sample_pts=pts)
    ref = r.pop("_ref")
    assert ref.shape == (8192, 4) and r["value"] > 0 and r["cores"] >= 1
    r = bench.cpu_baseline("ann", _Args(), sample_pts=pts,
                           gpu_out={"ang": ref.astype(np.float32)})
    assert r["parity"]["ok"] and r["parity"]["max_abs_diff_vs_oracle_fp32"] <= 1e-6


def test_launch_command_for_n_gpus():
    """`bench.py --gpus 8` runs 8 ranks itself through torch.distributed.run on
    127.0.0.1, passing its own arguments through (the driver calls
    `python3 bench.py --gpus N` with no launcher)."""
    import bench
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "1"]
    cmd = bench.launch_command(argv, 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py") and cmd[-len(argv):] == argv
    assert bench._gpus_arg(["--gpus=4"]) == 4 and bench._gpus_arg([]) == 1


def test_maybe_launch_spawns_child_not_exec(monkeypatch):
    import subprocess
    import bench
    seen = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.append((cmd, env)) or 3)
    assert bench.maybe_launch(["--gpus", "2", "--gather", "0"]) == 3  # the child's exit code
    (cmd, env), = seen
    assert "--nproc-per-node=2" in cmd and cmd[-3:] == ["--gpus", "2", "--gather", "0"][-3:]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.maybe_launch(["--gpus", "1"]) is None  # N = 1: this process is the bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(["--gpus", "2"]) is None  # already a rank
    assert len(seen) == 1


def test_rank_count_mismatch_exits_nonzero():
    """A rank whose WORLD_SIZE differs from --gpus never prints a line."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and p.stdout == ""
    assert "--gpus 8 but 1 rank" in p.stderr


def test_gather_check_compare_rows_bitwise():
    """compare_rows: bit-for-bit, row granular (a NaN equals itself by bits; -0.0
    differs from 0.0), over every output of the check."""
    import bench
    a = np.arange(40, dtype=np.float64).reshape(10, 4)
    it = np.arange(10, dtype=np.int32)
    assert bench.compare_rows({"ang": a, "iters": it}, {"ang": a.copy(), "iters": it.copy()}) == \
        (10, 0)
    b = a.copy()
    b[3, 2] = np.nextafter(b[3, 2], np.inf)  # one ulp in one row
    b[7, 0] = -0.0 if a[7, 0] == 0.0 else -a[7, 0]
    assert bench.compare_rows({"ang": a}, {"ang": b}) == (10, 2)
    n = a.copy()
    n[0, 0] = np.nan
    assert bench.compare_rows({"ang": n}, {"ang": n.copy()}) == (10, 0)
    it2 = it.copy()
    it2[9] += 1
    assert bench.compare_rows({"ang": a, "iters": it}, {"ang": a, "iters": it2}) == (10, 1)


def test_gather_verdict_exits_nonzero_on_mismatch():
    """a line whose gathered rows differ from their re-solve
    carries bit_exact false and the bench exits 3; no check (N = 1) is None / 0."""
    import bench
    assert bench.gather_verdict({"ann": None}) == (None, 0)
    ok = {"rows": 100, "mismatched_rows": 0, "bit_exact": True}
    bad = {"rows": 50, "mismatched_rows": 2, "bit_exact": False}
    g, rc = bench.gather_verdict({"ann": ok, "fabrik": ok})
    assert rc == 0 and g["bit_exact"] and g["rows"] == 200
    g, rc = bench.gather_verdict({"ann": ok, "fabrik": bad})
    assert rc == 3 and not g["bit_exact"] and g["rows"] == 150


def test_gather_check_parts_of_the_next_rank():
    """The rows a rank re-solves: rank (r+1) % N's first and last parts in the
    library's plan (chunks from ik_comm_info), and the check over them."""
    import bench
    from inversekinematicsann_amd import dist as D

    class _SC:
        def __init__(self, rank, chunks):
            self.rank, self._c = rank, chunks

        def info(self):
            return (4, self.rank, self._c)

    class _Job:
        world, total = 4, 1003

        def __init__(self, rank, chunks):
            self.sc = _SC(rank, chunks)

    assert bench._check_parts(_Job(0, 1)) == [D.part_bounds(1003, 4, 1, 1, 0)]
    assert bench._check_parts(_Job(3, 1)) == [D.part_bounds(1003, 4, 1, 0, 0)]
    parts = bench._check_parts(_Job(1, 3))
    assert parts == [D.part_bounds(1003, 4, 3, 2, 0), D.part_bounds(1003, 4, 3, 2, 2)]
    # the check over those parts: a gathered array equal to the re-solve passes,
    # one corrupted row of the next rank's last part fails (world 1 here: no
    # torch.distributed, the sums are the rank's own)
    full = np.arange(1003 * 4, dtype=np.float32).reshape(1003, 4)
    job = _Job(1, 3)
    job.world = 4
    res = bench.gather_check(job, {"ang": full}, lambda b, e: {"ang": full[b:e].copy()})
    assert res["bit_exact"] and res["rows"] == sum(e - b for b, e in parts)
    bad = full.copy()
    bad[parts[-1][1] - 1, 3] += 1
    res = bench.gather_check(job, {"ang": bad}, lambda b, e: {"ang": full[b:e].copy()})
    assert not res["bit_exact"] and res["mismatched_rows"] == 1


def test_roofline_fracs_headline_the_lower():
    """both the event and the rocprof figure, the lower one headlined."""
    import bench
    fr = bench.roofline_fracs(100.0, 2000.0, 1000.0, {"rocprof_avg_ms": 2500.0})
    assert abs(fr["frac_events"] - 0.05) < 1e-12 and abs(fr["frac_rocprof"] - 0.04) < 1e-12
    assert fr["headline"] == "rocprof" and abs(fr["_head"] - 40.0) < 1e-9
    fr = bench.roofline_fracs(100.0, 2000.0, 1000.0, {})
    assert fr["headline"] == "events" and fr["frac_rocprof"] is None
    assert bench.roofline_fracs(100.0, None, 1000.0, {})["headline"] is None


def test_strong_legs_are_configs_3_and_4_at_world_8():
    """at N > 1 the bench adds configs[3] (ANN fp32 + FK round trip)
    and configs[4] (FABRIK tol 1e-5 / 200) on the 10M-point batch sharded over the
    ranks, labelled by _config_ref; the weak headline stays configs[1] / [2] and
    one GPU never labels a line configs[3] / [4]."""
    import bench
    args = bench.parse(["--gpus", "8"])
    assert args.strong_legs == 1 and args.total_points == 0
    legs = bench.strong_legs()
    assert set(legs) == {"ann_strong10M", "fabrik_tol1e-5_strong10M"}
    assert bench.STRONG_POINTS == 10_000_000
    r2 = {"ms_per_step": 50.0, "dtype": "fp32", "roofline": {}, "workload": "w", "kernels": {}}
    e = bench.secondary_entry("ann_strong10M", r2, bench.STRONG_POINTS, 8, args)
    assert e["baseline_config"] == "configs[3]" and e["total_points"] == 10_000_000
    assert abs(e["value"] - 10_000_000 / 0.05) < 1e-3
    e = bench.secondary_entry("fabrik_tol1e-5_strong10M", dict(r2, dtype="f64"),
                              bench.STRONG_POINTS, 8, args)
    assert e["baseline_config"] == "configs[4]"
    assert bench.leg_settings("fabrik_tol1e-5_strong10M", args) == ("fabrik", 1e-5, 200)
    # the weak legs at world 8 (1M per GPU) and the split modes
    assert bench.secondary_entry("fabrik", r2, 8_000_000, 8, args)["baseline_config"] == \
        "configs[2]"
    assert "baseline_config" not in bench.secondary_entry("fabrik_tol1e-5", r2, 8_000_000, 8,
                                                          args)
    assert "baseline_config" not in bench.secondary_entry("ann_fp16x3", r2, 8_000_000, 8, args)
    assert bench._config_ref("ann", 8_000_000, 8, 1e-3, 100) == "configs[1]"
    # one GPU: never configs[3] / [4], whatever the batch
    assert bench._config_ref("ann", 10_000_000, 1, 1e-3, 100) is None
    assert bench._config_ref("fabrik", 10_000_000, 1, 1e-5, 200) is None
    for w in (2, 4):
        assert bench._config_ref("ann", 10_000_000, w, 1e-3, 100) == "configs[3]"
        assert bench._config_ref("fabrik", 10_000_000, w, 1e-5, 200) == "configs[4]"


def test_kernel_duration_longer_than_the_untimed_loop_is_dropped():
    """An events duration that fits its own event-timed step but exceeds the untimed
    loop's step by more than 1 % (the event-stamped launch ran slower: FK, r06) is
    not priced: the rocprof window stands alone, and the line says why."""
    import bench
    prof = {"rocprof_avg_ms": 0.407}
    fr = bench.roofline_fracs(1.0e9, 0.452, 8e12, prof, step_ms=0.47, loop_ms=0.413)
    assert not fr["kernel_ms_valid"] and fr["frac_events"] is None and "kernel_ms_note" in fr
    assert fr["headline"] == "rocprof"
    fr = bench.roofline_fracs(1.0e9, 21.55, 8e12, prof, step_ms=21.57, loop_ms=21.52)
    assert fr["kernel_ms_valid"] and "kernel_ms_note" not in fr


def test_kernel_duration_longer_than_its_step_is_dropped():
    """an events duration longer than the step that launched the
    kernel is not a kernel duration; the roofline then rests on rocprof alone."""
    import bench
    assert bench.kernel_time_ok(0.30, 0.36) and not bench.kernel_time_ok(0.52, 0.51)
    assert not bench.kernel_time_ok(None, 0.5) and not bench.kernel_time_ok(0.3, None)
    fr = bench.roofline_fracs(100.0, 0.52, 1000.0, {"rocprof_avg_ms": 0.467}, step_ms=0.511)
    assert fr["frac_events"] is None and not fr["kernel_ms_valid"]
    assert fr["headline"] == "rocprof"
    fr = bench.roofline_fracs(100.0, 0.47, 1000.0, {"rocprof_avg_ms": 0.467}, step_ms=0.511)
    assert fr["kernel_ms_valid"] and fr["frac_events"] is not None


def _lease_lines():
    """Every bench line committed under profiles/r06 (one JSON object per file, or
    JSON lines)."""
    import glob
    import json
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r06", "**", "*bench*.json"),
                              recursive=True)):
        with open(p) as f:
            txt = f.read().strip()
        for ln in ([txt] if txt.startswith("{") and txt.count("\n{") == 0 else txt.splitlines()):
            ln = ln.strip()
            if ln.startswith("{"):
                try:
                    d = json.loads(ln)
                except ValueError:
                    continue
                if "metric" in d and "ms_per_step" in d:
                    out.append((p, d))
    return out


def test_committed_bench_lines_kernel_fits_step():
    """in every committed r06 bench line, each method's roofline
    kernel_ms (the dispatch-stamped events) fits inside the step it was stamped in
    (roofline.event_step_ms, from the bench's last r06 revision; before it the timed
    loop's ms_per_step) and within 0.5 % of the timed loop's step, and where both
    figures exist frac_events is within 5 % of frac_rocprof."""
    lines = _lease_lines()
    for path, d in lines:
        entries = [("headline", d)] + list(d.get("secondary", {}).items())
        for name, e in entries:
            rf, step = e.get("roofline") or {}, e.get("ms_per_step")
            k = rf.get("kernel_ms")
            if k is None or step is None:
                continue
            own = rf.get("event_step_ms")
            if own is not None and rf.get("kernel_ms_valid") is False:
                continue  # (dropped by the line itself: kernel_ms_note says why)
            assert k <= (own if own is not None else step), (path, name, k, own, step)
            assert k <= step * 1.01, (path, name, k, step)
            fe, fr = rf.get("frac_events"), rf.get("frac_rocprof")
            # (against a rocprof profile of this round's kernels only)
            same_round = str(rf.get("profile", "")).startswith("profiles/r06")
            # (a rehearsal whose ranks share one device times each kernel under the
            # other ranks' load: config.devices_shared; its durations still fit)
            shared = bool(d.get("config", {}).get("devices_shared"))
            if fe and fr and same_round and not shared and name in ("headline", "fabrik", "fabrik_tol1e-5", "fk"):
                assert abs(fe / fr - 1.0) <= 0.05, (path, name, fe, fr)


def test_wall_budget_fits_the_driver_limit():
    """`bench.py --gpus 8` (weak headline, secondaries, both strong
    legs, gather checks, end-to-end, cold steps, start-up and RCCL init) fits the
    driver's 600 s limit at its --steps 20 --warmup 5 and at the defaults, and so
    does a run whose collective stalls until IKHIP_RCCL_TIMEOUT_S aborts it."""
    import bench
    for world in (1, 2, 4, 8):
        for steps, warmup in ((20, 5), (10, 2)):
            b = bench.wall_budget(world, steps, warmup)
            assert b["total_s"] <= bench.DRIVER_TIMEOUT_S, (world, b)
            assert b["stall_path_s"] <= bench.DRIVER_TIMEOUT_S, (world, b)
            if world > 1:
                assert {"ann_strong10M", "fabrik_tol1e-5_strong10M"} <= set(b["legs_s"])
    # the library's default deadline (ik_shard.hip) is the one the budget assumes
    src = open(os.path.join(ROOT, "inversekinematicsann_amd", "csrc", "ik_shard.hip")).read()
    assert "env = v > 0.0 ? v : 120.0;" in src


def test_rocprof_median_over_boxes():
    """The committed r06 traffic.json carries each kernel's rocprof window average on
    several boxes (tools/merge_boxes.py: the profiling lease's first, then the
    tools/trace_box.sh boxes) and their median; bench.profile_fields prices
    frac_rocprof on the median and reports the list (a driver box is one more draw)."""
    import statistics
    import bench
    path = os.path.join(ROOT, "profiles", "r06", "traffic.json")
    t = json.load(open(path))
    for k in ("ann_fused_kernel", "fabrik_iter_kernel", "fabrik_tol1e-5/fabrik_iter_kernel",
              "fk_kernel"):
        v = t[k]
        assert len(v["rocprof_boxes_ms"]) >= 4 and v["rocprof_boxes_ms"][0] == v["rocprof_avg_ms"]
        assert v["rocprof_median_ms"] == statistics.median(v["rocprof_boxes_ms"])
        pf = bench.profile_fields(path, k)
        assert pf["rocprof_avg_ms"] == v["rocprof_median_ms"]
        assert pf["rocprof_boxes_ms"] == v["rocprof_boxes_ms"]
    # a profile without the boxes keeps its own window average
    lb = os.path.join(ROOT, "profiles", "r06", "lease_b", "traffic.json")
    pf = bench.profile_fields(lb, "fabrik_iter_kernel")
    assert pf["rocprof_avg_ms"] == json.load(open(lb))["fabrik_iter_kernel"]["rocprof_avg_ms"]
    assert "rocprof_boxes_ms" not in pf
