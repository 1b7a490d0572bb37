"""Iteration-kernel counters of the FABRIK pipeline (diagnostic build
libikhip_diag.so, IKHIP_LIB=...): lane efficiency (useful lane-steps / 64 x
wave-steps), refills and chunk grabs per wave, the core-path fallbacks, and the
spread of wave start / end times (the launch tail).  Diagnostic only."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("IKHIP_LIB", os.path.join(ROOT, "inversekinematicsann_amd",
                                                "libikhip_diag.so"))
from inversekinematicsann_amd import _native  # noqa: E402
from inversekinematicsann_amd.robot.position_generator import random_dist  # noqa: E402

NAMES = ["loops", "steps", "lane_steps", "refills", "grabs", "fallbacks", "waves", "flushes",
         "flush_ticks", "prep_ticks", "refill_ticks", "park_ticks", "stage_ticks"]
REC = 24  # words per wave record (ik_fabrik.hip kDiagWords)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pts = torch.from_numpy(random_dist(n, seed=0)).cuda()
ang = torch.empty((n, 4), dtype=torch.float64, device="cuda")
it = torch.empty(n, dtype=torch.int32, device="cuda")
ctx = _native.Context(0)
out = {}
for tol, mi in ((1e-3, 100), (1e-5, 200)):
    for _ in range(3):  # the work order learns its cost table
        ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=_native.IK_F_DEVICE)
    ctx.set_debug(True)
    ctx.fabrik_solve_device(pts, ang, it, None, tol, mi, flags=_native.IK_F_DEVICE)
    w = ctx.debug_words(64 + REC * 4096).astype(np.int64)
    ctx.set_debug(False)
    c = dict(zip(NAMES, w[:len(NAMES)].tolist()))
    nw = min(c["waves"], 4096)
    t = w[64:64 + REC * nw].reshape(nw, REC)
    # per-wave record: the counters, then start, dry, last step, steps after
    # dry, drain, end (s_memrealtime, 100 MHz)
    T0, TDRY, TLAST, SDRY, TDRAIN, TEND = range(len(NAMES), len(NAMES) + 6)
    t0 = t[:, T0].min()
    if os.environ.get("FABRIK_DIAG_RAW"):  # the per-wave records, for offline analysis
        np.save(os.path.join(os.environ["FABRIK_DIAG_RAW"], f"fabrik_diag_raw_tol{tol:g}.npy"), t)
    pc = [0, 1, 10, 50, 90, 99, 100]
    us = lambda v: np.percentile((v - t0) / 100.0, pc).round(1).tolist()
    span = lambda a, b: np.percentile((t[:, b] - t[:, a]) / 100.0, pc).round(2).tolist()
    c["lane_eff"] = c["lane_steps"] / (64.0 * max(c["steps"], 1))
    c["sum_iters"] = int(it.sum().item())
    c["steps_per_refill"] = c["steps"] / max(c["refills"], 1)
    c["flush_us_per_wave"] = c["flush_ticks"] / 100.0 / max(c["waves"], 1)
    c["prep_us_per_wave"] = c["prep_ticks"] / 100.0 / max(c["waves"], 1)
    for k in ("refill", "park", "stage"):
        c[k + "_us_per_wave"] = c[k + "_ticks"] / 100.0 / max(c["waves"], 1)
    # the refill's rest: handing prepared entries to the free lanes
    c["handout_us_per_wave"] = c["refill_us_per_wave"] - c["park_us_per_wave"] - c["stage_us_per_wave"]
    c["pct"] = pc
    c["wave_start_us"] = us(t[:, T0])
    c["wave_dry_us"] = us(t[:, TDRY])       # queue and the wave's batch exhausted
    c["wave_last_step_us"] = us(t[:, TLAST])
    c["wave_drain_us"] = us(t[:, TDRAIN])   # loop left
    c["wave_end_us"] = us(t[:, TEND])       # after the final angles step
    c["steps_after_dry"] = np.percentile(t[:, SDRY], pc).tolist()
    c["dry_to_last_step_us"] = span(TDRY, TLAST)
    c["last_step_to_drain_us"] = span(TLAST, TDRAIN)
    c["drain_to_end_us"] = span(TDRAIN, TEND)
    c["wave_us"] = span(T0, TEND)
    # the drain: entries parked + flushed at the end, the optional first flush
    # (ring overflow) and the final one; the slowest 10 % of drains against the rest
    DRAINN, TDRAIN2 = T0 + 8, T0 + 9
    dn = t[:, DRAINN]
    d1 = (t[:, TDRAIN2] - t[:, TDRAIN]) / 100.0
    d2 = (t[:, TEND] - t[:, TDRAIN2]) / 100.0
    dd = (t[:, TEND] - t[:, TDRAIN]) / 100.0
    slow = dd >= np.percentile(dd, 90)
    c["drain_entries"] = np.percentile(dn, pc).tolist()
    c["drain_first_flush_us"] = np.percentile(d1, pc).round(2).tolist()
    c["drain_final_flush_us"] = np.percentile(d2, pc).round(2).tolist()
    c["drain_slow10"] = {"entries_median": float(np.median(dn[slow])),
                         "entries_median_rest": float(np.median(dn[~slow])),
                         "first_us_median": float(np.median(d1[slow])),
                         "final_us_median": float(np.median(d2[slow])),
                         "dry_us_median": float(np.median((t[slow, TDRY] - t0) / 100.0)),
                         "dry_us_median_rest": float(np.median((t[~slow, TDRY] - t0) / 100.0)),
                         "slot_in_block": np.bincount(np.arange(nw)[slow] % 4, minlength=4).tolist()}
    # block-mates (same CU) already finished when a wave's drain starts
    blk = np.arange(nw) // 4
    mates_done = np.array([int(((blk == blk[w]) & (t[:, TEND] < t[w, TDRAIN])).sum())
                           for w in range(nw)])
    c["drain_slow10"]["mates_done_hist"] = np.bincount(mates_done[slow], minlength=4).tolist()
    c["drain_rest_mates_done_hist"] = np.bincount(mates_done[~slow], minlength=4).tolist()
    # by XCD (blocks are dealt round-robin over the 8 XCDs; 4 waves per block):
    # median dry / end time, to tell clock domains from backlogs
    xcd = (np.arange(nw) // 4) % 8
    c["dry_us_by_xcd"] = [round(float(np.median((t[xcd == x, TDRY] - t0) / 100.0)), 1)
                          for x in range(8)]
    c["end_us_by_xcd"] = [round(float(np.median((t[xcd == x, TEND] - t0) / 100.0)), 1)
                          for x in range(8)]
    c["end_p99_us_by_xcd"] = [round(float(np.percentile((t[xcd == x, TEND] - t0) / 100.0, 99)), 1)
                              for x in range(8)]
    # busy waves over time (10 us bins): how the launch drains
    edges = np.arange(0, (t[:, TEND].max() - t0) / 100.0 + 10, 10)
    c["waves_running_10us"] = [int(((t[:, T0] - t0) / 100.0 <= e).sum() -
                                   ((t[:, TEND] - t0) / 100.0 <= e).sum()) for e in edges]
    out[f"tol{tol:g}"] = c
print(json.dumps(out, indent=1))
