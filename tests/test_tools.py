"""Measurement tooling on CPU: the PMC summary keeps only the timed launch
shape (tools/pmc_summary.py), and the committed summaries bench.py reads are
physically consistent (a kernel that stores every pixel once writes at least
the bytes it stores)."""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_summary  # noqa: E402

BIG = "void rtamd::render_kernel<0, false, true, 18>(rtamd::LaunchParams)"
ONE = "void rtamd::render_kernel<0, false, false, 18>(rtamd::LaunchParams)"
TRACE_COLS = ["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Scratch_Size",
              "VGPR_Count", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
PMC_COLS = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
            "End_Timestamp"]


def _write(path, cols, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _profile(tmp_path, launches):
    """A synthetic profile: launches = [(name, grid, duration_ns, write_kib)]
    in dispatch order, plus a fill kernel that is not ours."""
    trace, wr, sq = [], [], []
    t = 1000
    for i, (name, grid, dur, kib) in enumerate(launches, start=1):
        trace.append({"Kind": "KERNEL_DISPATCH", "Dispatch_Id": i, "Kernel_Name": name, "Start_Timestamp": t,
                      "End_Timestamp": t + dur, "Scratch_Size": 0, "VGPR_Count": 32, "Grid_Size_X": grid,
                      "Grid_Size_Y": 1, "Grid_Size_Z": 1})
        wr.append({"Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name, "Counter_Name": "WRITE_SIZE",
                   "Counter_Value": kib, "Start_Timestamp": t, "End_Timestamp": t + dur})
        sq.append({"Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name, "Counter_Name": "SQ_INSTS_VALU",
                   "Counter_Value": kib * 10, "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 10
    trace.append({"Kind": "KERNEL_DISPATCH", "Dispatch_Id": 99, "Kernel_Name": "__amd_rocclr_fillBufferAligned",
                  "Start_Timestamp": t, "End_Timestamp": t + 5, "Scratch_Size": 0, "VGPR_Count": 8,
                  "Grid_Size_X": 64, "Grid_Size_Y": 1, "Grid_Size_Z": 1})
    _write(tmp_path / "trace_kernel_trace.csv", TRACE_COLS, trace)
    _write(tmp_path / "pmc_write_counter_collection.csv", PMC_COLS, wr)
    _write(tmp_path / "pmc_sq_counter_collection.csv", PMC_COLS, sq)
    return str(tmp_path)


def test_two_launch_shapes_are_not_averaged(tmp_path):
    """Round 5's config-2 PMC pass held 55 256-frame launches and 3 single
    verification frames; their plain average put 'traffic' below the stored
    bytes. Only the timed shape may count."""
    launches = [(BIG, 1000, 7_000_000, 8_294_400)] * 55 + [(ONE, 4, 40_000, 32_400)] * 3
    o = pmc_summary.summarise(_profile(tmp_path, launches), "config2", 256)
    assert o["write_bytes_per_launch"] == 8_294_400 * 1024
    assert o["avg_kernel_ns"] == 7_000_000
    assert o["calls"] == 55
    assert o["sq_insts_valu_per_launch"] == 82_944_000
    assert o["dispatch_selection"]["pmc_write"]["dropped"]["other_shapes"] == 3


def test_same_grid_shorter_launches_and_warmup_dropped(tmp_path):
    """Queued launches of 1 and 7 views share symbol and grid: the short
    ones are another shape; --skip drops the warm-up launches."""
    k = "void rtamd::render_kernel<2, false, false, 48>(rtamd::LaunchParams)"
    launches = ([(k, 393216, 5_700_000, 700)] * 2 + [(k, 393216, 4_600_000, 700)] * 10 +
                [(k, 393216, 700_000, 100)] * 3)
    o = pmc_summary.summarise(_profile(tmp_path, launches), "config3", 7, skip=2)
    assert o["calls"] == 10
    assert o["avg_kernel_ns"] == 4_600_000
    assert o["write_bytes_per_launch"] == 700 * 1024
    sel = o["dispatch_selection"]["trace"]["dropped"]
    assert sel == {"other_shapes": 0, "short_in_shape": 3, "warmup": 2}


@pytest.mark.parametrize("workload", ["config2", "config3", "config4", "config5", "shipped"])
def test_committed_summaries_write_what_they_store(workload):
    """A render launch stores every pixel once: a committed summary whose
    WRITE_SIZE is below the launch's stored bytes mixes launch shapes."""
    path = os.path.join(ROOT, "profiles", "pmc_%s_latest.json" % workload)
    if not os.path.exists(path):
        pytest.skip("no committed summary for %s" % workload)
    d = json.load(open(path))
    sys.path.insert(0, ROOT)
    import bench
    cfg = bench.WORKLOADS[workload]
    stored = cfg["width"] * cfg["height"] * 16 * d.get("frames_per_launch", 1)
    assert d["write_bytes_per_launch"] >= 0.99 * stored, (d["write_bytes_per_launch"], stored)
    assert "dispatch_selection" in d


def test_bench_refuses_a_summary_that_writes_less_than_it_stores():
    """bench.py's traffic check: round 5's config-2 summary (8.056 GB written
    for a 256-frame launch that stores 8.493 GB) is left out of the line;
    the round-6 one (8.493 GB) is kept."""
    sys.path.insert(0, ROOT)
    import bench
    stored = 256 * 1920 * 1080 * 16
    pmc, rec = bench.check_traffic({"write_bytes_per_launch": 8.056e9, "hbm_bytes_per_launch": 8.058e9}, stored)
    assert pmc == {} and rec["ok"] is False
    good = {"write_bytes_per_launch": 8493465600.0, "hbm_bytes_per_launch": 8.4955e9}
    pmc, rec = bench.check_traffic(good, stored)
    assert pmc is good and rec["ok"] is True
    assert bench.check_traffic({}, stored) == ({}, None)
