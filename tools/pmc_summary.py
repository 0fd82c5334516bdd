"""Summarise a tools/profile.sh run into profiles/ (JSON + CSV copies).

HBM bytes per launch of the render kernel from the PMC passes, with the
gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md (§HBM):
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores; FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled.

Every figure belongs to ONE launch shape: the timed launch of the profiled
bench run. A bench run also makes other render launches (the N = 1
verification renders of single frames, a pipelined or RGBA8 pass), so the
render dispatches of every pass are grouped by (kernel symbol, grid size) —
both columns of rocprofv3's kernel-trace and counter CSVs — and only the
group with the most kernel time in the trace is kept. Queued launches of 1
and of 7 views share their symbol and grid (the grid is the resident
work-groups), so within the group a dispatch shorter than 0.6 x the group's
median duration is dropped as another shape; `--skip N` drops the group's
first N dispatches (the bench's warm-up launches, at the clock's ramp).
`avg_kernel_ns` is the mean over the same dispatches of the trace pass.
The summary lists what it kept and dropped (`dispatch_selection`).

With --frames N every figure is the sum over the kept dispatches divided by
the N frames the profiled bench run rendered, i.e. per frame; without it,
per dispatch.

usage: python tools/pmc_summary.py SRC DST [FRAMES_PER_LAUNCH] [WORKLOAD] [--frames N] [--skip N]
(FRAMES_PER_LAUNCH: views per render launch of the profiled bench run, default 8;
WORKLOAD: bench.py --workload of the run, default config2). Writes
profiles/pmc_<WORKLOAD>_latest.json (bench.py reads it) and, for config2,
profiles/pmc_latest.json.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

KERNELS = ("render_kernel",)
SHORT_FRACTION = 0.6  # a kept dispatch lasts at least this share of its group's median
PASSES = ("pmc_write", "pmc_fetch", "pmc_sq", "pmc_cyc", "pmc_l2", "pmc_lds")


def ours(name):
    return any(k in name for k in KERNELS)


def _grid(r):
    """rocprofv3 writes Grid_Size (total work-items) in counter CSVs and
    Grid_Size_X/Y/Z in the kernel trace: one comparable number."""
    if r.get("Grid_Size"):
        return int(float(r["Grid_Size"]))
    return int(r.get("Grid_Size_X") or 1) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)


def _dur(r):
    try:
        return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    except (KeyError, ValueError):
        return 0


def select(dispatches, skip=0):
    """dispatches: list of (dispatch_id, shape, duration_ns), in dispatch
    order. Returns (shape, kept dispatch ids, dropped dict): the shape with
    the most total duration; within it, dispatches shorter than
    SHORT_FRACTION x the shape's median dropped, then the first `skip`."""
    if not dispatches:
        return None, [], {}
    total = defaultdict(int)
    for _, shape, d in dispatches:
        total[shape] += d
    shape = max(total, key=lambda s: total[s])
    mine = [(i, d) for i, s, d in dispatches if s == shape]
    med = statistics.median(d for _, d in mine)
    kept = [i for i, d in mine if d >= SHORT_FRACTION * med]
    short = len(mine) - len(kept)
    warm = kept[:skip]
    kept = kept[skip:]
    return shape, kept, {"other_shapes": len(dispatches) - len(mine), "short_in_shape": short, "warmup": len(warm)}


def trace_dispatches(src):
    """(dispatch_id, (symbol, grid), duration) of our kernels in the trace pass."""
    path = os.path.join(src, "trace_kernel_trace.csv")
    out = []
    if os.path.exists(path):
        for r in csv.DictReader(open(path)):
            if ours(r.get("Kernel_Name", "")):
                out.append((int(r["Dispatch_Id"]), (r["Kernel_Name"], _grid(r)), _dur(r)))
    out.sort()
    return out


def counters(src, name, skip=0):
    """counter -> list of per-dispatch values of the selected launch shape
    of one PMC pass (its own dispatch ids and durations), plus the
    selection record."""
    path = os.path.join(src, name + "_counter_collection.csv")
    agg = defaultdict(dict)
    if not os.path.exists(path):
        return {}, None
    rows = [r for r in csv.DictReader(open(path)) if ours(r["Kernel_Name"])]
    disp = {}
    for r in rows:
        disp[int(r["Dispatch_Id"])] = ((r["Kernel_Name"], _grid(r)), _dur(r))
    shape, kept, dropped = select([(i, s, d) for i, (s, d) in sorted(disp.items())], skip)
    keep = set(kept)
    for r in rows:
        i = int(r["Dispatch_Id"])
        if i in keep:
            agg[r["Counter_Name"]][i] = float(r["Counter_Value"])
    sel = {"shape": {"kernel": shape[0], "grid_size": shape[1]} if shape else None, "kept": len(kept),
           "dropped": dropped}
    return {k: list(v.values()) for k, v in agg.items()}, sel


def summarise(src, workload="config2", frames_per_launch=8, frames=None, skip=0):
    def per_launch(vals):
        if not vals:
            return None
        return sum(vals) / frames if frames else sum(vals) / len(vals)

    tr = trace_dispatches(src)
    shape, kept, dropped = select(tr, skip)
    keep = set(kept)
    durs = [d for i, s, d in tr if i in keep]
    kernel_ns = None
    if durs:
        kernel_ns = sum(durs) / frames if frames else sum(durs) / len(durs)
    selection = {"trace": {"shape": {"kernel": shape[0], "grid_size": shape[1]} if shape else None,
                           "kept": len(kept), "dropped": dropped}}
    # registers and scratch of the selected kernel (kernel-trace columns)
    res = {}
    tpath = os.path.join(src, "trace_kernel_trace.csv")
    if os.path.exists(tpath) and shape:
        for r in csv.DictReader(open(tpath)):
            if r.get("Kernel_Name") == shape[0]:
                short = r["Kernel_Name"].split("(")[0].split("::")[-1]
                res[short] = {key: r[key] for key in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                      "Private_Segment_Size", "Scratch_Size", "LDS_Block_Size",
                                                      "Group_Segment_Size") if key in r and r[key] != ""}
                break
    build = None
    blog = os.path.join(src, "bench_trace.log")
    if os.path.exists(blog):
        for line in open(blog):
            if line.startswith("{"):
                try:
                    build = json.loads(line).get("build")
                except ValueError:
                    pass
    passes = {}
    for name in PASSES:
        vals, sel = counters(src, name, skip)
        passes[name] = vals
        if sel is not None:
            selection[name] = sel
    w, f, sq, cyc, l2 = (passes[n] for n in ("pmc_write", "pmc_fetch", "pmc_sq", "pmc_cyc", "pmc_l2"))
    write_b = per_launch(w.get("WRITE_SIZE", []))
    write_b = write_b * 1024 if write_b is not None else None
    fetch_b = per_launch(f.get("FETCH_SIZE", []))
    fetch_b = fetch_b * 1024 * 2 if fetch_b is not None else None
    scratch = [int(v.get("Scratch_Size") or v.get("Private_Segment_Size") or 0) for v in res.values()]
    out = {
        "workload": workload, "n_gpus": 1, "frames_per_launch": frames_per_launch, "build": build,
        "per": "frame (the selected launches of %d frames)" % frames if frames else
               "dispatch of the timed launch shape (dispatch_selection)",
        "dispatch_selection": selection,
        "kernel_resources": res,
        "scratch_bytes_per_lane": max(scratch) if scratch else None,
        "kernel": shape[0] if shape else None,
        "avg_kernel_ns": kernel_ns, "calls": len(kept),
        "write_bytes_per_launch": write_b, "fetch_bytes_per_launch": fetch_b,
        "hbm_bytes_per_launch": (write_b or 0) + (fetch_b or 0) if write_b is not None else None,
        "sq_insts_valu_per_launch": per_launch(sq.get("SQ_INSTS_VALU", [])),
        "sq_insts_salu_per_launch": per_launch(sq.get("SQ_INSTS_SALU", [])),
        "sq_insts_lds_per_launch": per_launch(sq.get("SQ_INSTS_LDS", [])),
        "sq_waves_per_launch": per_launch(sq.get("SQ_WAVES", [])),
        "sq_wave_cycles_per_launch": per_launch(cyc.get("SQ_WAVE_CYCLES", [])),
        "sq_busy_cycles_per_launch": per_launch(cyc.get("SQ_BUSY_CYCLES", [])),
        "sq_wait_inst_any_per_launch": per_launch(cyc.get("SQ_WAIT_INST_ANY", [])),
        "sq_wait_any_per_launch": per_launch(cyc.get("SQ_WAIT_ANY", [])),
        "grbm_gui_active_per_launch": per_launch(cyc.get("GRBM_GUI_ACTIVE", [])),
        "l2_hit_per_launch": per_launch(l2.get("TCC_HIT_sum", [])),
        "l2_miss_per_launch": per_launch(l2.get("TCC_MISS_sum", [])),
        "notes": "WRITE_SIZE*1024 exact for 16-B/lane stores; FETCH_SIZE*1024*2 (gfx950 half-count); "
                 "GRBM_GUI_ACTIVE summed over 8 XCDs; every figure over the timed launch shape only",
    }
    if out["grbm_gui_active_per_launch"] and out["avg_kernel_ns"]:
        out["effective_clock_ghz"] = out["grbm_gui_active_per_launch"] / 8 / out["avg_kernel_ns"]
    if out["sq_insts_valu_per_launch"] and out["avg_kernel_ns"]:
        # wave64 VALU issue: 2 cycles per instruction per SIMD, 1024 SIMDs
        clk = out.get("effective_clock_ghz") or 2.4
        out["valu_issue_utilisation"] = out["sq_insts_valu_per_launch"] * 2 / (1024 * clk * out["avg_kernel_ns"])
    if out["l2_hit_per_launch"] is not None and out["l2_miss_per_launch"] is not None:
        tot = out["l2_hit_per_launch"] + out["l2_miss_per_launch"]
        out["l2_hit_rate"] = out["l2_hit_per_launch"] / tot if tot else None
    allc = {}
    for name in PASSES:
        for cname, vals in passes[name].items():
            allc[cname] = per_launch(vals)
    out["counters_per_launch"] = allc
    return out


def main(argv):
    argv = list(argv)
    frames = skip = None
    for flag in ("--frames", "--skip"):
        if flag in argv:
            i = argv.index(flag)
            v = int(argv[i + 1])
            del argv[i:i + 2]
            if flag == "--frames":
                frames = v
            else:
                skip = v
    src, dst = argv[0], argv[1]
    frames_per_launch = int(argv[2]) if len(argv) > 2 else 8
    workload = argv[3] if len(argv) > 3 else "config2"
    out = summarise(src, workload, frames_per_launch, frames, skip or 0)
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst + "_pmc.json", "w") as fo:
        json.dump(out, fo, indent=1)
    shutil.copy(os.path.join(src, "trace_kernel_stats.csv"), dst + "_kernel_stats.csv")
    d = os.path.dirname(dst) or "."
    for name in ["pmc_%s_latest.json" % workload] + (["pmc_latest.json"] if workload == "config2" else []):
        with open(os.path.join(d, name), "w") as fo:
            json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
