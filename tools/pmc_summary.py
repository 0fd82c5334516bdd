"""Summarise a tools/profile.sh run into profiles/ (JSON + CSV copies).

HBM bytes per launch of the render kernel from the PMC passes, with the
gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md (§HBM):
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores; FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled.

With --frames N every figure is the sum over all the render kernel's
dispatches divided by the N frames the profiled bench run rendered (its
--steps + --warmup), i.e. per frame; without it, per dispatch.

usage: python tools/pmc_summary.py SRC DST [FRAMES_PER_LAUNCH] [WORKLOAD] [--frames N]
(FRAMES_PER_LAUNCH: views per render launch of the profiled bench run, default 8;
WORKLOAD: bench.py --workload of the run, default config2). Writes
profiles/pmc_<WORKLOAD>_latest.json (bench.py reads it) and, for config2,
profiles/pmc_latest.json.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

argv = [a for a in sys.argv[1:]]
frames = None
if "--frames" in argv:
    i = argv.index("--frames")
    frames = int(argv[i + 1])
    del argv[i:i + 2]
src, dst = argv[0], argv[1]
frames_per_launch = int(argv[2]) if len(argv) > 2 else 8
workload = argv[3] if len(argv) > 3 else "config2"
KERNELS = ("render_kernel",)


def ours(name):
    return any(k in name for k in KERNELS)


def counters(name):
    """counter -> list of per-dispatch values of our kernels"""
    path = os.path.join(src, name + "_counter_collection.csv")
    agg = defaultdict(list)
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if ours(r["Kernel_Name"]):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def per_launch(vals):
    if not vals:
        return None
    return sum(vals) / frames if frames else sum(vals) / len(vals)


stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace_kernel_stats.csv"))):
    stats[r["Name"]] = r
k = [v for n, v in stats.items() if ours(n)]
kernel_ns = None
breakdown = {}
if k:
    if frames:
        kernel_ns = sum(float(v["TotalDurationNs"]) for v in k) / frames
        for v in k:
            breakdown[v["Name"]] = {"calls": int(v["Calls"]), "ns_per_frame": float(v["TotalDurationNs"]) / frames}
    else:
        kernel_ns = float(k[0]["AverageNs"])
# registers and scratch of the dispatched kernels (kernel-trace columns)
res = {}
tpath = os.path.join(src, "trace_kernel_trace.csv")
if os.path.exists(tpath):
    for r in csv.DictReader(open(tpath)):
        if ours(r.get("Kernel_Name", "")):
            short = r["Kernel_Name"].split("(")[0].split("::")[-1]
            if short in res:
                continue
            res[short] = {key: r[key] for key in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                  "Private_Segment_Size", "Scratch_Size", "LDS_Block_Size",
                                                  "Group_Segment_Size") if key in r and r[key] != ""}
build = None
blog = os.path.join(src, "bench_trace.log")
if os.path.exists(blog):
    for line in open(blog):
        if line.startswith("{"):
            try:
                build = json.loads(line).get("build")
            except ValueError:
                pass
w, f, sq, cyc = counters("pmc_write"), counters("pmc_fetch"), counters("pmc_sq"), counters("pmc_cyc")
l2 = counters("pmc_l2")
write_b = per_launch(w.get("WRITE_SIZE", []))
write_b = write_b * 1024 if write_b is not None else None
fetch_b = per_launch(f.get("FETCH_SIZE", []))
fetch_b = fetch_b * 1024 * 2 if fetch_b is not None else None
scratch = [int(v.get("Scratch_Size") or v.get("Private_Segment_Size") or 0) for v in res.values()]
out = {
    "workload": workload, "n_gpus": 1, "frames_per_launch": frames_per_launch, "build": build,
    "per": "frame (all render kernels of %d frames)" % frames if frames else "dispatch of the render kernel",
    "kernel_resources": res,
    "scratch_bytes_per_lane": max(scratch) if scratch else None,
    "kernel": [v["Name"] for v in k] if frames else (k[0]["Name"] if k else None),
    "kernel_breakdown": breakdown or None,
    "avg_kernel_ns": kernel_ns, "calls": sum(int(v["Calls"]) for v in k) if k else None,
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
             "GRBM_GUI_ACTIVE summed over 8 XCDs",
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
for name in ("pmc_write", "pmc_fetch", "pmc_sq", "pmc_cyc", "pmc_l2", "pmc_lds"):
    for cname, vals in counters(name).items():
        allc[cname] = per_launch(vals)
out["counters_per_launch"] = allc
os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
with open(dst + "_pmc.json", "w") as fo:
    json.dump(out, fo, indent=1)
shutil.copy(os.path.join(src, "trace_kernel_stats.csv"), dst + "_kernel_stats.csv")
d = os.path.dirname(dst) or "."
for name in ["pmc_%s_latest.json" % workload] + (["pmc_latest.json"] if workload == "config2" else []):
    with open(os.path.join(d, name), "w") as fo:
        json.dump(out, fo, indent=1)
print(json.dumps(out, indent=1))
