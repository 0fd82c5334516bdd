"""Summarise a tools/profile.sh run into profiles/ (JSON + CSV copies).

HBM bytes per launch of the render kernel from the PMC passes, with the
gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md (§HBM):
WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores; FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled.

usage: python tools/pmc_summary.py gpurun_out/prof/r01 profiles/r01 [FRAMES_PER_LAUNCH] [WORKLOAD]
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

src, dst = sys.argv[1], sys.argv[2]
frames_per_launch = int(sys.argv[3]) if len(sys.argv) > 3 else 8
workload = sys.argv[4] if len(sys.argv) > 4 else "config2"
KERNEL = "render_kernel"


def counters(name):
    path = os.path.join(src, name + "_counter_collection.csv")
    agg = defaultdict(list)
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(v):
    return sum(v) / len(v) if v else None


stats = {}
for r in csv.DictReader(open(os.path.join(src, "trace_kernel_stats.csv"))):
    stats[r["Name"]] = r
k = [v for n, v in stats.items() if KERNEL in n]
# registers and scratch of the dispatched kernel (kernel-trace columns)
res = {}
tpath = os.path.join(src, "trace_kernel_trace.csv")
if os.path.exists(tpath):
    for r in csv.DictReader(open(tpath)):
        if KERNEL in r.get("Kernel_Name", ""):
            for key in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Private_Segment_Size", "Scratch_Size",
                        "LDS_Block_Size", "Group_Segment_Size"):
                if key in r and r[key] != "":
                    res[key] = r[key]
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
w, f, sq, cyc = counters("pmc_write"), counters("pmc_fetch"), counters("pmc_sq"), counters("pmc_cyc")
l2 = counters("pmc_l2")
write_b = mean(w.get("WRITE_SIZE", [])) * 1024 if w.get("WRITE_SIZE") else None
fetch_b = mean(f.get("FETCH_SIZE", [])) * 1024 * 2 if f.get("FETCH_SIZE") else None
out = {
    "workload": workload, "n_gpus": 1, "frames_per_launch": frames_per_launch, "build": build,
    "kernel_resources": res,
    "scratch_bytes_per_lane": int(res.get("Scratch_Size") or res.get("Private_Segment_Size") or 0) if res else None,
    "kernel": k[0]["Name"] if k else None,
    "avg_kernel_ns": float(k[0]["AverageNs"]) if k else None, "calls": int(k[0]["Calls"]) if k else None,
    "write_bytes_per_launch": write_b, "fetch_bytes_per_launch": fetch_b,
    "hbm_bytes_per_launch": (write_b or 0) + (fetch_b or 0) if write_b is not None else None,
    "sq_insts_valu_per_launch": mean(sq.get("SQ_INSTS_VALU", [])),
    "sq_insts_salu_per_launch": mean(sq.get("SQ_INSTS_SALU", [])),
    "sq_insts_lds_per_launch": mean(sq.get("SQ_INSTS_LDS", [])),
    "sq_waves_per_launch": mean(sq.get("SQ_WAVES", [])),
    "sq_wave_cycles_per_launch": mean(cyc.get("SQ_WAVE_CYCLES", [])),
    "sq_busy_cycles_per_launch": mean(cyc.get("SQ_BUSY_CYCLES", [])),
    "sq_wait_inst_any_per_launch": mean(cyc.get("SQ_WAIT_INST_ANY", [])),
    "grbm_gui_active_per_launch": mean(cyc.get("GRBM_GUI_ACTIVE", [])),
    "l2_hit_per_launch": mean(l2.get("TCC_HIT_sum", [])),
    "l2_miss_per_launch": mean(l2.get("TCC_MISS_sum", [])),
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
for name in ("pmc_write", "pmc_fetch", "pmc_sq", "pmc_cyc", "pmc_l2"):
    for cname, vals in counters(name).items():
        allc[cname] = mean(vals)
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
