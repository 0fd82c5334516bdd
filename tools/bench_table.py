"""DESIGN.md §5's per-config table from the committed bench lines of one session.

    python tools/bench_table.py TAG      (reads profiles/TAG_bench_<workload>.log)

One row per workload: frame, depth, kernel time per launch and per frame,
primary rays (samples) per second, the HBM-write roofline fraction, the PMC
traffic against the stored bytes, the VALU-issue fraction, what the line
verified, and the llvmpipe CPU baseline where the line carries one. Every
figure is copied from the JSON line; nothing is measured here.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORDER = ["config2", "config3", "config4", "config5", "shipped"]


def line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    return None


def row(wl, d):
    c, r = d["config"], d["roofline"]
    fpl = c.get("frames_per_launch", 1)
    kms = r["kernel_ms"]
    per_frame = kms / fpl
    unit = "samples/s" if wl == "config5" else "rays/s"
    val = "%.2f G %s" % (d["value"] / 1e3, unit)
    extra = []
    if d.get("single_frame"):
        extra.append("one frame per launch %.1f µs" % d["single_frame"]["us_per_frame"])
    if d.get("draw_loop"):
        extra.append("draw() loop with the scene update %.1f µs" % d["draw_loop"]["us_per_frame"])
    if d.get("pipelined"):
        extra.append("two streams %.2f G" % (d["pipelined"]["value"] / 1e3))
    traffic = r.get("traffic")
    stored = r.get("bytes_per_launch")
    tr = ("%.2f GB per launch (%.1f× the stored %.3f GB)" % (traffic / 1e9, traffic / stored, stored / 1e9)
          if traffic else "—")
    v = r.get("valu") or {}
    valu = ("%.0f %% (%.0f %% at the measured %.2f GHz)" % (100 * v["frac"], 100 * v.get("frac_at_measured_clock", 0),
                                                             v.get("measured_clock_ghz", 0)) if "frac" in v else "—")
    ver = d.get("verified") or {}
    vtext = ("bit-exact, %d px" % ver["pixels"]) if ver.get("bit_exact") else ("—" if not ver else "MISMATCH")
    cpu = d.get("cpu_baseline") or {}
    ctext = ("%.3f Mrays/s, %d threads" % (cpu["value"], cpu["cores"])) if cpu else "—"
    frame = "%d×%d" % (c["width"], c["height"]) + (" × %d spp" % c["spp"] if c.get("spp") else "")
    kernel = ("%.3f ms per %d frames = %.1f µs per frame" % (kms, fpl, per_frame * 1e3) if fpl > 1 else
              "%.3f ms" % kms)
    return ("| %s | %s | %d | %s | **%s**%s | %.4f | %s | %s | %s | %s |" % (
        wl, frame, c["max_depth"], kernel, val, (" · " + " · ".join(extra)) if extra else "", r["frac"], tr, valu,
        vtext, ctext))


def main():
    tag = sys.argv[1]
    print("| workload | frame | depth | kernel (HIP events) | value | HBM-write frac | PMC traffic | VALU issue | "
          "verified | llvmpipe |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for wl in ORDER:
        p = os.path.join(ROOT, "profiles", "%s_bench_%s.log" % (tag, wl))
        if os.path.exists(p):
            d = line(p)
            if d:
                print(row(wl, d))
    builds = set()
    for wl in ORDER:
        p = os.path.join(ROOT, "profiles", "%s_bench_%s.log" % (tag, wl))
        if os.path.exists(p):
            d = line(p)
            if d:
                builds.add(d.get("build"))
    print("\n(build%s: %s)" % ("s" if len(builds) > 1 else "", "; ".join(sorted(b for b in builds if b))))


if __name__ == "__main__":
    main()
