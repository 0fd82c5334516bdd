"""Registers and scratch of every render kernel in a built library (the A/B gate).

    python tools/resources.py [LIB.so | BUILD ...]        (default: the in-tree library)
    python tools/resources.py --gate BASE.so VARIANT.so   exit 1 if VARIANT spills more
    python tools/resources.py --markdown [BUILD]          DESIGN.md §3's occupancy table

Reads the gfx950 code object out of the library's .hip_fatbin section
(llvm-objcopy + clang-offload-bundler) and its kernel metadata notes
(llvm-readelf --notes): .vgpr_count, .sgpr_count and
.private_segment_fixed_size (scratch bytes per lane) — the numbers the
compiler's -Rpass-analysis=kernel-resource-usage remarks print (make
resource-usage), and what the occupancy follows from (512 VGPRs per SIMD
lane slot: 8 waves at <= 64, 6 at <= 80, 5 at <= 96).

rocprofv3's kernel trace reports `VGPR_Count` as half of these (32 for the
depth-0 kernel's 64, 40 for the 80 of the deep kernels): it decodes the
descriptor's granulated VGPR field with a granule of 4, where gfx950 (wave64)
allocates in granules of 8. Its scratch figure agrees with this tool.

The gate (round-4 verdict): every A/B variant's log starts with
both builds' lines for the kernels it times, and a variant whose scratch grows
at a register-capped kernel is not timed unless its prediction accounts for
the spill.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def lib_path(spec):
    if spec in ("main", None):
        return os.path.join(ROOT, "openglraytracer_amd", "libopenglraytracer_amd.so")
    if spec.endswith(".so"):
        return spec
    return os.path.join(ROOT, "_ab", spec, "libopenglraytracer_amd.so")


def kernel_name(mangled):
    """render_kernel<D, MC, DEV[, SHAPE]> from the mangled name (SHAPE: the
    scene shapes, rt_internal.h kShapeRoom), else the mangled name."""
    m = re.search(r"render_kernelILi(\d)ELb([01])ELb([01])E(?:Li(\d+)E)?", mangled)
    if m:
        name = "render_kernel<%s,%s,%s" % (m.group(1), "true" if m.group(2) == "1" else "false",
                                           "true" if m.group(3) == "1" else "false")
        if m.group(4) and m.group(4) != "0":
            name += ",%s" % m.group(4)
        return name + ">"
    return mangled


def resources(so):
    """{kernel: {"vgpr", "sgpr", "scratch", "waves_per_simd"}} of the library's gfx950 code object."""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.run([LLVM + "/llvm-objcopy", "--dump-section", ".hip_fatbin=" + fb, so, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                        "--targets=" + TARGET, "--output=" + co], check=True, capture_output=True)
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(name|vgpr_count|sgpr_count|private_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "name":
            cur = out.setdefault(kernel_name(val), {})
        else:
            cur[{"vgpr_count": "vgpr", "sgpr_count": "sgpr", "private_segment_fixed_size": "scratch"}[key]] = int(val)
    for r in out.values():
        if "vgpr" in r:
            r["waves_per_simd"] = min(8, 512 // max(8, -(-r["vgpr"] // 8) * 8))
    return {k: v for k, v in out.items() if k.startswith("render_kernel")}


def fmt(name, r):
    return "%-28s VGPR %3d  SGPR %3d  scratch %4d B/lane  %d waves/SIMD" % (
        name, r.get("vgpr", -1), r.get("sgpr", -1), r.get("scratch", -1), r.get("waves_per_simd", 0))


def report(spec, kernels=None):
    res = resources(lib_path(spec))
    lines = ["# resources of %s (%s)" % (spec or "main", lib_path(spec))]
    for k in sorted(res):
        if kernels is None or k in kernels:
            lines.append("#   " + fmt(k, res[k]))
    return res, "\n".join(lines)


def gate(base, variant, kernels=None):
    """Kernels whose scratch grows in `variant` against `base` (or whose
    occupancy drops): [(kernel, base, variant)]."""
    a, b = resources(lib_path(base)), resources(lib_path(variant))
    bad = []
    for k in sorted(set(a) & set(b)):
        if kernels is not None and k not in kernels:
            continue
        if b[k].get("scratch", 0) > a[k].get("scratch", 0) or b[k]["waves_per_simd"] < a[k]["waves_per_simd"]:
            bad.append((k, a[k], b[k]))
    return bad


# DESIGN.md §3's occupancy table: (row label, kernel) in the order it lists them
TABLE = [
    ("depth 0, config 2 (room, 2-B masks, > 8 views: device views)", "render_kernel<0,false,true,18>"),
    ("depth 0, the shipped scene (2-B masks, 4 boxes, device views)", "render_kernel<0,false,true,2>"),
    ("depth 0, Monte-Carlo, config 5", "render_kernel<0,true,false,18>"),
    ("depth 0, general", "render_kernel<0,false,false>"),
    ("depth 0, Monte-Carlo, general", "render_kernel<0,true,false>"),
    ("depth 1 (config 1)", "render_kernel<1,false,false>"),
    ("depth 2, config 3 (room, wide masks, origin lists)", "render_kernel<2,false,false,48>"),
    ("depth 2, general", "render_kernel<2,false,false>"),
    ("depth 4, config 4 (room, wide masks, origin lists)", "render_kernel<4,false,false,48>"),
    ("depth 4, general", "render_kernel<4,false,false>"),
]


def markdown(spec="main"):
    """The occupancy table of DESIGN.md §3, from the library's code object."""
    res = resources(lib_path(spec))
    rows = ["| kernel | VGPRs | SGPRs | waves / SIMD | scratch B / lane |", "|---|---|---|---|---|"]
    for label, k in TABLE:
        r = res.get(k)
        if r:
            rows.append("| %s: `%s` | %d | %d | %d | %d |" % (label, k, r["vgpr"], r["sgpr"], r["waves_per_simd"],
                                                            r["scratch"]))
    return "\n".join(rows)


def main():
    args = sys.argv[1:]
    if args[:1] == ["--markdown"]:
        print(markdown(args[1] if len(args) > 1 else "main"))
        return
    if args[:1] == ["--gate"]:
        bad = gate(args[1], args[2])
        for k, x, y in bad:
            print("GATE %s: %s -> %s" % (k, fmt("", x).strip(), fmt("", y).strip()))
        sys.exit(1 if bad else 0)
    for spec in args or ["main"]:
        print(report(spec)[1])


if __name__ == "__main__":
    main()
