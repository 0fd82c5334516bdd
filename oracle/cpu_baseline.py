"""CPU baseline for bench.py — TEST INFRASTRUCTURE ONLY (run as a child process).

Times the reference's own shader (raytrace_compute.glsl) on Mesa llvmpipe
(oracle/_ref/libglref.so, kind "reference") over a bounded band of the
benchmark frame (config 2: 1920x1080, room box + 16 spheres, depth 0), with
LP_NUM_THREADS worker threads. Falls back to the C restatement
(oracle/_build/librt_oracle.so, kind "port") when the harness is absent.
Prints one JSON object.
"""
import argparse
import json
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=8)
ap.add_argument("--budget", type=float, default=15.0, help="seconds of CPU rendering to aim for")
args = ap.parse_args()
os.environ["LP_NUM_THREADS"] = str(args.threads)  # read by llvmpipe at screen creation

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import glref, port, scenes  # noqa: E402

W, H, DEPTH = 1920, 1080, 0
objs = scenes.bench_objects(16)
mid = H // 2

if glref.available():
    # calibrate on a 16-row band (JIT excluded by glref's warm-up dispatch)
    _, t = glref.render(objs, W, H, DEPTH, 0.0, crop=(0, mid - 8, W, 16), repeats=1)
    per_row = t[0] / 16
    rows = int(max(16, min(H, args.budget / 2 / max(per_row, 1e-6))))
    y0 = max(0, mid - rows // 2)
    _, t = glref.render(objs, W, H, DEPTH, 0.0, crop=(0, y0, W, rows), repeats=1)
    secs = float(t[0])
    kind = "reference"
    how = "reference raytrace_compute.glsl on Mesa llvmpipe (%s)" % glref.renderer()
else:
    rows = H
    t0 = time.perf_counter()
    port.render(objs, W, H, DEPTH, 0.0, rows=(0, H), threads=args.threads)
    secs = time.perf_counter() - t0
    y0 = 0
    kind = "port"
    how = "C float32 restatement (oracle/rt_oracle.c), OpenMP"
px = W * rows
print(json.dumps({"value": round(px / secs / 1e6, 4), "unit": "Mrays/s", "cores": args.threads, "kind": kind,
                  "sample": "%s: rows [%d, %d) of the 1920x1080 config-2 frame (%d primary rays) in %.2f s"
                            % (how, y0, y0 + rows, px, secs)}))
