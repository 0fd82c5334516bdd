"""CPU baseline for bench.py — TEST INFRASTRUCTURE ONLY (run as a child process).

Times the reference's own shader (raytrace_compute.glsl) on Mesa llvmpipe
(oracle/_ref/libglref.so, kind "reference") as SURVEY.md §8(d) prescribes:
warm-up dispatch excluded (JIT), median of 3 dispatches each followed by
glFinish, wall clock, primary Mrays/s = pixels / t. Falls back to the C
restatement (oracle/_build/librt_oracle.so, kind "port") when the harness is
absent.

* value: the bench workload's frame at --threads llvmpipe threads
  (LP_NUM_THREADS); a full frame when it fits the budget, else a band of full
  rows around the middle, extrapolated (labelled);
* threads_1: the same with LP_NUM_THREADS=1 (a smaller band);
* per_config: configs 1-4 at --threads (1: the full 256x256 frame; 3-4: row
  bands, extrapolated); config 5 has no reference counterpart (one ray per
  pixel per dispatch) and is derived from config 2's rate.
LP_NUM_THREADS is read when llvmpipe creates its screen, so every thread
count runs in a process of its own (this script re-invoked with --measure).
Prints one JSON object.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MEDIAN_OF = 3


def measure(configs, threads, budget):
    """Child: time each config (name -> seconds share) at `threads` threads."""
    os.environ["LP_NUM_THREADS"] = str(threads)  # before llvmpipe's screen exists
    sys.path.insert(0, ROOT)
    from oracle import glref, port, scenes
    use_gl = glref.available()
    out = {}
    for name, share in configs:
        build, w, h, depth = scenes.CONFIGS[name]
        objs = build()
        if objs is None and not use_gl:  # the shipped scene (the harness keeps the shader's own)
            objs = port.reference_objects(0.0)

        def run(x0, y0, cw, ch, repeats):
            if use_gl:
                return list(glref.render(objs, w, h, depth, 0.0, crop=(x0, y0, cw, ch), repeats=repeats)[1])
            ts = []
            for _ in range(repeats + 1):  # first run: warm-up, as the harness does
                t0 = time.perf_counter()
                port.render(objs, w, h, depth, 0.0, rows=(y0, y0 + ch), threads=threads)
                ts.append(time.perf_counter() - t0)
            return sorted(ts[1:])

        # calibrate on a small crop at the middle of the frame
        cw, ch = (min(w, 64), min(h, 2)) if use_gl else (w, min(h, 2))
        x0, y0 = (w - cw) // 2, (h - ch) // 2
        t = run(x0, y0, cw, ch, 1)[0]
        per_px = t / (cw * ch)
        px_budget = share / (MEDIAN_OF + 1) / max(per_px, 1e-12)  # warm-up + timed dispatches
        rows = int(max(1, min(h, px_budget / w)))
        cols = w if (rows > 1 or not use_gl) else int(max(64, min(w, px_budget)))
        x0, y0 = (w - cols) // 2, (h - rows) // 2
        ts = run(x0, y0, cols, rows, MEDIAN_OF)
        med = float(ts[len(ts) // 2])
        px = cols * rows
        what = ("rows [%d, %d)" % (y0, y0 + rows) if cols == w else
                "columns [%d, %d) of row %d" % (x0, x0 + cols, y0))
        out[name] = {"mrays_s": round(px / med / 1e6, 5), "threads": threads, "median_of": MEDIAN_OF,
                     "dispatch_s": [round(float(v), 4) for v in ts],
                     "sample": "%s of the %dx%d depth-%d frame (%d primary rays)" % (what, w, h, depth, px),
                     "extrapolated": px < w * h,
                     "frame_s": round(med * (w * h) / px, 3)}
    renderer = glref.renderer() if use_gl else "C float32 restatement (oracle/rt_oracle.c), OpenMP"
    return {"kind": "reference" if use_gl else "port", "renderer": renderer, "configs": out}


def child(configs, threads, budget):
    cmd = [sys.executable, os.path.abspath(__file__), "--measure", ",".join("%s:%g" % c for c in configs),
           "--threads", str(threads), "--budget", str(budget)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=max(120, 10 * budget))
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--budget", type=float, default=25.0, help="seconds of CPU rendering to aim for")
    ap.add_argument("--workload", default="config2")
    ap.add_argument("--measure", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.measure:
        configs = [(c.split(":")[0], float(c.split(":")[1])) for c in args.measure.split(",")]
        print(json.dumps(measure(configs, args.threads, args.budget)))
        return
    wl = args.workload
    own = "config2" if wl == "config5" else wl  # config 5: one ray per pixel per reference dispatch
    b = args.budget
    others = [c for c in ("config1", "config2", "config3", "config4", "shipped") if c != own]
    main_run = child([(own, 0.4 * b)] + [(c, 0.1 * b) for c in others], args.threads, b)
    one = child([(own, 0.2 * b)], 1, b)
    per = dict(main_run["configs"])
    r = per[own]
    per["config5"] = {"mrays_s": per["config2"]["mrays_s"], "threads": args.threads,
                      "sample": "derived: the reference traces one ray per pixel per dispatch, so its 1024-spp "
                                "rate is config 2's primary-ray rate", "extrapolated": True,
                      "frame_s": round(per["config2"]["frame_s"] * 1024, 1)}
    print(json.dumps({
        "value": per[wl]["mrays_s"] if wl != "config5" else per["config5"]["mrays_s"],
        "unit": "Mrays/s", "cores": args.threads, "kind": main_run["kind"],
        "sample": "%s: %s, %d threads, median of %d dispatches%s" % (
            main_run["renderer"], r["sample"], args.threads, MEDIAN_OF,
            " (extrapolated to the frame)" if r["extrapolated"] else ""),
        "median_of": MEDIAN_OF,
        "threads_1": one["configs"][own],
        "per_config": per,
    }))


if __name__ == "__main__":
    main()
