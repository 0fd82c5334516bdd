"""Host cost of one render call and back-to-back frame rate, with and without
the context's per-launch timing events (development probe)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt

ctx = rt.Context(0)
sc = rt.Scene(ctx, rt.bench_objects(16, 0))
W, H = 1920, 1080
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream()
sh = stream.cuda_stream
views = [rt.make_view(None, 0.0)]
for timing in (1, 0):
    ctx.set_timing(timing)
    for fn in ("render_batch", "render_device"):
        call = (lambda: rt.render_batch(ctx, sc, out.data_ptr(), W, H, 0, views, stream=sh)) if fn == "render_batch" \
            else (lambda: rt.render_device(ctx, sc, out.data_ptr(), W, H, 0, view=views[0], stream=sh))
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        t0 = time.perf_counter()
        for _ in range(n):
            call()
        t1 = time.perf_counter()
        e1.record(stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("timing=%d %-13s host enqueue %.1f us/call | wall %.1f us/frame | events %.1f us/frame" % (
            timing, fn, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6, e0.elapsed_time(e1) / n * 1e3), flush=True)
