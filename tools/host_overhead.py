"""Host cost of one render call (tiny frame: the GPU is never the bottleneck)
and the back-to-back frame rate at 1920x1080, with and without the context's
per-launch timing events (development probe)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt

ctx = rt.Context(0)
sc = rt.Scene(ctx, rt.bench_objects(16, 0))
out = torch.empty((1080, 1920, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
sh = stream.cuda_stream
views = [rt.make_view(None, 0.0)]
arr = (rt.View * 1)(*views)
L = rt.lib()


def raw(W, H):
    return L.rt_render_batch(ctx.handle, sc.handle, arr, 1, W, H, 0, 8, 1, 0, C.c_void_p(out.data_ptr()), C.c_void_p(sh))


for timing in (1, 0):
    ctx.set_timing(timing)
    for W, H in ((8, 8), (1920, 1080)):
        for name, call in (("render_batch", lambda: rt.render_batch(ctx, sc, out.data_ptr(), W, H, 0, views, stream=sh)),
                           ("raw ctypes", lambda: raw(W, H))):
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
            print("timing=%d %4dx%-4d %-12s host %.1f us/call | wall %.1f us | events %.1f us/frame" % (
                timing, W, H, name, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6, e0.elapsed_time(e1) / n * 1e3),
                flush=True)

# single calls from an idle stream: host time of the call alone, then completion
for W, H in ((8, 8), (1920, 1080)):
    hs, cs = [], []
    for i in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        raw(W, H)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i >= 5:
            hs.append(t1 - t0)
            cs.append(t2 - t0)
    hs.sort(); cs.sort()
    print("%4dx%-4d single call: host %.1f us, call->complete %.1f us" % (W, H, hs[10] * 1e6, cs[10] * 1e6), flush=True)
