"""Host submission rate of one-frame launches against their GPU time
(development probe).

    python tools/launch_rate.py [CONFIG] [N]

Submits N one-frame rt_render_batch calls back to back on one stream
(no synchronisation inside the loop) and reports the host's time per call
beside the GPU's (HIP events around the same launches). When the host
needs longer per call than the GPU per frame, the one-frame-per-launch rate
is the host's, not the kernel's.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import openglraytracer_amd as rt  # noqa: E402
from oracle import scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
build, w, h, depth = scenes.CONFIGS[cfg]
ctx = rt.Context(0)
ctx.set_timing(False)
scene = rt.Scene(ctx, build())
out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
views = [rt.make_view(None, k / 60.0) for k in range(64)]
for k in range(20):
    rt.render_batch(ctx, scene, out.data_ptr(), w, h, depth, [views[k % 64]], stream=s.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
t0 = time.perf_counter()
for k in range(n):
    rt.render_batch(ctx, scene, out.data_ptr(), w, h, depth, [views[k % 64]], stream=s.cuda_stream)
t1 = time.perf_counter()
e1.record(s)
torch.cuda.synchronize()
host_us = (t1 - t0) / n * 1e6
gpu_us = e0.elapsed_time(e1) / n * 1e3
print("%s: %d one-frame launches: host %.2f us per call, GPU %.2f us per frame" % (cfg, n, host_us, gpu_us))
# the same with the ctypes argument array built once (the Python wrapper's share)
import ctypes as C  # noqa: E402
arrs = [(rt.View * 1)(v) for v in views]
L = rt.lib()
e0.record(s)
t0 = time.perf_counter()
for k in range(n):
    L.rt_render_batch(ctx.handle, scene.handle, arrs[k % 64], 1, w, h, depth, 8, 1, 0, C.c_void_p(out.data_ptr()),
                      C.c_void_p(s.cuda_stream))
t1 = time.perf_counter()
e1.record(s)
torch.cuda.synchronize()
print("%s: direct C calls: host %.2f us per call, GPU %.2f us per frame"
      % (cfg, (t1 - t0) / n * 1e6, e0.elapsed_time(e1) / n * 1e3))

# batches: host time per rt_render_batch call against its GPU time, whole
# frames and one of 8 row-tiled shards (the config-2 step's launch at N = 8)
if cfg == "config2":
    big = torch.empty((64, h, w, 4), dtype=torch.float32, device="cuda")
    for nv in (8, 64):
        for shards in (1, 8):
            vs = views[:nv]
            for _ in range(3):
                rt.render_batch(ctx, scene, big.data_ptr(), w, h, depth, vs, 8, shards, 0, stream=s.cuda_stream)
            torch.cuda.synchronize()
            reps = 40
            e0.record(s)
            t0 = time.perf_counter()
            for _ in range(reps):
                rt.render_batch(ctx, scene, big.data_ptr(), w, h, depth, vs, 8, shards, 0, stream=s.cuda_stream)
            t1 = time.perf_counter()
            e1.record(s)
            torch.cuda.synchronize()
            # the host's own cost: 3 calls from an idle GPU (fewer than the
            # context's 4 batch slots, so no call waits for a slot to free)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            for _ in range(3):
                rt.render_batch(ctx, scene, big.data_ptr(), w, h, depth, vs, 8, shards, 0, stream=s.cuda_stream)
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            print("%s: %d views, %d shard(s): back to back %.1f us per call on the host, GPU %.1f us per call; "
                  "the host's own cost (3 calls, no slot wait) %.1f us per call"
                  % (cfg, nv, shards, (t1 - t0) / reps * 1e6, e0.elapsed_time(e1) / reps * 1e3, (t3 - t2) / 3 * 1e6))
