"""Per-frame kernel time of config 2 when K identical views share one launch
(development probe: how much of a frame is launch ramp-up / tail)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt

if len(sys.argv) > 1:
    rt.LIB_PATH = os.path.join(ROOT, "tools", "_ablate", sys.argv[1], "libopenglraytracer_amd.so")
ctx = rt.Context(0)
sc = rt.Scene(ctx, rt.bench_objects(16, 0))
W, H = 1920, 1080
out = torch.empty((8, H, W, 4), dtype=torch.float32, device="cuda")
v = rt.make_view(None, 0.0)
for k in (1, 2, 4, 8):
    ms = []
    for i in range(23):
        rt.render_batch(ctx, sc, out.data_ptr(), W, H, 0, [v] * k)
        if i >= 3:
            ms.append(ctx.last_kernel_ms())
    ms.sort()
    print("views %d: %.4f ms/launch, %.4f ms/frame" % (k, ms[len(ms) // 2], ms[len(ms) // 2] / k), flush=True)
