"""Time config 2 with each ablation build from tools/ablate.sh (timing only)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (HIP runtime first)
import openglraytracer_amd as rt
name = sys.argv[1]
rt.LIB_PATH = os.path.join(ROOT, "tools", "_ablate", name, "libopenglraytracer_amd.so")
ctx = rt.Context(0)
sc = rt.Scene(ctx, rt.bench_objects(16))
out = torch.empty((1080, 1920, 4), dtype=torch.float32, device="cuda")
view = rt.make_view(None, 0.0)
ms = []
for i in range(30):
    rt.render_device(ctx, sc, out.data_ptr(), 1920, 1080, 0, view=view)
    if i >= 5:
        ms.append(ctx.last_kernel_ms())
print(name, "config2 kernel ms median %.4f" % np.median(ms))
