"""Time one build from tools/ablate.sh (timing only):
    python tools/ablate_time.py NAME [config2 config3 ...]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (HIP runtime first)
import openglraytracer_amd as rt
from oracle import scenes
name = sys.argv[1]
cfgs = sys.argv[2:] or ["config2"]
rt.LIB_PATH = os.path.join(ROOT, "tools", "_ablate", name, "libopenglraytracer_amd.so")
ctx = rt.Context(0)
view = rt.make_view(None, 0.0)
for cfg in cfgs:
    build, w, h, depth = scenes.CONFIGS[cfg]
    sc = rt.Scene(ctx, build())
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    reps = 30 if cfg in ("config1", "config2") else 5
    ms = []
    for i in range(reps + 3):
        rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
        if i >= 3:
            ms.append(ctx.last_kernel_ms())
    print(name, cfg, "kernel ms median %.4f min %.4f" % (np.median(ms), np.min(ms)), flush=True)
    sc.close()
