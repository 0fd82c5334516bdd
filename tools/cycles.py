"""Wave time per kernel phase (development probe; RT_CYCLES builds):
    tools/ablate.sh flags cycles "-DRT_CYCLES"; python tools/cycles.py cycles [config ...]
Prints, per config, the shader-clock cycles the render kernel's waves spent
in each phase of one frame (issue and stalls alike, summed over waves) as
shares of the total, and per pixel."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import openglraytracer_amd as rt  # noqa: E402
from oracle import scenes  # noqa: E402

PHASES = ["prologue", "raygen", "closest_primary", "closest_secondary", "resolve", "phong", "shadow",
          "walk_other", "store_fetch"]
name = sys.argv[1]
cfgs = sys.argv[2:] or ["config2", "config3", "config4"]
rt.LIB_PATH = os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
L = rt.lib()
L.rt_debug_cycles.argtypes = [C.c_void_p, C.c_int]
ctx = rt.Context(0)
view = rt.make_view(None, 0.0)
buf = np.zeros(16, np.uint64)
for cfg in cfgs:
    build, w, h, depth = scenes.CONFIGS[cfg]
    sc = rt.Scene(ctx, build())
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)  # warm-up
    assert L.rt_debug_cycles(buf.ctypes.data, 1) == 0
    reps = 3
    for _ in range(reps):
        rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
    torch.cuda.synchronize()
    assert L.rt_debug_cycles(buf.ctypes.data, 1) == 0
    tot = float(buf[:len(PHASES)].sum())
    print("%s %dx%d depth %d: %.3g wave-cycles per frame" % (cfg, w, h, depth, tot / reps))
    for k, n in enumerate(PHASES):
        print("   %-18s %6.2f %%  %10.1f wave-cycles per pixel" % (n, 100 * buf[k] / tot, buf[k] / reps / (w * h)))
    sc.close()
