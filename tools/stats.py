"""Event counts of the render kernel (development probe; RT_STATS builds):
    tools/ablate.sh flags stats "-DRT_STATS"; python tools/stats.py stats [config ...]
Prints, per config, the counters of one frame normalised per pixel."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import openglraytracer_amd as rt  # noqa: E402
from oracle import scenes  # noqa: E402

NAMES = ["rays_primary", "rays_secondary", "closest2_wave_calls", "bvh_node_tests", "bvh_wave_iters",
         "bvh_leaf_visits", "primary_sphere_tests", "shadow_queries", "shadow_exact_tests", "gmask_wave_iters",
         "occluded_wave_calls", "trace_wave_iters", "dmask_wave_iters", "closest1_wave_calls", "olist_wave_passes",
         "olist_tests"]
name = sys.argv[1]
cfgs = sys.argv[2:] or ["config2", "config3", "config4"]
rt.LIB_PATH = os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
L = rt.lib()
L.rt_debug_stats.argtypes = [C.c_void_p, C.c_int]
ctx = rt.Context(0)
view = rt.make_view(None, 0.0)
buf = np.zeros(16, np.uint64)
for cfg in cfgs:
    build, w, h, depth = scenes.CONFIGS[cfg]
    sc = rt.Scene(ctx, build())
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    assert L.rt_debug_stats(buf.ctypes.data, 1) == 0
    rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
    torch.cuda.synchronize()
    assert L.rt_debug_stats(buf.ctypes.data, 1) == 0
    px = w * h
    tiles = px / 64
    print("%s %dx%d depth %d" % (cfg, w, h, depth))
    for k, n in enumerate(NAMES):
        if n == "-" or not buf[k]:
            continue
        per = buf[k] / (tiles if "wave" in n else px)
        print("   %-22s %14d  %10.3f per %s" % (n, buf[k], per, "wave tile" if "wave" in n else "pixel"))
    sc.close()
