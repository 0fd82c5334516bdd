"""What the blocking context stream costs a NULL-stream call (development probe).

    python tools/null_stream_ab.py BUILD_A BUILD_B [N]

Round 5 made the context's own stream a blocking HIP stream, so that a call
with hip_stream = NULL is ordered after the device's null stream like
glDispatchCompute (include/rt.h). A NULL-stream call is synchronous (the
reference's glFinish, main.cpp:238), so its cost is wall time: this times N
one-frame config-2 rt_render_view calls with a NULL stream per build (BUILD:
"main" = the in-tree library, or a directory under _ab, e.g. the round-4
library built by `tools/ablate.sh rev 7038a0d`), rounds interleaved so clock
drift hits both alike, and prints the median microseconds per call.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import openglraytracer_amd as rt  # noqa: E402
from oracle import scenes  # noqa: E402


def load(name):
    path = rt.LIB_PATH if name == "main" else os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
    L = C.CDLL(path)
    vp, i = C.c_void_p, C.c_int
    L.rt_create.argtypes = [i, vp]
    L.rt_scene_create.argtypes = [vp, vp, i, vp, i, vp, i, vp]
    L.rt_context_set.argtypes = [vp, i, i]
    L.rt_render_view.argtypes = [vp, vp, vp, i, i, i, i, i, vp, i, vp]
    ctx = C.c_void_p()
    assert L.rt_create(0, C.byref(ctx)) == 0
    L.rt_context_set(ctx, rt.abi.RT_OPT_TIMING, 0)
    build, w, h, depth = scenes.CONFIGS["config2"]
    objs, mats, lights = build(), rt.reference_materials(), rt.reference_lights()
    sc = C.c_void_p()
    assert L.rt_scene_create(ctx, (rt.Object * len(objs))(*objs), len(objs), (rt.Material * len(mats))(*mats),
                             len(mats), (rt.Light * len(lights))(*lights), len(lights), C.byref(sc)) == 0
    return L, ctx, sc, w, h, depth


def main():
    names = sys.argv[1:3]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    libs = {b: load(b) for b in names}
    out = torch.empty((1080, 1920, 4), dtype=torch.float32, device="cuda")
    views = [rt.make_view(None, k / 60.0) for k in range(64)]
    times = {b: [] for b in names}
    for b, (L, ctx, sc, w, h, depth) in libs.items():
        for k in range(50):
            assert L.rt_render_view(ctx, sc, C.byref(views[k % 64]), w, h, depth, 0, h,
                                    C.c_void_p(out.data_ptr()), 1, None) == 0
    for _ in range(7):
        for b, (L, ctx, sc, w, h, depth) in libs.items():
            t0 = time.perf_counter()
            for k in range(n):
                L.rt_render_view(ctx, sc, C.byref(views[k % 64]), w, h, depth, 0, h, C.c_void_p(out.data_ptr()), 1,
                                 None)
            times[b].append((time.perf_counter() - t0) / n * 1e6)
    for b in names:
        t = np.array(times[b])
        print("%-10s NULL-stream one-frame config-2 call: median %.2f us  min %.2f us  (7 rounds of %d)"
              % (b, np.median(t), t.min(), n), flush=True)
    a, c = (np.median(times[x]) for x in names)
    print("%s / %s = %.4f" % (names[1], names[0], c / a))


if __name__ == "__main__":
    main()
