"""Parity soak (development probe, run on the GPU box): many seeded random
scenes (tests/test_gpu_parity.py random_scene, larger frames) through the HIP
kernel against the oracle, bit for bit, culling on and off.

    python tools/soak.py FIRST_SEED N [MAX_W MAX_H]
    SOAK_KIND=boxes python tools/soak.py ...   (tests/test_gpu_parity.py box_scene:
                                               4-12 rotated boxes, round 6's box culling)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402  (HIP runtime first)
import openglraytracer_amd as rt  # noqa: E402
from oracle import port  # noqa: E402
from test_gpu_parity import box_scene, random_scene  # noqa: E402

make_scene = box_scene if os.environ.get("SOAK_KIND") == "boxes" else random_scene

first, n = int(sys.argv[1]), int(sys.argv[2])
max_w, max_h = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (200, 150)
ctx = rt.Context(0)
bad, pixels, rays_depth, olist = [], 0, {}, 0
for seed in range(first, first + n):
    objs, mats, lights, t, depth, w, h = make_scene(seed)
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(w, max_w + 1)), int(rng.integers(h, max_h + 1))
    view = rt.make_view(None, t)
    sc = rt.Scene(ctx, objs, materials=mats, lights=lights)
    try:
        on = rt.render(ctx, sc, w, h, depth, view=view)
        ctx.set_culling(False)
        off = rt.render(ctx, sc, w, h, depth, view=view)
    finally:
        ctx.set_culling(True)
        sc.close()
    o = port.render(objs, w, h, depth, t, materials=mats, lights=lights)
    ok = np.array_equal(on, o, equal_nan=True) and np.array_equal(off, o, equal_nan=True)
    pixels += w * h
    rays_depth[depth] = rays_depth.get(depth, 0) + 1
    ns = sum(1 for ob in objs if not any(ob.box_mins[:] + ob.box_maxs[:]) and ob.radius != -1.0)  # spheres (:749-771)
    if depth >= 2 and 33 <= ns <= 256:  # rt_internal.h RT_OLIST_FROM
        olist += 1  # the origin-sphere lists take the secondary rays (rt_scene.cpp)
    if not ok:
        diff = int((~((on == o) | (np.isnan(on) & np.isnan(o)))).any(-1).sum())
        bad.append((seed, len(objs), depth, w, h, diff))
        print("MISMATCH seed %d: %d objects, depth %d, %dx%d, %d pixels differ" % bad[-1], flush=True)
    if (seed - first + 1) % 50 == 0:
        print("%d scenes, %d pixels, %d mismatching" % (seed - first + 1, pixels, len(bad)), flush=True)
print("soak: %d random scenes (seeds %d..%d), %d pixels, depths %s, %d with origin-sphere lists: %d mismatching"
      % (n, first, first + n - 1, pixels, dict(sorted(rays_depth.items())), olist, len(bad)), flush=True)
sys.exit(1 if bad else 0)
