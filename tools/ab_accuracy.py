"""Per-channel accuracy of a build against the reference's GL renders (development probe).

    python tools/ab_accuracy.py BUILD [BUILD ...]

BUILD as in tools/ab.py: a directory under _ab (tools/ablate.sh) or "main",
optionally with context options (main:1=0 = culling off; round 4 used it on the
RT_FAST_* ablation builds of the price-of-exactness table). Every colour
fixture of tests/golden (the reference's own shader on llvmpipe, configs 1-4
and the shipped scene) is rendered through the drop-in call rt_render(cam =
NULL, time) and compared per channel: max, p99 and mean |d|, pixels beyond
1e-5, pixels beyond 1e-3 ("flips": a discrete decision — hit / miss, lit /
shadowed — that went the other way) and GL_RGBA8 bytes that change.
One JSON line per (build, fixture), then a summary line per build.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import openglraytracer_amd as rt  # noqa: E402
from conftest import fixture_objects, load_fixture, manifest  # noqa: E402


def load(spec):
    name, *opts = spec.split(":")
    path = rt.LIB_PATH if name == "main" else os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
    L = C.CDLL(path)
    vp, i = C.c_void_p, C.c_int
    L.rt_create.argtypes = [i, vp]
    L.rt_scene_create.argtypes = [vp, vp, i, vp, i, vp, i, vp]
    L.rt_scene_destroy.argtypes = [vp]
    L.rt_context_set.argtypes = [vp, i, i]
    L.rt_render.argtypes = [vp, vp, vp, C.c_float, i, i, i, i, i, vp, i, vp]
    ctx = C.c_void_p()
    assert L.rt_create(0, C.byref(ctx)) == 0
    for o in opts:
        k, v = o.split("=")
        assert L.rt_context_set(ctx, int(k), int(v)) == 0, spec
    return L, ctx


def stats(g, ref):
    d = np.abs(g[..., :3].astype(np.float64) - ref[..., :3].astype(np.float64))
    pm = d.max(-1)
    b8 = (rt.pack_rgba8(g.astype(np.float32)) != rt.pack_rgba8(np.dstack([ref[..., :3], np.zeros(ref.shape[:2])])
                                                               .astype(np.float32))).sum()
    return {"max": float(pm.max()), "p99": float(np.percentile(d, 99)), "mean": float(d.mean()),
            "px_gt_1e5": int((pm > 1e-5).sum()), "flips_gt_1e3": int((pm > 1e-3).sum()),
            "rgba8_bytes_changed": int(b8), "n_px": int(pm.size)}


def main():
    man = manifest()
    mats, lights = rt.reference_materials(), rt.reference_lights()
    for spec in sys.argv[1:]:
        L, ctx = load(spec)
        tot = {"px": 0, "gt": 0, "flips": 0, "max": 0.0, "b8": 0}
        for name in sorted(n for n, m in man.items() if m["probe"] == 0):
            m = man[name]
            rgb, _ = load_fixture(name)
            x0, y0, w, h = m["crop"]
            objs = fixture_objects(m, rt.reference_objects)
            oa = (rt.Object * len(objs))(*objs)
            ma = (rt.Material * len(mats))(*mats)
            la = (rt.Light * len(lights))(*lights)
            sc = C.c_void_p()
            assert L.rt_scene_create(ctx, oa, len(objs), ma, len(mats), la, len(lights), C.byref(sc)) == 0
            out = np.zeros((h, m["width"], 4), np.float32)
            rc = L.rt_render(ctx, sc, None, m["time"], m["width"], m["height"], m["max_depth"], y0, y0 + h,
                             out.ctypes.data, 0, None)
            assert rc == 0, rc
            L.rt_scene_destroy(sc)
            s = stats(out[:, x0:x0 + w], rgb)
            print(json.dumps({"build": spec, "fixture": name, "depth": m["max_depth"], **s}), flush=True)
            tot["px"] += s["n_px"]
            tot["gt"] += s["px_gt_1e5"]
            tot["flips"] += s["flips_gt_1e3"]
            tot["b8"] += s["rgba8_bytes_changed"]
            tot["max"] = max(tot["max"], s["max"])
        print(json.dumps({"build": spec, "summary": tot}), flush=True)


if __name__ == "__main__":
    main()
