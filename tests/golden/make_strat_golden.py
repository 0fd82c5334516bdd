"""Stratified llvmpipe crops of the deep configs (run in the dev container).

Config 4 (7680x4320, 256 spheres, depth 4) and config 3 (3840x2160, 64
spheres, depth 2) are too large for llvmpipe whole, so make_golden.py pins
them on a few crops. This script adds stratified sets: a grid of small crops
spread over the whole frame — the four edges and the corners included — plus
the crops where the frame is most glass-heavy (most spawned refraction rays:
chosen from a cheap oracle pass over a coarse grid of candidate crops, the
checker only picks WHERE to look, the values come from llvmpipe). Every crop
is the reference's own shader (oracle/glref, patches P2 depth, P3 scene, P5
crop) at the orbit camera time given, read back as RGBA32F.

Writes tests/golden/<name>.npz: rgb float32 (n, h, w, 3) of the n crops,
crops int32 (n, 4) = (x0, y0, w, h), unproj float32 (4, 4) (llvmpipe's
inverse(proj*view), probe 5), and an entry in tests/golden/strat_manifest.json.

    python tests/golden/make_strat_golden.py       # needs oracle/_ref (make -C oracle ref)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import glref, port, scenes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

# name: (config, time, crop w, crop h, grid columns, grid rows, glass-heavy extras)
SETS = {
    "config4_strat": ("config4", 0.0, 64, 8, 6, 5, 4),
    "config4_t7_strat": ("config4", 7.0, 64, 8, 3, 3, 2),
    "config3_strat": ("config3", 0.0, 3840, 2, 1, 16, 0),
}


def grid_crops(width, height, cw, ch, nx, ny):
    """nx x ny crops spread evenly, the first / last column and row on the
    frame's edges."""
    xs = np.linspace(0, width - cw, nx).astype(int) if nx > 1 else np.array([0])
    ys = np.linspace(0, height - ch, ny).astype(int)
    ys = (ys // ch) * ch  # rows on the crop height's grid (8-row blocks for config 4)
    return [(int(x), int(y), cw, ch) for y in ys for x in xs]


def glass_heavy(objs, width, height, depth, t, cw, ch, n, taken):
    """The n candidate crops (on a 24 x 24 grid) whose pixels' colour changes
    most between depth 1 and depth `depth` in the oracle at a coarse
    sample — i.e. where the deep refraction / reflection trees matter."""
    cands = [(x, y) for x in np.linspace(0, width - cw, 24).astype(int)
             for y in (np.linspace(0, height - ch, 24).astype(int) // ch) * ch]
    score = []
    for x, y in cands:
        rows = (int(y), int(y) + 1)
        a = port.render(objs, width, height, depth, t, rows=rows)[0, x:x + cw:4]
        b = port.render(objs, width, height, 1, t, rows=rows)[0, x:x + cw:4]
        score.append(float(np.abs(a - b).sum()))
    out = []
    for i in np.argsort(score)[::-1]:
        c = (int(cands[i][0]), int(cands[i][1]), cw, ch)
        if c not in taken and c not in out:
            out.append(c)
        if len(out) == n:
            break
    return out


def main(names=None):
    mpath = os.path.join(OUT, "strat_manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    info = {"renderer": glref.renderer(), "shader": dict(glref.shader_info(), path="OpenGLRaytracer/raytrace_compute.glsl")}
    for name, (cfg, t, cw, ch, nx, ny, extra) in SETS.items():
        if names and name not in names:
            continue
        build, width, height, depth = scenes.CONFIGS[cfg]
        objs = build()
        crops = grid_crops(width, height, cw, ch, nx, ny)
        if extra:
            crops += glass_heavy(objs, width, height, depth, t, cw, ch, extra, crops)
        t0 = time.time()
        rgb = []
        for c in crops:
            rgba, _ = glref.render(objs, width, height, depth, t, crop=c)
            assert np.all(rgba[..., 3] == 0.0), (name, c)  # imageStore(vec4(rgb, 0.0)), :404
            rgb.append(rgba[..., :3].copy())
        dt = time.time() - t0
        pm, _ = glref.render(objs, width, height, depth, t, crop=(0, 0, 4, 4), probe=5)
        unproj = np.ascontiguousarray(pm[:, :, 0].T)  # [col][row]
        np.savez_compressed(os.path.join(OUT, name + ".npz"), rgb=np.stack(rgb), crops=np.array(crops, np.int32),
                            unproj=unproj)
        manifest[name] = {"scene": cfg, "width": width, "height": height, "max_depth": depth, "time": t,
                          "n_crops": len(crops), "crop_size": [cw, ch], "pixels": len(crops) * cw * ch,
                          "seconds": round(dt, 2), **info}
        print("%-20s %3d crops, %6d pixels, %6.1fs" % (name, len(crops), len(crops) * cw * ch, dt), flush=True)
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
