"""Generate the golden fixtures from the reference itself (run in the dev container).

Every fixture is the output of the reference's own shader,
/root/reference/OpenGLRaytracer/raytrace_compute.glsl, run unmodified except
for the declared patches (oracle/glref/glref.c header: P1 writeonly, P2 depth,
P3 scene, P4 probe, P5 crop) on Mesa llvmpipe, read back as RGBA32F.

Writes tests/golden/<name>.npz (float32 `rgb`, shape (h, w, 3); alpha is
checked to be 0 and dropped; float32 `unproj`, llvmpipe's inverse(proj*view)
as a column-major 4x4, from probe 5) and tests/golden/manifest.json.

    python tests/golden/make_golden.py            # needs oracle/_ref (make -C oracle ref)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import glref, scenes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

# name: (scene, width, height, depth, time, crop (x0,y0,w,h) or None, probe)
# scene: "shipped" (raytrace_compute.glsl:261-321 as written) or a configs key.
FIXTURES = {
    # shipped scene, static (t = 0)
    "shipped_t0_d0_256": ("shipped", 256, 256, 0, 0.0, None, 0),
    "shipped_t0_d1_256": ("shipped", 256, 256, 1, 0.0, None, 0),
    "shipped_t0_d2_160x90": ("shipped", 160, 90, 2, 0.0, None, 0),
    "shipped_t0_d4_64x36": ("shipped", 64, 36, 4, 0.0, None, 0),
    # odd width/height (integer halves, :377-378)
    "shipped_t0_d0_129x73": ("shipped", 129, 73, 0, 0.0, None, 0),
    # reference native size, a band of rows (P5 crop)
    "shipped_t0_d0_1280x720_rows": ("shipped", 1280, 720, 0, 0.0, (0, 352, 1280, 16), 0),
    # animated scene (boxes bob / rotate / tumble, :277-307; camera orbit)
    "shipped_t3.7_d0_160x90": ("shipped", 160, 90, 0, 3.7, None, 0),
    "shipped_t11.25_d1_160x90": ("shipped", 160, 90, 1, 11.25, None, 0),
    # unit-level probes (P4): world ray dir, (object, t, shadow mask), normal, point
    "probe_dir_t0_128": ("shipped", 128, 128, 0, 0.0, None, 1),
    "probe_hit_t0_128": ("shipped", 128, 128, 0, 0.0, None, 2),
    "probe_normal_t0_128": ("shipped", 128, 128, 0, 0.0, None, 3),
    "probe_point_t0_128": ("shipped", 128, 128, 0, 0.0, None, 4),
    # benchmark configurations; large frames as crops
    "config1_256": ("config1", 256, 256, 1, 0.0, None, 0),
    "config2_1920x1080_rows": ("config2", 1920, 1080, 0, 0.0, (0, 532, 1920, 16), 0),
    "config2_1920x1080_cols": ("config2", 1920, 1080, 0, 0.0, (944, 0, 32, 1080), 0),
    "config3_3840x2160_rows": ("config3", 3840, 2160, 2, 0.0, (0, 1076, 3840, 4), 0),
    "config4_7680x4320_crop": ("config4", 7680, 4320, 4, 0.0, (3776, 2112, 128, 16), 0),
    # the orbit camera moved (t != 0): the product's own camera path
    # (rt_make_view) against the reference at other camera positions
    "config2_t1_1920x1080_rows": ("config2", 1920, 1080, 0, 1.0, (0, 300, 1920, 8), 0),
    "config3_t2.5_3840x2160_rows": ("config3", 3840, 2160, 2, 2.5, (0, 700, 3840, 2), 0),
    "config4_t7_7680x4320_crop": ("config4", 7680, 4320, 4, 7.0, (2000, 3000, 128, 8), 0),
}


def scene_objects(scene):
    if scene == "shipped":
        return None
    return scenes.CONFIGS[scene][0]()


def main(names=None):
    manifest_path = os.path.join(OUT, "manifest.json")
    manifest = {}
    if os.path.exists(manifest_path):
        with open(manifest_path) as f:
            manifest = json.load(f)
    info = {"renderer": glref.renderer(), "shader": shader_meta()}
    for name, (scene, w, h, depth, t, crop, probe) in FIXTURES.items():
        if names and name not in names:
            continue
        objs = scene_objects(scene)
        t0 = time.time()
        rgba, _ = glref.render(objs, w, h, depth, t, crop=crop, probe=probe)
        dt = time.time() - t0
        assert np.all(rgba[..., 3] == 0.0), name  # imageStore(vec4(rgb, 0.0)), :404
        # llvmpipe's own inverse(proj*view) (:383) for this scene/time (probe 5),
        # so tests can pin the frame constants and compare per-pixel work alone
        pm, _ = glref.render(objs, w, h, depth, t, crop=(0, 0, 4, 4), probe=5)
        unproj = np.ascontiguousarray(pm[:, :, 0].T)  # [col][row]
        np.savez_compressed(os.path.join(OUT, name + ".npz"), rgb=rgba[..., :3].copy(), unproj=unproj)
        manifest[name] = {"scene": scene, "width": w, "height": h, "max_depth": depth, "time": t,
                          "crop": list(crop) if crop else [0, 0, w, h], "probe": probe,
                          "seconds": round(dt, 3), **info}
        print("%-32s %8.2fs" % (name, dt), flush=True)
    with open(manifest_path, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def shader_meta():
    s = glref.shader_info()
    s["path"] = "OpenGLRaytracer/raytrace_compute.glsl"
    return s


if __name__ == "__main__":
    main(sys.argv[1:] or None)
