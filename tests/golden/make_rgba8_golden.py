"""Golden RGBA8 surfaces from the reference itself (the shipped app's format).

The reference renders into a GL_RGBA8 texture (OpenGLRaytracer/main.cpp:
152-159, bound with glBindImageTexture(..., GL_RGBA8) at :223), so the GL
driver converts each imageStore(vec4(final_color, 0.0)) (:404) to unorm
bytes. The llvmpipe harness (oracle/glref, glref_render_rgba8) renders the
reference's own shader into such a surface; this script stores those bytes
next to the RGBA32F render of the same frame, for:
  * the host packing rt_pack_rgba8 (float frame -> bytes, tests/test_host.py);
  * the kernel's RGBA8 epilogue (RT_OUTPUT_RGBA8) through rt_render with the
    product's own camera (tests/test_gpu_parity.py).

Writes tests/golden/rgba8_llvmpipe.npz: for each case, `<name>_rgba8` uint8
(h, w, 4), `<name>_rgba32f` float32 (h, w, 4) and `<name>_meta`
(width, height, depth, time, x0, y0, w, h; scene "shipped" or a configs key
in `<name>_scene`).

    python tests/golden/make_rgba8_golden.py      # needs oracle/_ref (make -C oracle ref)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import glref, scenes  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rgba8_llvmpipe.npz")
# name: (scene, width, height, depth, time, crop)
CASES = {
    "shipped_t0_d0_256": ("shipped", 256, 256, 0, 0.0, (0, 0, 256, 256)),
    "shipped_t3.7_d1_160x90": ("shipped", 160, 90, 1, 3.7, (0, 0, 160, 90)),
    "config2_rows": ("config2", 1920, 1080, 0, 0.0, (0, 532, 1920, 16)),
}


def main():
    data = {}
    for name, (scene, w, h, depth, t, crop) in CASES.items():
        objs = None if scene == "shipped" else scenes.CONFIGS[scene][0]()
        b = glref.render_rgba8(objs, w, h, depth, t, crop)
        f, _ = glref.render(objs, w, h, depth, t, crop)
        data[name + "_rgba8"] = b
        data[name + "_rgba32f"] = f
        data[name + "_meta"] = np.array([w, h, depth, t, *crop], np.float64)
        data[name + "_scene"] = np.array(scene)
        print(name, b.shape)
    data["renderer"] = np.array(glref.renderer())
    np.savez_compressed(OUT, **data)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
