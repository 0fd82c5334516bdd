"""ctypes front-end of the llvmpipe harness (oracle/glref/glref.c).

TEST INFRASTRUCTURE ONLY. Runs the reference's own raytrace_compute.glsl on
Mesa llvmpipe; needs oracle/_ref/libglref.so (built from /root/reference by
`make -C oracle ref`). Used to generate tests/golden and, where the built
library travelled to the GPU box, as bench.py's CPU baseline.
"""
import ctypes as C
import os

import numpy as np

from openglraytracer_amd.abi import MATERIAL_NAMES

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_ref", "libglref.so")
_lib = None


def available():
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise RuntimeError("llvmpipe harness not built (needs /root/reference): make -C oracle ref")
        L = C.CDLL(LIB_PATH)
        L.glref_render.argtypes = [C.c_char_p, C.c_int, C.c_float] + [C.c_int] * 8 + [C.c_void_p, C.c_void_p]
        L.glref_render.restype = C.c_int
        L.glref_last_error.restype = C.c_char_p
        L.glref_renderer.restype = C.c_char_p
        L.glref_shader_hash.restype = C.c_ulonglong
        L.glref_shader_size.restype = C.c_long
        L.glref_init.restype = C.c_int
        L.glref_render_rgba8.argtypes = [C.c_char_p, C.c_int, C.c_float] + [C.c_int] * 6 + [C.c_void_p]
        L.glref_render_rgba8.restype = C.c_int
        _lib = L
    return _lib


def _f(x):
    return "%.9e" % float(np.float32(x))


def objects_glsl(objects):
    """GLSL text replacing raytrace_compute.glsl:261-321 (patch P3)."""
    items = []
    for o in objects:
        mins = "vec3(%s, %s, %s)" % tuple(_f(v) for v in o.box_mins)
        maxs = "vec3(%s, %s, %s)" % tuple(_f(v) for v in o.box_maxs)
        pos = "vec3(%s, %s, %s)" % tuple(_f(v) for v in o.position)
        ang = "vec3(%s, %s, %s)" % tuple(_f(v) for v in o.angles)
        items.append("\t{ { %s, %s }, { %s }, %s, %s, %s }" % (
            mins, maxs, _f(o.radius), pos, ang, MATERIAL_NAMES[o.material]))
    return "Object[] objects =\n{\n%s\n};\nint objects_count = %d;" % (",\n".join(items), len(objects))


def renderer():
    L = lib()
    if L.glref_init() != 0:
        raise RuntimeError(L.glref_last_error().decode())
    return L.glref_renderer().decode()


def shader_info():
    L = lib()
    return {"fnv1a64": "%016x" % L.glref_shader_hash(), "bytes": int(L.glref_shader_size())}


def render(objects, width, height, max_depth=0, time=0.0, crop=None, probe=0, repeats=0):
    """Render the reference shader. objects=None keeps the shipped scene.
    crop=(x0, y0, w, h). Returns (rgba float32 (h, w, 4), sorted dispatch seconds)."""
    x0, y0, w, h = crop if crop is not None else (0, 0, width, height)
    out = np.zeros((h, w, 4), np.float32)
    times = np.zeros(max(repeats, 1), np.float64)
    src = objects_glsl(objects).encode() if objects is not None else None
    rc = lib().glref_render(src, max_depth, C.c_float(time), width, height, x0, y0, w, h, probe,
                            repeats, out.ctypes.data, times.ctypes.data)
    if rc != 0:
        raise RuntimeError("glref: " + lib().glref_last_error().decode())
    return out, times[:repeats]


def render_rgba8(objects, width, height, max_depth=0, time=0.0, crop=None):
    """The same render into the shipped app's GL_RGBA8 surface: uint8 (h, w, 4)."""
    x0, y0, w, h = crop if crop is not None else (0, 0, width, height)
    out = np.zeros((h, w, 4), np.uint8)
    src = objects_glsl(objects).encode() if objects is not None else None
    rc = lib().glref_render_rgba8(src, max_depth, C.c_float(time), width, height, x0, y0, w, h, out.ctypes.data)
    if rc != 0:
        raise RuntimeError("glref: " + lib().glref_last_error().decode())
    return out
