"""ctypes mirror of include/rt.h (data layout only; loads nothing).

Every struct follows the GLSL struct it replaces
(/root/reference/OpenGLRaytracer/raytrace_compute.glsl:36-50, 56-69, 190-196,
244-258); see include/rt.h for the field-by-field citations.
"""
import ctypes as C

import numpy as np

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_HIP = -2
RT_ERR_NOMEM = -3
RT_ERR_UNSUPPORTED = -4
RT_ERR_NO_DEVICE = -5
RT_MAX_DEPTH = 9
RT_MAX_OBJECTS = 1024
RT_MAX_LIGHTS = 16
RT_MAX_MATERIALS = 256
RT_OPT_CULLING = 1
RT_OPT_TIMING = 2
RT_OPT_OUTPUT = 3
RT_OPT_FRAME_CONSTS = 4
RT_OPT_ORIGIN_LISTS = 7
RT_OPT_SCENE_SHAPES = 8
RT_OUTPUT_RGBA32F = 0
RT_OUTPUT_RGBA8 = 1
RT_OUTPUT_RGB32F = 2
RT_MAX_BATCH = 256
RT_MULTI_RCCL = 0
RT_MULTI_COPY = 1

# material indices of the reference table (raytrace_compute.glsl:74-157)
MATERIAL1, MATERIAL2, RED_GLASS, GREEN_GLASS, BLUE_GLASS, MIRROR, WALL = range(7)
MATERIAL_NAMES = ["material1", "material2", "red_glass_material", "green_glass_material",
                  "blue_glass_material", "mirror_material", "wall_material"]

F3 = C.c_float * 3
F4 = C.c_float * 4


class Material(C.Structure):
    _fields_ = [("ambient", F4), ("diffuse", F4), ("specular", F4), ("shininess", C.c_float),
                ("emissive", F4), ("reflectivity", C.c_float), ("transparency", C.c_float),
                ("refraction_index", C.c_float)]


class Object(C.Structure):
    _fields_ = [("box_mins", F3), ("box_maxs", F3), ("radius", C.c_float), ("position", F3),
                ("angles", F3), ("material", C.c_int32)]


class Light(C.Structure):
    _fields_ = [("position", F3), ("ambient", F4), ("diffuse", F4), ("specular", F4)]


class Camera(C.Structure):
    _fields_ = [("position", F3), ("angles", F3), ("v_fov", C.c_float), ("aspect", C.c_float),
                ("near_plane", C.c_float), ("far_plane", C.c_float)]


def array(struct, items):
    """Build a ctypes array of `struct` from a list of structs."""
    arr = (struct * max(len(items), 1))()
    for i, it in enumerate(items):
        arr[i] = it
    return arr


def to_numpy(arr, n=None):
    """Flat float32 view of a ctypes struct array (for fixtures / hashing)."""
    n = len(arr) if n is None else n
    raw = bytes(memoryview(arr).cast("B"))[: n * C.sizeof(arr._type_)]
    return np.frombuffer(raw, dtype=np.uint8).copy()
