"""MI355X-native per-pixel ray tracer — host-side Python front-end of the C-ABI.

The hot path (raytrace_compute.glsl of blubs/OpenGLRaytracer) runs as a HIP
kernel in libopenglraytracer_amd.so (built in-tree by `make -C
openglraytracer_amd/csrc`, or __graft_entry__.build()). This module is a thin
ctypes binding of include/rt.h mirroring the reference's frame driver
(OpenGLRaytracer/main.cpp:219-238): build a scene, pick `time`, render a
W x H frame into a float RGBA surface.

There is no CPU fallback: if the library is missing, or no GPU is present,
every render call raises.
"""
import ctypes as C
import os

import numpy as np

from .abi import (RT_MAX_DEPTH, RT_OK, Camera, Light, Material, Object)  # noqa: F401
from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libopenglraytracer_amd.so")
_lib = None


class RTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("rt error %d: %s" % (code, msg))
        self.code = code


class View(C.Structure):
    """rt_view: column-major inverse(proj*view) + ray origin (include/rt.h)."""
    _fields_ = [("unprojection", C.c_float * 16), ("origin", C.c_float * 3)]


def lib():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libopenglraytracer_amd.so not built: run __graft_entry__.build() "
                               "or `make -C openglraytracer_amd/csrc`")
        # One HIP runtime per process: PyTorch-ROCm bundles its own
        # libamdhip64 (loaded by `import torch` under the unversioned name),
        # while this library links the SONAME libamdhip64.so.7. Importing torch
        # first lets the dynamic linker bind this library to torch's runtime,
        # so device pointers, streams and RCCL are shared; the other order
        # would load two runtimes and torch would find no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, i, f = C.c_void_p, C.c_int, C.c_float
        sig = {
            "rt_reference_materials": ([vp], i), "rt_reference_lights": ([vp], i),
            "rt_reference_objects": ([f, vp], i), "rt_reference_camera": ([f, vp], i),
            "rt_bench_objects": ([i, C.c_uint64, vp], i), "rt_make_view": ([vp, f, vp], i),
            "rt_object_transforms": ([vp, vp, vp, vp], i),
            "rt_create": ([i, vp], i), "rt_destroy": ([vp], None),
            "rt_scene_create": ([vp, vp, i, vp, i, vp, i, vp], i), "rt_scene_destroy": ([vp], None),
            "rt_scene_update": ([vp, vp, vp, i, vp, i, vp, i], i),
            "rt_render": ([vp, vp, vp, f, i, i, i, i, i, vp, i, vp], i),
            "rt_render_view": ([vp, vp, vp, i, i, i, i, i, vp, i, vp], i),
            "rt_shard_rows": ([i, i, i, i], i),
            "rt_render_shard": ([vp, vp, vp, i, i, i, i, i, i, vp, vp], i),
            "rt_last_kernel_ms": ([vp, C.POINTER(C.c_float)], i),
            "rt_context_set": ([vp, i, i], i),
            "rt_render_batch": ([vp, vp, vp, i, i, i, i, i, i, i, vp, vp], i),
            "rt_batch_launches": ([vp, vp, i, i], i),
            "rt_render_batch_scenes": ([vp, vp, vp, i, i, i, i, i, i, i, vp, vp], i),
            "rt_render_accumulate": ([vp, vp, vp, i, i, i, i, i, C.c_uint32, i, i, i, vp, vp], i),
            "rt_pack_rgba8": ([vp, C.c_size_t, vp], i),
            "rt_write_ppm": ([C.c_char_p, vp, i, i], i), "rt_write_pfm": ([C.c_char_p, vp, i, i], i),
            "rt_last_error": ([], C.c_char_p), "rt_version": ([], C.c_char_p),
            "rt_scene_desc_parse": ([C.c_char_p, f, vp, i, vp, vp, i, vp, vp, i, vp, vp, vp], i),
            "rt_multi_create": ([i, vp, i, vp], i), "rt_multi_destroy": ([vp], None),
            "rt_render_multi": ([vp, vp, vp, f, i, i, i, i, vp, i], i),
            "rt_render_multi_view": ([vp, vp, vp, i, i, i, i, vp, i], i),
            "rt_multi_last_ms": ([vp, vp, vp, vp], i),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def _check(rc):
    if rc != RT_OK:
        raise RTError(rc, lib().rt_last_error().decode())


# ---- reference scene / camera (raytrace_compute.glsl:74-364) ---------------
def reference_materials():
    m = (Material * 7)()
    _check(lib().rt_reference_materials(m))
    return list(m)


def reference_lights():
    ls = (Light * 3)()
    _check(lib().rt_reference_lights(ls))
    return list(ls)


def reference_objects(time=0.0):
    o = (Object * 5)()
    _check(lib().rt_reference_objects(time, o))
    return list(o)


def reference_camera(time=0.0):
    c = Camera()
    _check(lib().rt_reference_camera(time, C.byref(c)))
    return c


def bench_objects(n_spheres, seed=0):
    o = (Object * (n_spheres + 1))()
    _check(lib().rt_bench_objects(n_spheres, seed, o))
    return list(o)


def parse_scene(text, time=0.0):
    """rt_scene_desc_parse: a JSON scene description -> (objects, materials,
    lights, camera or None) as ctypes records (format:
    openglraytracer_amd/csrc/rt_scene_json.cpp)."""
    objs = (Object * abi.RT_MAX_OBJECTS)()
    mats = (Material * abi.RT_MAX_MATERIALS)()
    lts = (Light * abi.RT_MAX_LIGHTS)()
    cam = Camera()
    no, nm, nl, hc = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    data = text.encode() if isinstance(text, str) else bytes(text)
    _check(lib().rt_scene_desc_parse(data, time, objs, abi.RT_MAX_OBJECTS, C.byref(no), mats, abi.RT_MAX_MATERIALS,
                                     C.byref(nm), lts, abi.RT_MAX_LIGHTS, C.byref(nl), C.byref(cam), C.byref(hc)))
    return list(objs[:no.value]), list(mats[:nm.value]), list(lts[:nl.value]), (cam if hc.value else None)


def make_view(camera=None, time=0.0):
    v = View()
    _check(lib().rt_make_view(C.byref(camera) if camera is not None else None, time, C.byref(v)))
    return v


def view_from_matrix(unprojection, origin):
    """An explicit view: 16 column-major floats + 3-float origin."""
    v = View()
    v.unprojection[:] = [float(x) for x in np.asarray(unprojection, np.float32).reshape(-1)]
    v.origin[:] = [float(x) for x in np.asarray(origin, np.float32).reshape(-1)]
    return v


def shard_rows(height, block_rows, n_shards, shard):
    n = lib().rt_shard_rows(height, block_rows, n_shards, shard)
    if n < 0:
        raise RTError(n, "bad shard arguments")
    return n


def shard_row_ids(height, block_rows, n_shards, shard):
    """Frame rows owned by `shard`, in the order rt_render_shard packs them."""
    rows = np.arange(height)
    return rows[(rows // block_rows) % n_shards == shard]


def pack_rgba8(rgba):
    """GL_RGBA8 unorm packing of a float frame (the shipped surface)."""
    a = np.ascontiguousarray(rgba, np.float32)
    out = np.zeros(a.shape, np.uint8)
    _check(lib().rt_pack_rgba8(a.ctypes.data, a.size // 4, out.ctypes.data))
    return out


def write_ppm(path, rgba):
    """8-bit PPM of a frame (RGBA8 rounding, top row first)."""
    a = np.ascontiguousarray(rgba, np.float32)
    _check(lib().rt_write_ppm(os.fsencode(path), a.ctypes.data, a.shape[1], a.shape[0]))


def write_pfm(path, rgba):
    """Float PFM of a frame (bottom row first, little-endian)."""
    a = np.ascontiguousarray(rgba, np.float32)
    _check(lib().rt_write_pfm(os.fsencode(path), a.ctypes.data, a.shape[1], a.shape[0]))


class Context:
    """One device (rt_create). Not thread-safe, like a GL context."""

    def __init__(self, device=0):
        self._h = C.c_void_p()
        _check(lib().rt_create(device, C.byref(self._h)))
        self.device = device
        self.output = abi.RT_OUTPUT_RGBA32F  # RT_OPT_OUTPUT (set_output)

    def close(self):
        if self._h:
            lib().rt_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_culling(self, on):
        """RT_OPT_CULLING: conservative sphere culling (output identical)."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_CULLING, 1 if on else 0))

    def set_timing(self, on):
        """RT_OPT_TIMING: HIP events around every launch (for last_kernel_ms)."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_TIMING, 1 if on else 0))

    def set_host_frame_consts(self, on):
        """RT_OPT_FRAME_CONSTS: per-frame constants from the host when they fit
        (default), else derived by every work-group (output identical)."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_FRAME_CONSTS, 1 if on else 0))

    def set_origin_lists(self, on):
        """RT_OPT_ORIGIN_LISTS: secondary rays leaving a sphere test its
        precomputed candidate list instead of walking the BVH (output identical)."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_ORIGIN_LISTS, 1 if on else 0))

    def set_scene_shapes(self, on):
        """RT_OPT_SCENE_SHAPES: a render whose scene has a common shape runs
        the kernel compiled for it (include/rt.h): at depth 0, LDS-mask scenes
        (the mask width as a constant); at depth >= 2 without Monte-Carlo,
        scenes with wide masks, their candidate lists and origin-sphere lists;
        each with or without the room (one translate-only box holding every
        live light). Output identical either way."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_SCENE_SHAPES, 1 if on else 0))

    def set_output(self, fmt):
        """RT_OPT_OUTPUT: abi.RT_OUTPUT_RGBA32F (float4 per pixel),
        abi.RT_OUTPUT_RGBA8 (the shipped GL_RGBA8 surface, 4 bytes per pixel)
        or abi.RT_OUTPUT_RGB32F (packed float3, the constant alpha dropped)."""
        _check(lib().rt_context_set(self._h, abi.RT_OPT_OUTPUT, fmt))
        self.output = fmt

    def last_kernel_ms(self):
        ms = C.c_float()
        _check(lib().rt_last_kernel_ms(self._h, C.byref(ms)))
        return ms.value


class Scene:
    """Device-resident scene (rt_scene_create). Defaults: the reference's
    7 materials and 3 lights."""

    def __init__(self, ctx, objects, materials=None, lights=None):
        materials = materials if materials is not None else reference_materials()
        lights = lights if lights is not None else reference_lights()
        objs = (Object * max(len(objects), 1))(*objects)
        mats = (Material * len(materials))(*materials)
        lts = (Light * max(len(lights), 1))(*lights)
        self._h = C.c_void_p()
        _check(lib().rt_scene_create(ctx.handle, objs, len(objects), mats, len(materials), lts,
                                     len(lights), C.byref(self._h)))
        self.ctx = ctx

    def update(self, objects, materials=None, lights=None):
        """Replace the contents (rt_scene_update), e.g. the next animation frame."""
        materials = materials if materials is not None else reference_materials()
        lights = lights if lights is not None else reference_lights()
        objs = (Object * max(len(objects), 1))(*objects)
        mats = (Material * len(materials))(*materials)
        lts = (Light * max(len(lights), 1))(*lights)
        _check(lib().rt_scene_update(self.ctx.handle, self._h, objs, len(objects), mats, len(materials), lts,
                                     len(lights)))

    def close(self):
        if self._h:
            lib().rt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h


def surface(fmt, *shape):
    """A zeroed host array for `shape` pixels in surface format `fmt`
    (RT_OPT_OUTPUT): float32 x4 (RGBA32F), float32 x3 (RGB32F) or uint8 x4
    (RGBA8)."""
    if fmt == abi.RT_OUTPUT_RGBA8:
        return np.zeros(shape + (4,), np.uint8)
    if fmt == abi.RT_OUTPUT_RGB32F:
        return np.zeros(shape + (3,), np.float32)
    return np.zeros(shape + (4,), np.float32)


def render(ctx, scene, width, height, max_depth=0, time=0.0, camera=None, view=None, rows=None):
    """Render rows [r0, r1) to a host array, synchronously (the reference's
    glDispatchCompute + glFinish): (r1-r0, width, C) in the context's surface
    format (ctx.set_output): float32 RGBA (default), float32 RGB or uint8
    RGBA."""
    r0, r1 = rows if rows is not None else (0, height)
    out = surface(ctx.output, max(r1 - r0, 1), max(width, 1))  # the C-ABI validates the range
    if view is None:
        view = make_view(camera, time)
    _check(lib().rt_render_view(ctx.handle, scene.handle, C.byref(view), width, height, max_depth,
                                r0, r1, out.ctypes.data, 0, None))
    return out[: r1 - r0, :width]


def render_rgba8(ctx, scene, width, height, max_depth=0, time=0.0, camera=None, view=None, rows=None):
    """Render rows [r0, r1) as the shipped app's GL_RGBA8 surface: a host
    array (r1-r0, width, 4) uint8, packed by the kernel's epilogue (equal to
    pack_rgba8 of the float frame)."""
    r0, r1 = rows if rows is not None else (0, height)
    out = np.zeros((max(r1 - r0, 1), max(width, 1), 4), np.uint8)
    if view is None:
        view = make_view(camera, time)
    prev = getattr(ctx, "output", abi.RT_OUTPUT_RGBA32F)
    ctx.set_output(abi.RT_OUTPUT_RGBA8)
    try:
        _check(lib().rt_render_view(ctx.handle, scene.handle, C.byref(view), width, height, max_depth,
                                    r0, r1, out.ctypes.data, 0, None))
    finally:
        ctx.set_output(prev)
    return out[: r1 - r0, :width]


def render_device(ctx, scene, out_ptr, width, height, max_depth=0, view=None, rows=None,
                  stream=None):
    """Render into device memory `out_ptr` (e.g. torch tensor.data_ptr()),
    laid out (rows, width, C) in the context's surface format; with `stream`
    (a hipStream_t as int) the call is asynchronous on that stream."""
    r0, r1 = rows if rows is not None else (0, height)
    if view is None:
        view = make_view(None, 0.0)
    _check(lib().rt_render_view(ctx.handle, scene.handle, C.byref(view), width, height, max_depth,
                                r0, r1, C.c_void_p(out_ptr), 1,
                                C.c_void_p(stream) if stream else None))


def render_batch(ctx, scene, out_ptr, width, height, max_depth, views, block_rows=8, n_shards=1,
                 shard=0, stream=None):
    """K frames (K = len(views) <= abi.RT_MAX_BATCH = 256) in one launch
    (depth 0-1; deeper frames in even queued launches of as many views as fit
    beside the scene in LDS, include/rt.h) into device memory laid out
    (K, rows, width, C) (C and dtype: the context's surface format); rows =
    height, or this shard's rows."""
    arr = (View * len(views))(*views)
    _check(lib().rt_render_batch(ctx.handle, scene.handle, arr, len(views), width, height, max_depth,
                                 block_rows, n_shards, shard, C.c_void_p(out_ptr),
                                 C.c_void_p(stream) if stream else None))


def batch_launches(ctx, scene, n_views, max_depth):
    """Kernel launches render_batch makes for n_views views of `scene` at
    max_depth (deep batches split into queued launches of as many views as
    fit beside the scene in LDS)."""
    n = lib().rt_batch_launches(ctx.handle, scene.handle, n_views, max_depth)
    if n < 0:
        raise RTError(n, lib().rt_last_error().decode())
    return n


def render_batch_scenes(ctx, scenes, out_ptr, width, height, max_depth, views, block_rows=8, n_shards=1,
                        shard=0, stream=None):
    """K animated frames in one launch: views[k] of scenes[k] (same layout),
    into device memory (K, rows, width, C) in the context's surface format."""
    arr = (View * len(views))(*views)
    sarr = (C.c_void_p * len(scenes))(*[s.handle for s in scenes])
    _check(lib().rt_render_batch_scenes(ctx.handle, sarr, arr, len(views), width, height, max_depth, block_rows,
                                        n_shards, shard, C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None))


def render_accumulate(ctx, scene, accum_ptr, width, height, max_depth, spp, sample_offset=0, seed=0,
                      jitter=True, view=None, rows=None, stream=None):
    """Monte-Carlo: add the sum of samples [sample_offset, sample_offset+spp)
    of every pixel to the float4 device accumulator at accum_ptr."""
    r0, r1 = rows if rows is not None else (0, height)
    if view is None:
        view = make_view(None, 0.0)
    _check(lib().rt_render_accumulate(ctx.handle, scene.handle, C.byref(view), width, height, max_depth, spp,
                                      sample_offset, seed, 1 if jitter else 0, r0, r1, C.c_void_p(accum_ptr),
                                      C.c_void_p(stream) if stream else None))


def render_shard(ctx, scene, out_ptr, width, height, max_depth, block_rows, n_shards, shard,
                 view=None, stream=None):
    """Render this shard's interleaved row blocks into device memory
    (rows, width, C) in the context's surface format."""
    if view is None:
        view = make_view(None, 0.0)
    _check(lib().rt_render_shard(ctx.handle, scene.handle, C.byref(view), width, height, max_depth,
                                 block_rows, n_shards, shard, C.c_void_p(out_ptr),
                                 C.c_void_p(stream) if stream else None))


class Multi:
    """One frame on several GPUs of this process (rt_multi_create /
    rt_render_multi): interleaved row blocks per context, gathered to the
    first context's GPU (RCCL, or peer copies with transport=RT_MULTI_COPY,
    which also serves contexts sharing a device) and de-interleaved there."""

    def __init__(self, contexts, transport=abi.RT_MULTI_RCCL):
        self.contexts = list(contexts)
        arr = (C.c_void_p * len(self.contexts))(*[c.handle for c in self.contexts])
        self._h = C.c_void_p()
        _check(lib().rt_multi_create(len(self.contexts), arr, transport, C.byref(self._h)))

    def render(self, scenes, width, height, max_depth=0, time=0.0, camera=None, view=None, block_rows=8):
        """The whole frame as a host array in the root context's surface format."""
        out = surface(self.contexts[0].output, max(height, 1), max(width, 1))
        self._render(scenes, width, height, max_depth, time, camera, view, block_rows, out.ctypes.data, 0)
        return out[:height, :width]

    def render_device(self, scenes, out_ptr, width, height, max_depth=0, time=0.0, camera=None, view=None,
                      block_rows=8):
        """The whole frame into device memory of the root context's GPU."""
        self._render(scenes, width, height, max_depth, time, camera, view, block_rows, out_ptr, 1)

    def _render(self, scenes, width, height, max_depth, time, camera, view, block_rows, ptr, is_device):
        sarr = (C.c_void_p * len(scenes))(*[s.handle for s in scenes])
        if view is not None:
            _check(lib().rt_render_multi_view(self._h, sarr, C.byref(view), width, height, max_depth, block_rows,
                                              C.c_void_p(ptr), is_device))
        else:
            _check(lib().rt_render_multi(self._h, sarr, C.byref(camera) if camera is not None else None, time,
                                         width, height, max_depth, block_rows, C.c_void_p(ptr), is_device))

    def last_ms(self):
        """(per-GPU kernel ms, gather ms, assembly ms) of the last render."""
        k = (C.c_float * len(self.contexts))()
        g, a = C.c_float(), C.c_float()
        _check(lib().rt_multi_last_ms(self._h, k, C.byref(g), C.byref(a)))
        return list(k), g.value, a.value

    def close(self):
        if self._h:
            lib().rt_multi_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
