// rt_api.cpp — the C-ABI (include/rt.h): contexts, scenes, render calls.
//
// The counterpart of the reference's frame driver (OpenGLRaytracer/main.cpp:
// 203 program creation, :219-238 draw(): bind image, set `time`,
// glDispatchCompute(W, H, 1), glFinish). No exception crosses this boundary;
// failures return RT_ERR_* and leave a thread-local message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt_internal.h"

namespace rtamd {

namespace {
thread_local std::string g_error;

int hip_fail(const char *what, hipError_t e) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RT_ERR_HIP;
}

// Largest LDS a work-group may request on gfx950 (160 KiB).
constexpr size_t kMaxLds = 160 * 1024;
}  // namespace

void set_error(const std::string &msg) { g_error = msg; }

int build_scene(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats, const rt_light *lights,
                int n_lights, std::vector<float4> &blob, DeviceScene &ds);
hipError_t allow_large_lds(size_t bytes);
bool view_projection(const rt_view &v, float proj[16]);

}  // namespace rtamd

using namespace rtamd;

namespace {

int check_render_args(const rt_context *ctx, const rt_scene *scene, int width, int height, int max_depth) {
    if (!ctx || !scene) {
        set_error("null context or scene");
        return RT_ERR_INVALID;
    }
    if (scene->device != ctx->device) {
        set_error("scene was created on another device");
        return RT_ERR_INVALID;
    }
    if (width <= 0 || height <= 0 || width > 65536 || height > 65536) {
        set_error("bad frame size");
        return RT_ERR_INVALID;
    }
    if (max_depth < 0 || max_depth > RT_MAX_DEPTH) {
        set_error("max_depth " + std::to_string(max_depth) + " outside [0, " + std::to_string(RT_MAX_DEPTH) + "]");
        return RT_ERR_UNSUPPORTED;
    }
    return RT_OK;
}

LaunchParams base_params(const rt_context *ctx, const rt_scene *scene, const rt_view *views, int n_views,
                         int width, int height) {
    LaunchParams p{};
    p.n_views = n_views;
    for (int k = 0; k < n_views; ++k) {
        FrameView &v = p.view[k];
        v.cull = (view_projection(views[k], v.proj) && ctx->culling) ? 1 : 0;
        std::memcpy(v.unproj, views[k].unprojection, sizeof v.unproj);
        std::memcpy(v.origin, views[k].origin, sizeof v.origin);
    }
    p.width = width;
    p.height = height;
    const DeviceScene &d = scene->dev;
    p.n_spheres = d.n_spheres;
    p.n_boxes = d.n_boxes;
    p.n_mats = d.n_mats;
    p.n_lights = d.n_lights;
    p.scene = d.blob;
    p.off_spheres = d.off_spheres;
    p.off_smeta = d.off_smeta;
    p.off_boxes = d.off_boxes;
    p.off_mats = d.off_mats;
    p.off_lights = d.off_lights;
    p.off_lightmat = d.off_lightmat;
    p.off_bvh = d.off_bvh;
    p.off_cone = d.off_cone;
    p.off_dmask = d.off_dmask;
    p.dmask_n = d.dmask_n;
    p.dmask_bytes = d.dmask_bytes;
    p.off_gmask = d.off_gmask;
    p.gmask_words = d.gmask_words;
    p.out_format = ctx->output;
    p.n_bvh = d.n_bvh;
    p.blob_units = d.blob_units;
    if (ctx->host_consts) {
        const float4 *blobs[kMaxViews];
        for (int k = 0; k < n_views; ++k) blobs[k] = scene->host.empty() ? nullptr : scene->host.data();
        host_frame_setup(p, blobs);
    }
    return p;
}

// Launch on `stream` with kernel-time events on the context.
int launch(rt_context *ctx, LaunchParams &p, int max_depth, hipStream_t stream) {
    p.n_cu = ctx->n_cu;
    p.sched = ctx->sched + static_cast<size_t>(ctx->sched_next++ % kSchedSlots) * kSchedInts;
    hipError_t e;
    if (ctx->timing && (e = hipEventRecord(ctx->ev0, stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
    e = launch_render(p, max_depth, stream);
    if (e != hipSuccess) return hip_fail("kernel launch", e);
    if (ctx->timing) {
        if ((e = hipEventRecord(ctx->ev1, stream)) != hipSuccess) return hip_fail("hipEventRecord", e);
        ctx->timed = true;
    } else {
        ctx->timed = false;
    }
    return RT_OK;
}

}  // namespace

extern "C" {

const char *rt_last_error(void) { return g_error.c_str(); }
const char *rt_version(void) { return "openglraytracer_amd 0.1 (gfx950)"; }

int rt_create(int device, rt_context **out) {
    if (!out) { set_error("rt_create: null out"); return RT_ERR_INVALID; }
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        set_error("rt_create: no HIP device");
        return RT_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= n) {
        set_error("rt_create: device " + std::to_string(device) + " out of range");
        return RT_ERR_NO_DEVICE;
    }
    if ((e = hipSetDevice(device)) != hipSuccess) return hip_fail("hipSetDevice", e);
    rt_context *ctx = new (std::nothrow) rt_context;
    if (!ctx) { set_error("rt_create: out of memory"); return RT_ERR_NOMEM; }
    ctx->device = device;
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&ctx->ev0)) != hipSuccess || (e = hipEventCreate(&ctx->ev1)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess ||
        (e = hipMalloc(&ctx->sched, sizeof(int32_t) * kSchedInts * kSchedSlots)) != hipSuccess ||
        (e = hipMemset(ctx->sched, 0, sizeof(int32_t) * kSchedInts * kSchedSlots)) != hipSuccess ||
        (e = allow_large_lds(kMaxLds)) != hipSuccess) {
        rt_destroy(ctx);
        return hip_fail("rt_create", e);
    }
    *out = ctx;
    return RT_OK;
}

void rt_destroy(rt_context *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->staging) (void)hipFree(ctx->staging);
    if (ctx->sched) (void)hipFree(ctx->sched);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int rt_scene_create(rt_context *ctx, const rt_object *objs, int n_objs, const rt_material *mats, int n_mats,
                    const rt_light *lights, int n_lights, rt_scene **out) {
    if (!out) { set_error("rt_scene_create: null out"); return RT_ERR_INVALID; }
    *out = nullptr;
    if (!ctx || (n_objs > 0 && !objs) || n_objs < 0 || n_objs > RT_MAX_OBJECTS || !mats || n_mats <= 0 ||
        n_mats > RT_MAX_MATERIALS || n_lights < 0 || n_lights > RT_MAX_LIGHTS || (n_lights > 0 && !lights)) {
        set_error("rt_scene_create: bad arguments");
        return RT_ERR_INVALID;
    }
    std::vector<float4> blob;
    DeviceScene ds;
    int rc = build_scene(objs, n_objs, mats, n_mats, lights, n_lights, blob, ds);
    if (rc != RT_OK) return rc;
    LaunchParams probe{};
    probe.blob_units = ds.blob_units;
    probe.n_spheres = ds.n_spheres;
    probe.n_boxes = ds.n_boxes;
    const size_t lds = lds_bytes(probe);
    if (lds > kMaxLds) {
        set_error("rt_scene_create: scene needs " + std::to_string(lds) + " B of LDS (> 160 KiB)");
        return RT_ERR_UNSUPPORTED;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    e = hipMalloc(&ds.blob, blob.size() * sizeof(float4));
    if (e != hipSuccess) return hip_fail("hipMalloc(scene)", e);
    e = hipMemcpy(ds.blob, blob.data(), blob.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(ds.blob);
        return hip_fail("hipMemcpy(scene)", e);
    }
    rt_scene *s = new (std::nothrow) rt_scene;
    if (!s) {
        (void)hipFree(ds.blob);
        set_error("rt_scene_create: out of memory");
        return RT_ERR_NOMEM;
    }
    s->device = ctx->device;
    s->dev = ds;
    s->host.swap(blob);
    s->capacity_units = static_cast<int32_t>(s->host.size());
    *out = s;
    return RT_OK;
}

int rt_scene_update(rt_context *ctx, rt_scene *scene, const rt_object *objs, int n_objs, const rt_material *mats,
                    int n_mats, const rt_light *lights, int n_lights) {
    if (!ctx || !scene || scene->device != ctx->device || (n_objs > 0 && !objs) || n_objs < 0 ||
        n_objs > RT_MAX_OBJECTS || !mats || n_mats <= 0 || n_mats > RT_MAX_MATERIALS || n_lights < 0 ||
        n_lights > RT_MAX_LIGHTS || (n_lights > 0 && !lights)) {
        set_error("rt_scene_update: bad arguments");
        return RT_ERR_INVALID;
    }
    std::vector<float4> blob;
    DeviceScene ds;
    int rc = build_scene(objs, n_objs, mats, n_mats, lights, n_lights, blob, ds);
    if (rc != RT_OK) return rc;
    LaunchParams probe{};
    probe.blob_units = ds.blob_units;
    probe.n_spheres = ds.n_spheres;
    probe.n_boxes = ds.n_boxes;
    if (lds_bytes(probe) > kMaxLds) {
        set_error("rt_scene_update: scene needs more than 160 KiB of LDS");
        return RT_ERR_UNSUPPORTED;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    // renders already queued on the context's stream may still read the blob
    e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    if (static_cast<int32_t>(blob.size()) > scene->capacity_units) {
        void *nb = nullptr;
        e = hipMalloc(&nb, blob.size() * sizeof(float4));
        if (e != hipSuccess) return hip_fail("hipMalloc(scene)", e);
        (void)hipFree(scene->dev.blob);
        scene->dev.blob = nb;
        scene->capacity_units = static_cast<int32_t>(blob.size());
    }
    e = hipMemcpy(scene->dev.blob, blob.data(), blob.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail("hipMemcpy(scene)", e);
    void *keep = scene->dev.blob;
    scene->dev = ds;
    scene->dev.blob = keep;
    scene->host.swap(blob);
    return RT_OK;
}

void rt_scene_destroy(rt_scene *scene) {
    if (!scene) return;
    (void)hipSetDevice(scene->device);
    (void)hipDeviceSynchronize();
    if (scene->dev.blob) (void)hipFree(scene->dev.blob);
    delete scene;
}

int rt_render_view(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width, int height, int max_depth,
                   int row_begin, int row_end, float *out, int out_is_device, void *hip_stream) {
    int rc = check_render_args(ctx, scene, width, height, max_depth);
    if (rc != RT_OK) return rc;
    if (!view || !out || row_begin < 0 || row_end > height || row_begin >= row_end) {
        set_error("rt_render: bad view / output / row range");
        return RT_ERR_INVALID;
    }
    if (hip_stream && !out_is_device) {
        set_error("rt_render: an asynchronous render needs a device output buffer");
        return RT_ERR_INVALID;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    LaunchParams p = base_params(ctx, scene, view, 1, width, height);
    p.row_begin = row_begin;
    p.n_rows = row_end - row_begin;
    const size_t n_px = static_cast<size_t>(p.n_rows) * width;
    hipStream_t stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    const size_t px_bytes = p.out_format == RT_OUTPUT_RGBA8 ? 4 : (p.out_format == RT_OUTPUT_RGB32F ? 12 : sizeof(float4));
    if (out_is_device) {
        p.out = reinterpret_cast<float4 *>(out);
    } else {
        if (ctx->staging_px < n_px) {
            if (ctx->staging) (void)hipFree(ctx->staging);
            ctx->staging = nullptr;
            ctx->staging_px = 0;
            e = hipMalloc(&ctx->staging, n_px * sizeof(float4));  // sized for float4: serves every format
            if (e != hipSuccess) return hip_fail("hipMalloc(staging)", e);
            ctx->staging_px = n_px;
        }
        p.out = ctx->staging;
    }
    rc = launch(ctx, p, max_depth, stream);
    if (rc != RT_OK) return rc;
    if (!out_is_device) {
        e = hipMemcpyAsync(out, ctx->staging, n_px * px_bytes, hipMemcpyDeviceToHost, stream);
        if (e != hipSuccess) return hip_fail("hipMemcpyAsync(out)", e);
    }
    if (!hip_stream) {
        e = hipStreamSynchronize(stream);  // glFinish (main.cpp:238)
        if (e != hipSuccess) return hip_fail("render", e);
    }
    return RT_OK;
}

int rt_render(rt_context *ctx, const rt_scene *scene, const rt_camera *cam, float time, int width, int height,
              int max_depth, int row_begin, int row_end, float *out, int out_is_device, void *hip_stream) {
    rt_view view;
    int rc = rt_make_view(cam, time, &view);
    if (rc != RT_OK) return rc;
    return rt_render_view(ctx, scene, &view, width, height, max_depth, row_begin, row_end, out, out_is_device,
                          hip_stream);
}

int rt_shard_rows(int height, int block_rows, int n_shards, int shard) {
    if (height <= 0 || block_rows <= 0 || n_shards <= 0 || shard < 0 || shard >= n_shards) return RT_ERR_INVALID;
    const int full = height / block_rows, tail = height % block_rows;
    int rows = (full / n_shards) * block_rows;
    const int extra = full % n_shards;  // leftover full blocks go to shards 0..extra-1
    if (shard < extra) rows += block_rows;
    if (tail && shard == full % n_shards) rows += tail;
    return rows;
}

int rt_render_shard(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width, int height,
                    int max_depth, int block_rows, int n_shards, int shard, float *out_device, void *hip_stream) {
    int rc = check_render_args(ctx, scene, width, height, max_depth);
    if (rc != RT_OK) return rc;
    const int rows = rt_shard_rows(height, block_rows, n_shards, shard);
    if (!view || !out_device || rows < 0) {
        set_error("rt_render_shard: bad view / output / shard arguments");
        return RT_ERR_INVALID;
    }
    if (rows == 0) return RT_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    LaunchParams p = base_params(ctx, scene, view, 1, width, height);
    p.row_begin = 0;
    p.n_rows = rows;
    p.block_rows = block_rows;
    p.n_shards = n_shards;
    p.shard = shard;
    p.out = reinterpret_cast<float4 *>(out_device);
    hipStream_t stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    rc = launch(ctx, p, max_depth, stream);
    if (rc != RT_OK) return rc;
    if (!hip_stream) {
        e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail("render", e);
    }
    return RT_OK;
}

}  // extern "C"

namespace {
// Same blob layout (section offsets and counts): views of these scenes can
// share one launch, each work-group staging its own view's blob.
bool same_layout(const DeviceScene &a, const DeviceScene &b) {
    return a.blob_units == b.blob_units && a.off_spheres == b.off_spheres && a.off_smeta == b.off_smeta &&
           a.off_boxes == b.off_boxes && a.off_mats == b.off_mats && a.off_lights == b.off_lights &&
           a.off_lightmat == b.off_lightmat && a.off_bvh == b.off_bvh && a.n_bvh == b.n_bvh &&
           a.off_cone == b.off_cone && a.off_dmask == b.off_dmask && a.dmask_n == b.dmask_n &&
           a.dmask_bytes == b.dmask_bytes && a.off_gmask == b.off_gmask && a.gmask_words == b.gmask_words &&
           a.n_spheres == b.n_spheres && a.n_boxes == b.n_boxes &&
           a.n_mats == b.n_mats && a.n_lights == b.n_lights;
}

int render_batch_impl(rt_context *ctx, const rt_scene *const *scenes, const rt_view *views, int n_views, int width,
                      int height, int max_depth, int block_rows, int n_shards, int shard, float *out_device,
                      void *hip_stream) {
    const rt_scene *scene = scenes[0];
    int rc = check_render_args(ctx, scene, width, height, max_depth);
    if (rc != RT_OK) return rc;
    if (!views || n_views <= 0 || n_views > RT_MAX_BATCH || !out_device) {
        set_error("rt_render_batch: need 1.." + std::to_string(RT_MAX_BATCH) + " views and a device output");
        return RT_ERR_INVALID;
    }
    const bool sharded = n_shards > 1;
    const int rows = sharded ? rt_shard_rows(height, block_rows, n_shards, shard) : height;
    if (rows < 0 || (n_shards > 1 && block_rows <= 0)) {
        set_error("rt_render_batch: bad shard arguments");
        return RT_ERR_INVALID;
    }
    if (rows == 0) return RT_OK;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    LaunchParams p = base_params(ctx, scene, views, n_views, width, height);
    for (int k = 1; k < n_views; ++k) {
        if (scenes[k] == scene) continue;
        if (!scenes[k] || scenes[k]->device != ctx->device || !same_layout(scenes[k]->dev, scene->dev)) {
            set_error("rt_render_batch_scenes: scene " + std::to_string(k) +
                      " is missing, on another device or laid out differently from scene 0");
            return RT_ERR_INVALID;
        }
        p.view[k].blob = scenes[k]->dev.blob;
    }
    if (ctx->host_consts) {  // each view's constants from its own scene
        const float4 *blobs[kMaxViews];
        for (int k = 0; k < n_views; ++k) blobs[k] = scenes[k]->host.empty() ? nullptr : scenes[k]->host.data();
        host_frame_setup(p, blobs);
    }
    p.row_begin = 0;
    p.n_rows = rows;
    if (sharded) {
        p.block_rows = block_rows;
        p.n_shards = n_shards;
        p.shard = shard;
    }
    p.out = reinterpret_cast<float4 *>(out_device);
    hipStream_t stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    rc = launch(ctx, p, max_depth, stream);
    if (rc != RT_OK) return rc;
    if (!hip_stream) {
        e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail("render", e);
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_batch(rt_context *ctx, const rt_scene *scene, const rt_view *views, int n_views, int width,
                    int height, int max_depth, int block_rows, int n_shards, int shard, float *out_device,
                    void *hip_stream) {
    const rt_scene *scenes[RT_MAX_BATCH];
    for (int k = 0; k < RT_MAX_BATCH; ++k) scenes[k] = scene;
    return render_batch_impl(ctx, scenes, views, n_views, width, height, max_depth, block_rows, n_shards, shard,
                             out_device, hip_stream);
}

int rt_render_batch_scenes(rt_context *ctx, const rt_scene *const *scenes, const rt_view *views, int n_views,
                           int width, int height, int max_depth, int block_rows, int n_shards, int shard,
                           float *out_device, void *hip_stream) {
    if (!scenes || !scenes[0]) {
        set_error("rt_render_batch_scenes: null scenes");
        return RT_ERR_INVALID;
    }
    return render_batch_impl(ctx, scenes, views, n_views, width, height, max_depth, block_rows, n_shards, shard,
                             out_device, hip_stream);
}

int rt_render_accumulate(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width, int height,
                         int max_depth, int spp, int sample_offset, uint32_t seed, int jitter, int row_begin,
                         int row_end, float *accum_device, void *hip_stream) {
    int rc = check_render_args(ctx, scene, width, height, max_depth);
    if (rc != RT_OK) return rc;
    if (!view || !accum_device || spp <= 0 || sample_offset < 0 || row_begin < 0 || row_end > height ||
        row_begin >= row_end) {
        set_error("rt_render_accumulate: bad view / accumulator / spp / row range");
        return RT_ERR_INVALID;
    }
    if (ctx->output != RT_OUTPUT_RGBA32F) {
        set_error("rt_render_accumulate: the accumulator is float (RT_OPT_OUTPUT must be RT_OUTPUT_RGBA32F)");
        return RT_ERR_UNSUPPORTED;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    LaunchParams p = base_params(ctx, scene, view, 1, width, height);
    p.row_begin = row_begin;
    p.n_rows = row_end - row_begin;
    p.spp = spp;
    p.sample0 = sample_offset;
    p.seed = seed;
    p.jitter = jitter ? 1 : 0;
    p.out = reinterpret_cast<float4 *>(accum_device);
    hipStream_t stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->stream;
    rc = launch(ctx, p, max_depth, stream);
    if (rc != RT_OK) return rc;
    if (!hip_stream) {
        e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail("render", e);
    }
    return RT_OK;
}

int rt_context_set(rt_context *ctx, int option, int value) {
    if (!ctx) { set_error("rt_context_set: null context"); return RT_ERR_INVALID; }
    switch (option) {
        case RT_OPT_CULLING: ctx->culling = value ? 1 : 0; return RT_OK;
        case RT_OPT_TIMING: ctx->timing = value ? 1 : 0; return RT_OK;
        case RT_OPT_FRAME_CONSTS: ctx->host_consts = value ? 1 : 0; return RT_OK;
        case RT_OPT_OUTPUT:
            if (value != RT_OUTPUT_RGBA32F && value != RT_OUTPUT_RGBA8 && value != RT_OUTPUT_RGB32F) {
                set_error("rt_context_set: unknown output format " + std::to_string(value));
                return RT_ERR_INVALID;
            }
            ctx->output = value;
            return RT_OK;
        default: set_error("rt_context_set: unknown option " + std::to_string(option)); return RT_ERR_INVALID;
    }
}

int rt_last_kernel_ms(rt_context *ctx, float *ms) {
    if (!ctx || !ms || !ctx->timed) {
        set_error("rt_last_kernel_ms: nothing timed yet");
        return RT_ERR_INVALID;
    }
    hipError_t e = hipEventSynchronize(ctx->ev1);
    if (e != hipSuccess) return hip_fail("hipEventSynchronize", e);
    e = hipEventElapsedTime(ms, ctx->ev0, ctx->ev1);
    if (e != hipSuccess) return hip_fail("hipEventElapsedTime", e);
    return RT_OK;
}

// GL_RGBA8 unorm store of a float colour (main.cpp:152-159, :223): clamp to
// [0, 1] and round to nearest (alpha stored as written, 0, :404).
int rt_pack_rgba8(const float *in, size_t n_pixels, uint8_t *out) {
    if ((!in || !out) && n_pixels) {
        set_error("rt_pack_rgba8: null buffer");
        return RT_ERR_INVALID;
    }
    for (size_t i = 0; i < n_pixels * 4; ++i) {
        float v = in[i];
        v = v != v ? 0.0f : std::min(std::max(v, 0.0f), 1.0f);
        out[i] = static_cast<uint8_t>(v * 255.0f + 0.5f);
    }
    return RT_OK;
}

}  // extern "C"
