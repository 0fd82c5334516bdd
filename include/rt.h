/*
 * rt.h — C-ABI of the MI355X per-pixel ray tracer (libopenglraytracer_amd.so).
 *
 * Drop-in for the reference's frame-driver -> compute-shader boundary:
 *
 *   reference (OpenGLRaytracer/main.cpp)          this ABI
 *   ------------------------------------------    ------------------------------
 *   :203 createShaderProgram("raytrace_compute")  rt_create()           (once)
 *   :129-159 RGBA8 W x H texture (host-owned)     caller-owned float4 buffer
 *   raytrace_compute.glsl:74-321 scene consts     rt_scene_create()     (per scene/time)
 *   :213 get_current_time(), :226 uniform time    `time` argument
 *   :223 glBindImageTexture + :235 glDispatch     rt_render()
 *   :238 glFinish                                 rt_render() with stream == NULL
 *
 * All structs are plain C, float32, no padding surprises (4-byte members
 * only). Every entry point returns RT_OK (0) or a negative RT_ERR_* code and
 * never throws across the boundary; rt_last_error() returns a thread-local
 * message for the last failure on the calling thread.
 *
 * Output layout (identical to the reference image, raytrace_compute.glsl:404):
 * row-major, row 0 = y 0 (GL's bottom row), pixel (x, y) at index y*W + x,
 * 4 floats (r, g, b, 0) per pixel, unclamped (the shipped RGBA8 surface
 * clamps; rt_pack_rgba8 reproduces that).
 */
#ifndef OPENGLRAYTRACER_AMD_RT_H
#define OPENGLRAYTRACER_AMD_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_ERR_INVALID (-1)     /* bad argument */
#define RT_ERR_HIP (-2)         /* HIP runtime error */
#define RT_ERR_NOMEM (-3)       /* allocation failed */
#define RT_ERR_UNSUPPORTED (-4) /* e.g. max_depth above RT_MAX_DEPTH */
#define RT_ERR_NO_DEVICE (-5)   /* no GPU / bad device index */

/* Deepest recursion compiled into the kernel. The reference's stack machine
 * (raytrace_compute.glsl:873-874,1077-1101) holds 100 elements and gives up
 * after 10000 steps; with at most 2^(D+1)-1 traced rays of 6 steps each the
 * step guard cannot trigger for D <= 9, so results are exact up to here. */
#define RT_MAX_DEPTH 9

/* raytrace_compute.glsl:56-69 Material */
typedef struct rt_material {
    float ambient[4];
    float diffuse[4];
    float specular[4];
    float shininess;
    float emissive[4];
    float reflectivity;
    float transparency;
    float refraction_index;
} rt_material;

/* raytrace_compute.glsl:244-258 Object (Box :166-170, Sphere :172-175).
 * Type test exactly as get_closest_collision (:749-771): a box when
 * box_mins/box_maxs are not both (0,0,0) (null_box, :178); otherwise a sphere
 * when radius != -1 (null_sphere, :179); otherwise skipped. */
typedef struct rt_object {
    float box_mins[3];
    float box_maxs[3];
    float radius;
    float position[3];
    float angles[3]; /* pitch, yaw, roll in degrees (:254) */
    int32_t material; /* index into the scene's material table */
} rt_object;

/* raytrace_compute.glsl:190-196 Light (point light, Phong terms) */
typedef struct rt_light {
    float position[3];
    float ambient[4];
    float diffuse[4];
    float specular[4];
} rt_light;

/* raytrace_compute.glsl:36-50 Camera */
typedef struct rt_camera {
    float position[3];
    float angles[3]; /* pitch, yaw, roll in degrees */
    float v_fov;     /* degrees */
    float aspect;    /* the reference fixes 16/9 whatever W/H is (:363) */
    float near_plane;
    float far_plane;
} rt_camera;

/* The per-frame camera constants the kernel consumes: the column-major
 * inverse(proj * view) that unprojects NDC (:383) and the ray origin, the
 * camera position (:391). rt_make_view(NULL, time) — the reference's orbit
 * camera, and what rt_render(cam = NULL) uses — evaluates them in float32
 * exactly as the reference's GL (llvmpipe) does (rt_camera.cpp; bit-exact vs
 * tests/golden/camera_llvmpipe.npz); an explicit rt_camera, which the
 * reference does not have, is evaluated in float64 and rounded once to
 * float32. Callers may also supply their own (e.g. a value another renderer
 * computed). */
typedef struct rt_view {
    float unprojection[16];
    float origin[3];
} rt_view;

typedef struct rt_context rt_context; /* one per device; not thread-safe */
typedef struct rt_scene rt_scene;     /* device-resident, precomputed scene */

/* ---- reference scene / camera (host functions, no GPU) --------------- */

/* The 7 materials of raytrace_compute.glsl:74-157, in this order:
 * material1, material2, red_glass, green_glass, blue_glass, mirror, wall. */
#define RT_MAT_MATERIAL1 0
#define RT_MAT_MATERIAL2 1
#define RT_MAT_RED_GLASS 2
#define RT_MAT_GREEN_GLASS 3
#define RT_MAT_BLUE_GLASS 4
#define RT_MAT_MIRROR 5
#define RT_MAT_WALL 6
#define RT_REFERENCE_MATERIALS 7
#define RT_REFERENCE_LIGHTS 3
#define RT_REFERENCE_OBJECTS 5

int rt_reference_materials(rt_material out[RT_REFERENCE_MATERIALS]);
/* raytrace_compute.glsl:199-224 */
int rt_reference_lights(rt_light out[RT_REFERENCE_LIGHTS]);
/* raytrace_compute.glsl:236-237,261-321: the shipped, time-animated scene. */
int rt_reference_objects(float time, rt_object out[RT_REFERENCE_OBJECTS]);
/* raytrace_compute.glsl:334-364: the orbiting camera at `time`. */
int rt_reference_camera(float time, rt_camera *out);
/* Benchmark scenes: object 0 is the reference room box
 * (+-11, wall material); then n_spheres seeded spheres (splitmix64 stream,
 * centre U([-8,8]x[-8,8]x[-4,4]), radius U(0.3,1.2), materials cycling
 * material1, material2, red_glass, green_glass, blue_glass, mirror).
 * `out` holds n_spheres + 1 objects. */
int rt_bench_objects(int n_spheres, uint64_t seed, rt_object *out);

/* cam == NULL: the reference orbit camera at `time`. */
int rt_make_view(const rt_camera *cam, float time, rt_view *out);

/* The transforms a box object is intersected with, as the reference's GL
 * evaluates them per ray (raytrace_compute.glsl:650-652, :718, replacing
 * calc_transform_matrix / inverse / transpose(inverse(mat3(.)))):
 * local_to_world and world_to_local (column-major 4x4, m[col][row] at
 * col * 4 + row) and the normal matrix (column-major 3x3). The scene builder
 * stores exactly these; exposed for tests and tools. */
int rt_object_transforms(const rt_object *obj, float l2w[16], float w2l[16], float nrm[9]);

/* Scene description input: the content the reference
 * compiles into its shader (materials :74-157, lights :199-224, the animated
 * objects :261-321 at `time`, the camera :334-364) read from JSON text —
 * format in openglraytracer_amd/csrc/rt_scene_json.cpp. Fills the caller's
 * arrays (capacities max_*; n_* = entries written); *has_camera = 1 when the
 * text sets a camera (written to *cam, which may be NULL), else 0 (use the
 * reference orbit camera). Host only; RT_ERR_INVALID with a message naming
 * the problem (and the byte offset of a syntax error). */
int rt_scene_desc_parse(const char *json, float time, rt_object *objs, int max_objs, int *n_objs,
                        rt_material *mats, int max_mats, int *n_mats, rt_light *lights, int max_lights,
                        int *n_lights, rt_camera *cam, int *has_camera);

/* ---- device API ------------------------------------------------------ */
int rt_create(int device, rt_context **out);
void rt_destroy(rt_context *ctx);

/* Copies and precomputes (transforms, inverse transforms, normal matrices)
 * the scene and uploads it to the context's device. Arrays are host memory
 * and may be freed after the call. n_objs <= RT_MAX_OBJECTS.
 * Host cost (make -C openglraytracer_amd/csrc scene-build-time, 8 host
 * threads): about 2-5 ms up to 256 spheres. A scene of 33-256 spheres also
 * gets origin-sphere candidate lists for depth >= 2 renders (RT_OPT_ORIGIN_
 * LISTS; 12.6 MB and about 30 ms at 256 spheres): they are built and
 * appended to the device copy by the first render that reads them, never by
 * create or update, and are not kept on the host.
 * Stream order: create, update and destroy run on the context's stream, a
 * blocking HIP stream (see rt_render): their uploads and stream-ordered
 * frees are ordered after work queued earlier on the device's null stream
 * (torch's default stream), and null-stream work queued later waits for
 * them; create and update return only after their upload is complete. */
#define RT_MAX_OBJECTS 1024
#define RT_MAX_LIGHTS 16
#define RT_MAX_MATERIALS 256
int rt_scene_create(rt_context *ctx, const rt_object *objs, int n_objs, const rt_material *mats,
                    int n_mats, const rt_light *lights, int n_lights, rt_scene **out);
/* Frees the scene's device memory in stream order behind every render that
 * reads it — on the context's stream and on any caller stream (an event per
 * stream is recorded at each render, for up to 8 distinct caller streams);
 * no device-wide synchronisation, except when the scene was rendered on more
 * than 8 distinct caller streams (or an event wait fails): then it waits for
 * the whole device before freeing. rt_scene_update waits the same way. */
void rt_scene_destroy(rt_scene *scene);
/* Replace the scene's contents in place (an animated frame: the reference
 * recomputes its objects from `time` every frame, raytrace_compute.glsl:
 * 277-307); reallocates only if the new scene is larger. Waits (on the host)
 * for the renders queued that read the scene, on any stream. The per-frame
 * host cost is rt_scene_create's build (about 2-5 ms up to 256 spheres, tens
 * of microseconds for the shipped scene) plus the upload; a deep render of
 * the new contents rebuilds the origin-sphere lists once. */
int rt_scene_update(rt_context *ctx, rt_scene *scene, const rt_object *objs, int n_objs, const rt_material *mats,
                    int n_mats, const rt_light *lights, int n_lights);

/* Render rows [row_begin, row_end) of a width x height frame.
 *  cam        NULL = the reference orbit camera at `time` (main(), :334-364).
 *  out        (row_end-row_begin)*width*4 floats; device memory of this
 *             context's GPU if out_is_device, else host memory.
 *  hip_stream hipStream_t; NULL = the context's own stream and the call
 *             returns after the frame is complete (the reference's glFinish,
 *             main.cpp:238). That stream is a blocking HIP stream: the
 *             render starts after all work queued earlier on the device's
 *             null stream (torch's default stream, e.g. a fill of `out`), as
 *             glDispatchCompute follows the earlier commands of its context
 *             (main.cpp:220-238). A non-NULL stream makes the call
 *             asynchronous and ordered only on that stream (out_is_device
 *             must then be 1). Every render entry point below treats
 *             hip_stream the same way.
 * No allocation happens here after the first call at a given size. */
int rt_render(rt_context *ctx, const rt_scene *scene, const rt_camera *cam, float time, int width,
              int height, int max_depth, int row_begin, int row_end, float *out, int out_is_device,
              void *hip_stream);

/* Same, with explicit frame constants. */
int rt_render_view(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width, int height,
                   int max_depth, int row_begin, int row_end, float *out, int out_is_device,
                   void *hip_stream);

/* Row-block interleaved shard for multi-GPU frames: renders the rows r of the
 * frame with (r / block_rows) % n_shards == shard, in increasing order, packed
 * densely into out_device (rt_shard_rows() rows of width*4 floats). */
int rt_shard_rows(int height, int block_rows, int n_shards, int shard);
int rt_render_shard(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width,
                    int height, int max_depth, int block_rows, int n_shards, int shard,
                    float *out_device, void *hip_stream);

/* Several frames in one launch (the reference's frame loop, main.cpp:81-86,
 * batched): views[k] renders into out_device + k * rows * width * 4 floats,
 * where rows = height, or rt_shard_rows(...) when n_shards > 1 (each frame
 * then gets this shard's interleaved row blocks). The scene is shared. Up to
 * 8 views travel in the kernel arguments; 9..RT_MAX_BATCH views of a
 * max_depth 0 or 1 frame go through a device buffer of the context (one
 * launch). Deeper frames run as even launches of as many views as one
 * launch holds beside the scene in GPU local memory (1..8, by the scene's
 * size: 7 for 64 spheres, 1 for 256). */
#define RT_MAX_BATCH 256
/* The number of kernel launches rt_render_batch makes for n_views views of
 * this scene at max_depth (1 up to RT_MAX_BATCH views at depth 0-1; deep
 * batches: ceil(n_views / views per queued launch)), or a negative RT_ERR_*.
 * No GPU work; for callers that time or size per launch. */
int rt_batch_launches(rt_context *ctx, const rt_scene *scene, int n_views, int max_depth);
int rt_render_batch(rt_context *ctx, const rt_scene *scene, const rt_view *views, int n_views, int width,
                    int height, int max_depth, int block_rows, int n_shards, int shard, float *out_device,
                    void *hip_stream);

/* Animated frames in one launch (the reference's frame loop, main.cpp:81-86,
 * where the shipped scene moves with `time`, raytrace_compute.glsl:277-307):
 * as rt_render_batch, but views[k] renders scenes[k]. Every scene must have
 * scene 0's layout — the same object kinds in the same order and the same
 * material and light counts (e.g. rt_reference_objects at successive times,
 * each built with rt_scene_create). */
int rt_render_batch_scenes(rt_context *ctx, const rt_scene *const *scenes, const rt_view *views, int n_views,
                           int width, int height, int max_depth, int block_rows, int n_shards, int shard,
                           float *out_device, void *hip_stream);

/* Monte-Carlo extension (the reference has one
 * ray per pixel): adds, for every pixel of rows [row_begin, row_end), the sum
 * of samples [sample_offset, sample_offset + spp) — in sample order — to
 * accum_device (float4 per pixel, caller-zeroed, device memory). Sample s of
 * pixel (x, y) is the reference ray through NDC ((x - W/2 + jx) / (W/2),
 * (y - H/2 + jy) / (H/2)) with (jx, jy) in [0, 1)^2 from a counter-based hash
 * of (seed, s, y*W + x) when jitter != 0, else (0, 0) (then every sample
 * equals the reference frame). With hip_stream NULL a zero fill queued on
 * the null stream (torch's default stream) is complete before the
 * accumulation reads the buffer. The mean is accum / total samples. Disjoint
 * sample ranges on several GPUs sum (RCCL all-reduce) to the same estimate
 * up to float re-association. */
int rt_render_accumulate(rt_context *ctx, const rt_scene *scene, const rt_view *view, int width, int height,
                         int max_depth, int spp, int sample_offset, uint32_t seed, int jitter, int row_begin,
                         int row_end, float *accum_device, void *hip_stream);

/* ---- one frame on several GPUs of this process ----
 * The reference renders a frame with one glDispatchCompute(W, H, 1) +
 * glFinish (OpenGLRaytracer/main.cpp:228-238). A multi-GPU group deals the
 * frame's rows in interleaved blocks of block_rows rows to its GPUs (the
 * rt_shard_rows / rt_render_shard layout), every GPU renders its blocks on
 * its context's stream, one gather brings the shards to the first context's
 * GPU (the root) — RCCL point-to-point over xGMI (ncclCommInitAll over the
 * contexts' devices; one context per device) or peer copies — and the root
 * de-interleaves them into the frame. The result is bit-identical to
 * rt_render of the whole frame on one GPU. */
typedef struct rt_multi rt_multi;
#define RT_MULTI_RCCL 0 /* RCCL grouped ncclSend / ncclRecv to the root */
#define RT_MULTI_COPY 1 /* hipMemcpyPeerAsync; also serves contexts that share a device */
/* ctxs[0..n_gpus) stay owned by the caller and must outlive the group. */
int rt_multi_create(int n_gpus, rt_context *const *ctxs, int transport, rt_multi **out);
void rt_multi_destroy(rt_multi *m);
/* scenes[i]: the frame's scene on ctxs[i]'s device (the same content on
 * every device). out: the whole frame in the root context's surface format
 * (RT_OPT_OUTPUT, the same on every context), device memory of the root's
 * GPU if out_is_device, else host memory. Synchronous, like glFinish. */
int rt_render_multi(rt_multi *m, const rt_scene *const *scenes, const rt_camera *cam, float time, int width,
                    int height, int max_depth, int block_rows, float *out, int out_is_device);
int rt_render_multi_view(rt_multi *m, const rt_scene *const *scenes, const rt_view *view, int width, int height,
                         int max_depth, int block_rows, float *out, int out_is_device);
/* Times of the last rt_render_multi: kernel_ms[i] per GPU (-1 when its
 * context's RT_OPT_TIMING is off or it had no rows), the gather (from the
 * moment every shard is complete) and the de-interleave on the root. */
int rt_multi_last_ms(rt_multi *m, float *kernel_ms, float *gather_ms, float *assemble_ms);

/* Context options. RT_OPT_CULLING (default 1): skip spheres that provably
 * cannot be hit (conservative footprints / light cones with margins far
 * above float error) — output is bit-identical either way. */
#define RT_OPT_CULLING 1
/* RT_OPT_TIMING (default 1): record HIP events around every launch for
 * rt_last_kernel_ms. Each event is a marker on the stream; 0 leaves the
 * stream with the kernels alone (back-to-back launches, e.g. a benchmark
 * timing many frames with one event pair of its own). */
#define RT_OPT_TIMING 2
/* RT_OPT_OUTPUT (default RT_OUTPUT_RGBA32F): the surface format renders
 * write. RT_OUTPUT_RGBA8 is the shipped app's GL_RGBA8 texture
 * (OpenGLRaytracer/main.cpp:152-159, :223; raytrace_compute.glsl:404): the
 * kernel packs each pixel in its epilogue — clamp to [0, 1], unorm rounding,
 * exactly rt_pack_rgba8 of the float frame — and stores 4 bytes per pixel, so
 * every `out` buffer then holds width*rows*4 bytes (uint8 r, g, b, a).
 * RT_OUTPUT_RGB32F drops the alpha channel, which is always 0.0 (:404): 3
 * floats per pixel (width*rows*12 bytes), the compact transport form of a
 * float frame (the multi-GPU frame exchange ships 3/4 of the bytes).
 * rt_render_accumulate keeps float4 sums and refuses the other formats. */
#define RT_OPT_OUTPUT 3
#define RT_OUTPUT_RGBA32F 0
#define RT_OUTPUT_RGBA8 1
#define RT_OUTPUT_RGB32F 2
/* RT_OPT_FRAME_CONSTS (default 1): a launch's per-frame constants (every
 * sphere's and box's camera-origin terms and every sphere's pixel footprint,
 * per view) are computed on the host and carried in the kernel arguments when
 * all views' records fit (272 records, at most 256 per view: e.g. 8 views of
 * 16 spheres + 1 box);
 * 0: every work-group derives them on the device. Output is identical. */
#define RT_OPT_FRAME_CONSTS 4
/* RT_OPT_ORIGIN_LISTS (default 1): a secondary ray that starts on a sphere
 * of a scene of 33-256 spheres tests the candidates its direction selects in
 * that sphere's precomputed list instead of walking the sphere BVH
 * (depth >= 2); 0: every secondary ray walks the BVH. Output is identical. */
#define RT_OPT_ORIGIN_LISTS 7
/* RT_OPT_SCENE_SHAPES (default 1): a render whose scene has one of the
 * common shapes runs a kernel compiled for that shape, the way the
 * reference's shader is compiled for its own scene: at depth 0, shadow
 * queries that walk LDS direction masks (at most 64 spheres, 12-texel masks,
 * culling on; the mask width as a constant); at depth >= 2 without
 * Monte-Carlo, wide masks with their candidate lists and origin-sphere lists
 * (33-256 spheres, culling on); either with or without the room (exactly one
 * translate-only box holding every live light). 0: every render runs the
 * general kernel. Output is identical. */
#define RT_OPT_SCENE_SHAPES 8
/* (option 6, a tolerance tier that summed the recursion's colours forward
 * instead of mixing them on the way back up, measured even with the exact
 * walk and was removed: DESIGN.md §3.) */
/* (option 5, a level-by-level wavefront path for deep trees, was measured
 * 2x slower than the depth-first walk and removed: DESIGN.md §3.) */
int rt_context_set(rt_context *ctx, int option, int value);

/* Kernel-only timing of the last render call (ms, from HIP events around the
 * launch on its stream — around all of its launches when a deep batch is
 * split into several); needs RT_OPT_TIMING. */
int rt_last_kernel_ms(rt_context *ctx, float *ms);

/* RGBA8 unorm packing of a float frame as the shipped GL_RGBA8 surface stores
 * it (NaN -> 0, clamp to [0,1], v * 255 rounded to nearest even, as the
 * reference's GL converts; pinned by tests/golden/rgba8_llvmpipe.npz). Host
 * memory, n pixels. */
int rt_pack_rgba8(const float *rgba32f, size_t n_pixels, uint8_t *out_rgba8);

/* Headless image dump (replaces the display pass, draw_screen_*.glsl and
 * main.cpp:240-260). `rgba32f` is a frame in this ABI's layout (row 0 = GL's
 * bottom row). PPM: binary P6, 8-bit, RGBA8 unorm rounding (rt_pack_rgba8),
 * rows written top-down (the on-screen orientation). PFM: float RGB, rows
 * bottom-up as the PFM format stores them, little-endian. */
int rt_write_ppm(const char *path, const float *rgba32f, int width, int height);
int rt_write_pfm(const char *path, const float *rgba32f, int width, int height);

const char *rt_last_error(void);
const char *rt_version(void);

#ifdef __cplusplus
}
#endif
#endif
