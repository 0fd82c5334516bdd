// rt_internal.h — shared declarations of the product library (host side).
//
// Layout of the device-resident scene (one hipMalloc'd blob per rt_scene, see
// rt_scene.cpp) and the per-launch parameter block consumed by the kernel in
// rt_kernel.hip. Everything is float32 / int32; offsets are in 16-byte units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt.h"

namespace rtamd {

// One sphere of the closest-hit loop: centre and radius*radius (the float
// product raytrace_compute.glsl:588 forms), 16 B.
struct SphereRec {
    float cx, cy, cz, rr;
};
// Identity of a sphere: its index in the reference object order (tie-break
// of get_closest_collision, :773) and its material.
struct SphereMeta {
    int32_t obj_index;
    int32_t material;
    float radius;  // |radius|, for the culling bounds (intersection uses rr)
    int32_t pad;
};

// One oriented box (:647-724) with its frame constants precomputed once per
// scene: world_to_local (:652), local_to_world (:650) and the normal matrix
// transpose(inverse(mat3(L))) (:718). Matrices are row-major 3x4 (the x/y/z
// rows of the GLSL mat4; the w row of an affine transform is (0,0,0,1)).
struct BoxRec {
    float w2l[12];
    float l2w[12];
    float nrm[9];
    float mins[3];
    float maxs[3];
    int32_t obj_index;
    int32_t material;
    uint32_t light_inside;  // bit j: light j strictly inside the box with margin (shadow shortcut)
    int32_t translate_only;  // w2l's 3x3 block is exactly the identity (world->local = + w2l[3,7,11])
    float w2l_w0[3];  // w2l[r][3] * 0.0f: the w column's term of (w2l * vec4(d, 0.0)) per row (+-0 or NaN)
    int32_t pad[2];
};  // 48 words = 192 B
static_assert(sizeof(BoxRec) == 192, "BoxRec layout");

// Material (:56-69) plus the per-material light products the shading loop
// would otherwise recompute: amb_sum = sum_j La_j * Ma (:801, same order),
// and for each light j: Ld_j * Md (:830), Ls_j * Ms (:832).
struct MatRec {
    float amb_sum[4];
    float emissive[4];
    float shininess, reflectivity, transparency, refraction_index;
    float eta_in, eta_out;  // 1.0 / refraction_index and 1.0 / that (:1013-1016), each correctly rounded
    float pad[2];
};  // 64 B
// The flags decide whether a light's direct term can change the Phong sums;
// the shadow ray is cast only then (lit and shadowed agree otherwise):
// d_nz / s_nz: some component of Ld*Md / Ls*Ms is nonzero; always: the
// material is not "tame" (a product is not finite, or the shininess is not a
// positive finite number), so the diffuse / specular factors may be NaN or
// infinite and every light's term is taken as changing the sums.
struct LightMatRec {
    float ld_md[4];
    float ls_ms[4];
    int32_t d_nz, s_nz, always, pad;
};  // 48 B
// Shadow-ray culling cone of sphere s seen from light j (host, float64):
// v = unit direction light -> centre; far = d - rp where d = |centre - light|
// and rp = |radius| + 0.021 + 1e-3 d (the 0.01 start offset plus margins);
// sin / cos of the half-angle asin(rp / d); near = 1 when d <= rp (the light
// is inside the inflated sphere: always a candidate).
struct ShadowCone {
    float v[3];
    float far;
    float sph, cph, near, pad;
};  // 32 B
constexpr size_t kConeLdsBudget = 24 * 1024;
// Shadow-ray direction masks (scenes of at most 64 spheres): for every light
// that casts shadow rays (not `dead`), a cube map of 6 x n x n texels around
// the light; texel bit s is set when some direction of the texel lies within
// sphere s's inflated cone from the light (the ShadowCone geometry, float64,
// plus the texel's own angular radius and a margin). A shadow ray whose
// direction from the light falls in the texel can only be blocked by the
// spheres of its mask. Face f = 2 * axis + (component < 0); within the face
// the two other axes in increasing order give (column, row). Kept while the
// work-group's LDS stays within kMaskLdsBudget (full occupancy); masks are
// 16, 32 or 64 bits wide (scenes of at most 16, 32, 64 spheres).
constexpr int kMaskMaxSpheres = 64;
constexpr size_t kMaskLdsBudget = 19 * 1024;
// Larger scenes (up to kGMaskMaxSpheres) use the same masks as 64-bit words
// per texel, kGMaskTexels per face edge, in the device blob after the part
// the work-groups stage (read through L2: 256 spheres, 768 KB per live light at 64 texels).
constexpr int kGMaskMaxSpheres = 256;
#ifndef RT_GMASK_TEXELS
#define RT_GMASK_TEXELS 64  // tuning knob (tools/ablate.sh flags); 8/16/24/32/48/64: config 4 28.2/25.9/25.2/25.0/24.9/24.8 ms
                            // (r01); after the ordered BVH 32/48/64: 18.29/17.91/17.73 ms, config 3 1.002/1.005/0.996 ms
#endif
constexpr int kGMaskTexels = RT_GMASK_TEXELS;
// The same wide masks as short candidate lists, one 16-B record per (live
// light, texel): byte 0 = the number of candidate spheres (0..15), bytes
// 1..15 = their slots (< 256), the sphere of the largest angular size from
// the light first (rt_scene.cpp); kGListOverflow in byte 0: more than
// 15 candidates, use the texel's mask words. A query then walks its own list:
// a wave loops max-over-lanes-of-count times, once per candidate, instead of
// once per set bit per mask word (the sum over the words of the per-word
// maxima), from one 16-B load instead of one 8-B load per word.
constexpr int kGListMax = 15;
constexpr uint32_t kGListOverflow = 255u;
static_assert(kGMaskMaxSpheres <= 256, "candidate lists hold sphere slots in bytes");
// Secondary rays that start on a sphere (round 5; tools/model/
// origin_list_model.py: 66-73 % of config 4's secondary rays, 58 % of
// config 3's) look up the spheres they can hit instead of walking the BVH:
// per sphere s, a cube map of kOListTexels x kOListTexels texels per face
// (direction_texel's layout) whose texel lists every sphere j that a ray
// from the ball B(c_s, r_s + 0.001) — every reflection or refraction origin
// on s (:1010-1023) — with its direction in the texel can hit: the cone of
// the texel from c_s meets the ball B(c_j, r_j + r_s + 0.001) (the shadow
// masks' test, float64, with margins), s itself first (a ray inside s
// leaves through it). The candidates follow in increasing order of a lower
// bound of their hit distance, |c_j - c_s| - r_j - r_s - margins, so a lane
// whose closest hit so far (the box's, tested first) lies below the next
// bound can stop. One 32-B record per (sphere, texel):
//   byte 0      the number of candidates (255: 255 or more);
//   bytes 1..25 the first kOListSlots candidates' sphere slots;
//   bytes 26..31 three uint16 bounds in 1/256 units (rounded down, 65535 at
//               most): of candidate 8, of candidate 16, and of candidate
//               kOListSlots (the first one not in the record; 65535 when
//               there is none). A lane checks the first two before testing
//               candidates 8 and 16; one that has tested the whole record
//               and still lies above the third walks the BVH instead.
// Built for scenes of kOListMinSpheres..kGMaskMaxSpheres spheres, read by the
// recursive kernels (depth >= 2) through L2, never staged.
#ifndef RT_OLIST_TEXELS
#define RT_OLIST_TEXELS 16
#endif
constexpr int kOListTexels = RT_OLIST_TEXELS;
constexpr int kOListSlots = 25;
constexpr int kOListRecordBytes = 32;
#ifndef RT_OLIST_FROM
#define RT_OLIST_FROM 33  // (the wide masks' threshold: smaller scenes keep the BVH walk, their blob unchanged)
#endif
constexpr int kOListMinSpheres = RT_OLIST_FROM;
constexpr float kOListBoundUnit = 1.0f / 256.0f;
// Sphere BVH node (depth-first order; the left child is the next node):
// lo = (min xyz, skip) and hi = (max xyz, leaf) where skip is the node after
// this subtree (-1: end) and leaf = (count << 24) | first sphere slot (0 for
// an inner node). Bounds are the spheres' boxes inflated by a margin far
// above float error, so the approximate box test never drops a sphere the
// exact test could hit.
struct BvhNode {
    float lo[3];
    int32_t skip;
    float hi[3];
    int32_t leaf;
};
static_assert(sizeof(BvhNode) == 32, "BvhNode layout");
// Ordered traversal of the closest-hit walk: per node, 8 link words, one per
// ray-direction octant (bit a set: d[a] < 0), each (next node on a hit) |
// (next node on a miss) << 16, 0xFFFF = end. The octant's depth-first order
// enters every inner node's children nearer-first along its split axis, so
// near hits shrink the search interval before the far subtree is tested.
constexpr int kBvhOctants = 8;

struct LightRec {
    float pos[3];
    float dead;  // 1: zero diffuse and specular for every material (no direct term, no shadow ray)
};

// Per-launch parameters (kernarg, read through the scalar cache).
// Per-frame camera constants of one view of a launch.
struct FrameView {
    float unproj[16];  // column-major inverse(proj*view) (:383)
    float proj[16];    // column-major proj*view = inverse(unproj) (float64 on the host), for culling
    float origin[3];   // ray start = camera position (:391)
    int32_t cull;      // 1: exactness-preserving culling enabled (consistent pinhole view)
    const void *blob;  // this view's scene blob (rt_render_batch_scenes); nullptr: LaunchParams::scene
};
constexpr int kMaxViews = 8;  // frames per launch (blockIdx.z) with the views in the kernel arguments
// Larger batches (up to RT_MAX_BATCH views, depth 0-1): the views and their
// frame constants go to a per-context device buffer (one of kBatchSlots,
// reused behind an event), read by render_kernel<D, false, true>.
constexpr int kBatchSlots = 4;
// per-frame constant records carried in the kernel arguments: all views'
// (8 views of 16 spheres + 1 box = 264), at most kMaxViewConsts per view
// (one record per thread of a work-group)
constexpr int kMaxFrameConsts = 272;
constexpr int kMaxViewConsts = 256;
// Largest LDS a work-group may request on gfx950 (160 KiB).
constexpr size_t kMaxLds = 160 * 1024;

struct LaunchParams {
    FrameView view[kMaxViews];
    int32_t n_views;
    int32_t width, height;
    int32_t row_begin, n_rows;          // contiguous band [row_begin, row_begin+n_rows)
    int32_t block_rows, n_shards, shard;  // interleaved shard mapping when n_shards > 0
    int32_t n_spheres, n_boxes, n_mats, n_lights;
    const void *scene;  // device blob
    float4 *out;        // n_views x n_rows x width float4
    int32_t off_spheres, off_smeta, off_boxes, off_mats, off_lights, off_lightmat;  // 16-B units
    int32_t off_bvh, n_bvh;  // sphere BVH nodes (2 x float4 each), 16-B units / count
    int32_t off_blink;       // n_bvh x kBvhOctants uint32 traversal links, 16-B units
    int32_t off_cone;        // n_lights x n_spheres ShadowCone, 16-B units; -1: none
                             // (kept only while the LDS total stays within kConeLdsBudget)
    int32_t off_dmask, dmask_n;  // shadow direction masks (live lights x 6 x n x n), 16-B units; -1: none
    int32_t dmask_bytes;         // bytes per mask: 2, 4 or 8 (at most 16, 32, 64 spheres)
    int32_t off_gmask, gmask_words;  // wide masks in the blob past blob_units (not staged), 16-B units; -1: none
    int32_t off_glist;               // their candidate lists (kGListMax), 16-B units; -1: none
    int32_t blob_units;      // blob size, 16-B units
    // Monte-Carlo accumulation (render_kernel<D, true>): samples
    // [sample0, sample0 + spp) per pixel, jittered inside the pixel when
    // jitter != 0, summed in sample order and added to out.
    int32_t spp, sample0, jitter;
    uint32_t seed;
    // Queued work distribution (rt_kernel.hip, render_kernel): the counters of
    // this launch (kSchedInts zeroed ints, left zeroed by the kernel), and the
    // compute units the resident grid is sized for. nullptr: one work-group
    // per tile.
    int32_t *sched;
    int32_t n_cu;
    int32_t out_format;  // RT_OUTPUT_*: float4, GL_RGBA8 unorm bytes (uchar4) or packed float3 per pixel
    // Each view's per-frame constants ([sphere camera terms][sphere pixel
    // footprints][box camera terms], the LDS image the kernel's frame_setup
    // derives), computed on the host when all views' fit here
    // (host_frame_setup): n_frame_consts records per view, view k's at
    // k * n_frame_consts; 0: every work-group derives them.
    int32_t n_frame_consts;
    // 1: every view's camera-ray perspective divisions take the short form,
    // exact for every pixel (rt_scene.cpp camera_short_divisions)
    int32_t cam_short;
    // Rows [slice_begin, slice_begin + slice_rows) of the launch's local rows
    // (the whole launch when slice_rows = 0).
    int32_t slice_begin, slice_rows;
    // > kMaxViews views (render_kernel<D, false, true>): n_views FrameViews
    // and n_views x n_frame_consts records in device memory; nullptr: the
    // arrays above
    const FrameView *views_dev;
    const float4 *consts_dev;
    float4 frame_consts[kMaxFrameConsts];
    // secondary rays' origin-sphere candidate lists (kOListSlots), 16-B units;
    // -1: none (last: the depth-0/1 kernels, which never read it, keep their
    // argument layout)
    int32_t off_olist;
    // 1: the LDS direction masks carry a bit per box (bit n_spheres + b)
    int32_t dmask_box;
    // per (box, light) a plane that separates the box from the light's end
    // of every shadow segment (rt_scene.cpp), 16-B units; -1: none
    int32_t off_bplane;
    // host only (the kernels never read it): 1 when every view of the launch
    // culls, so the depth-0 kernels may take the scene's shape (scene_shape)
    int32_t shape_cull;
    int32_t scene_room;  // host only: every scene of the launch is a room (DeviceScene::room)
    // 1 (set by launch_kernel for the wide-shape recursive kernels): a view's
    // records in LDS are its footprints and box terms only, not the spheres'
    // camera terms (the primary rays compute them as secondary rays do: the
    // same arithmetic, so the same values) — 16 B less per sphere per view
    int32_t lean_views;
};
// ROCm passes kernel arguments above 4 KiB (an 8 KB argument block checked on
// MI355X); this block stays under 6 KiB.
static_assert(sizeof(LaunchParams) <= 6144, "kernel argument block");
// Scene shapes (render_kernel<D, ..., kShape>): the scene's features that
// decide the path a ray takes, as compile-time constants, so the kernel
// carries none of their run-time tests. Depth 0: the LDS direction masks'
// bytes (2, 4, 8; culling on, so every shadow query walks them). Depth >= 2:
// kShapeWide (culling on; wide masks with their candidate lists and the
// origin-sphere lists present). Either | kShapeRoom (exactly one box, a room:
// translate-only, every live light inside it).
// 0: everything read at run time. Chosen per launch on the host
// (scene_shape), like the reference's shader, compiled for its own scene.
constexpr int kShapeMaskBytes = 15;
constexpr int kShapeMaskTexels = 12;  // the LDS masks' texels per face edge in a depth-0 shape (rt_scene.cpp picks 12 where it fits)
constexpr int kShapeRoom = 16;
constexpr int kShapeWide = 32;
int scene_shape(const LaunchParams &p, int max_depth);
// Lean views (LaunchParams::lean_views): the wide-shape kernels.
constexpr bool kLeanViews(int shape) { return (shape & kShapeWide) != 0; }
// 16-B records of one view's per-frame constants in LDS: the spheres' camera
// terms (not with lean views) and footprints, the boxes' camera terms.
inline int view_units(const LaunchParams &p) { return (p.lean_views ? 1 : 2) * p.n_spheres + p.n_boxes; }
constexpr int kQueues = 32;                            // wave-tile queues of a queued launch
constexpr int kQueueStride = 64;                       // ints: each counter on a 256-B line of its own
constexpr int kSchedInts = 2 * kQueues * kQueueStride; // heads + done counters of one launch
constexpr int kSchedSlots = 64;                        // launches that may be in flight at once

struct DeviceScene {
    void *blob = nullptr;
    int32_t blob_units = 0;
    int32_t off_spheres = 0, off_smeta = 0, off_boxes = 0, off_mats = 0, off_lights = 0, off_lightmat = 0;
    int32_t off_bvh = 0, n_bvh = 0, off_blink = 0, off_cone = 0;
    int32_t off_dmask = -1, dmask_n = 0, dmask_bytes = 4;
    int32_t dmask_box = 0;  // the LDS masks carry a bit per box, bit n_spheres + b (round 6)
    int32_t off_bplane = -1;  // n_boxes x n_lights separating planes (float4), 16-B units; -1: none (round 6)
    int32_t off_gmask = -1, gmask_words = 0, off_glist = -1;
    int32_t off_olist = -1;   // -1 until the lists are built (ensure_origin_lists)
    int32_t olist_eligible = 0;  // kOListMinSpheres..256 spheres: depth >= 2 renders get the lists
    int32_t n_spheres = 0, n_boxes = 0, n_mats = 0, n_lights = 0;
    // 1: the one box is a room: translate-only, every live light strictly
    // inside it (the shadow queries' box shortcut always applies; kShapeRoom)
    int32_t room = 0;
};

// rt_scene.cpp: every view's per-frame constants on the host, bit-identical
// to the kernel's frame_setup for the camera terms (float32, same operation
// order) and conservative pixel footprints; view k's 2 * n_spheres + n_boxes
// records (from its scene's host blob, blobs[k]) go to p.frame_consts at
// k * p.n_frame_consts, p.n_frame_consts = records per view, or 0 when they
// do not all fit.
void host_frame_setup(LaunchParams &p, const float4 *const *blobs);
// One view's records for a device-side batch (render_batch_impl, > kMaxViews
// views): writes 2 * n_spheres + n_boxes records of view V (p: the launch's
// scene parameters) to out; the record count, or 0 if it exceeds
// kMaxViewConsts (then every work-group derives them).
int host_view_consts(const LaunchParams &p, const FrameView &V, const float4 *blob, float4 *out);
// A view's kernel-side constants (unprojection, proj for culling, origin,
// cull flag); false if its perspective divisions may not take the short form.
bool fill_view(const rt_context *ctx, const rt_view &view, int width, int height, FrameView &out);

// rt_camera.cpp: the reference orbit camera as llvmpipe evaluates it
float gl_sin(float a);  // gallivm's polynomial sin / cos (run-time GLSL sin / cos)
float gl_cos(float a);
void reference_orbit(float time, float *speed, float pos[3], float *yaw);
void reference_view_gl(float time, float unproj[16], float view[16]);
// a box object's local_to_world, world_to_local and normal matrix as
// llvmpipe evaluates intersect_box_object (column-major)
void reference_box_transforms(const float pos[3], const float ang[3], float l2w[16], float w2l[16], float nrm[9]);

// rt_kernel.hip. Clears p.sched when the launch does not use the queued
// distribution (so the caller knows whether the counter slot is in use).
hipError_t launch_render(LaunchParams &p, int max_depth, hipStream_t stream);
size_t lds_bytes(const LaunchParams &p);
// Views of one scene a queued launch at this depth holds (deep frames: every
// view's per-frame constants beside the scene in LDS at the one-view
// launch's occupancy), 1..kMaxViews; 1 below the queued depths.
int queued_views(const LaunchParams &p, int max_depth);
// Self-test of the kernel argument block on the context's stream (rt_create).
int check_kernarg_block(hipStream_t stream);

// rt_api.cpp
void set_error(const std::string &msg);
int hip_fail(const char *what, hipError_t e);  // sets the message, returns RT_ERR_HIP
// The event a render call records after its launch on a caller stream, shared
// by every scene the call reads (a batch of 256 animated frames with a scene
// each records one event, not 256: round 6, the shipped workload's host gap
// of 1.2 ms per launch) and destroyed with its last user (a pending event is
// released once complete).
struct UseEvent {
    hipEvent_t ev = nullptr;
    UseEvent() = default;
    UseEvent(const UseEvent &) = delete;
    UseEvent &operator=(const UseEvent &) = delete;
    ~UseEvent() {
        if (ev) (void)hipEventDestroy(ev);
    }
};
int check_render_args(const rt_context *ctx, const rt_scene *scene, int width, int height, int max_depth);
// launch parameters of n_views views of `scene` on `ctx` (output and rows left to the caller)
LaunchParams base_params(const rt_context *ctx, const rt_scene *scene, const rt_view *views, int n_views,
                         int width, int height);
// launch on `stream` with the context's queue slot and kernel-time events
int launch(rt_context *ctx, LaunchParams &p, int max_depth, hipStream_t stream);
// Before a render at max_depth: a scene that reads origin-sphere lists at
// this depth (max_depth >= 2, RT_OPT_ORIGIN_LISTS on, 33-256 spheres) gets
// them built and appended to its device blob the first time (the region past
// the blob the earlier renders read; a larger blob is reallocated and the old
// one freed behind its renders). One host build + synchronous upload per
// scene contents; RT_OK at once when nothing is needed.
int ensure_origin_lists(rt_context *ctx, const rt_scene *scene, int max_depth);
// a render on `stream` reads `scene`'s blob: remember it (an event on that
// stream) so that rt_scene_destroy / rt_scene_update wait for it
// `shared`: the render call's event (created and recorded after its launch
// by the first scene noted, then reused for the call's other scenes); nullptr:
// an event of this call alone
int note_scene_use(const rt_scene *scene, hipStream_t stream, std::shared_ptr<UseEvent> *shared = nullptr);
// bytes per pixel of a surface format (RT_OUTPUT_*)
inline size_t surface_bytes(int fmt) { return fmt == RT_OUTPUT_RGBA8 ? 4 : (fmt == RT_OUTPUT_RGB32F ? 12 : 16); }

}  // namespace rtamd

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float4 *staging = nullptr;  // device buffer for host-destination renders
    size_t staging_px = 0;
    bool timed = false;
    int culling = 1;  // RT_OPT_CULLING
    int timing = 1;   // RT_OPT_TIMING
    int output = RT_OUTPUT_RGBA32F;  // RT_OPT_OUTPUT
    int host_consts = 1;  // RT_OPT_FRAME_CONSTS
    int origin_lists = 1;  // RT_OPT_ORIGIN_LISTS
    int scene_shapes = 1;  // RT_OPT_SCENE_SHAPES
    // device-side view batches (> kMaxViews views): per slot a device buffer,
    // its pinned host staging and an event after the last launch that read it
    void *batch_dev[rtamd::kBatchSlots] = {};
    void *batch_host[rtamd::kBatchSlots] = {};
    hipEvent_t batch_done[rtamd::kBatchSlots] = {};
    bool batch_used[rtamd::kBatchSlots] = {};
    unsigned batch_next = 0;
    int n_cu = 0;               // compute units of the device
    int32_t *sched = nullptr;   // kSchedSlots x kSchedInts queue counters (zeroed)
    unsigned sched_next = 0;    // next slot: launches in flight on several streams use distinct slots
    // per slot: an event recorded after the slot's last queued launch; a
    // launch that reuses the slot waits for it on its own stream, so more
    // than kSchedSlots queued launches in flight never share counters
    hipEvent_t sched_done[rtamd::kSchedSlots] = {};
    bool sched_used[rtamd::kSchedSlots] = {};
    std::vector<struct rt_scene *> scenes;  // live scenes (detached by rt_destroy)
};

struct rt_scene {
    int device = 0;
    rtamd::DeviceScene dev;
    std::vector<float4> host;    // host copy of the blob (per-frame constants on the host)
    int32_t capacity_units = 0;  // allocated blob size (16-B units)
    rt_context *ctx = nullptr;   // owning context (nullptr once it is destroyed)
    // Renders that read the blob on streams other than the owning context's:
    // per stream, an event recorded after its latest such render. The blob
    // is freed or overwritten only behind all of them (stream order covers
    // the context's own stream). More than kMaxUseStreams streams: `overflow`,
    // and the release synchronises the device instead.
    static constexpr int kMaxUseStreams = 8;
    using Event = rtamd::UseEvent;
    struct Use {
        hipStream_t stream;
        std::shared_ptr<Event> done;
    };
    mutable std::vector<Use> uses;
    mutable bool overflow = false;
    mutable bool warned = false;  // the overflow's one-time stderr notice was printed
};
