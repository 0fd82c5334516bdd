// rt_scene.cpp — host side of the hot path: the reference scene / camera
// restated as C++ data, the frame constants (camera unprojection, per-object
// transforms) and the device-resident scene blob.
//
// The reference orbit camera's unprojection is evaluated as the reference's
// GL evaluates it (rt_camera.cpp, bit-identical to llvmpipe). The per-object
// transforms (:650-652, :718) and explicit cameras are evaluated in float64
// and rounded once to float32 ("Parity").
// Everything the kernel evaluates per pixel stays float32 in GLSL order.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "rt_internal.h"

using namespace rtamd;

namespace {

constexpr float kPi = 3.14159265358f;            // raytrace_compute.glsl:13
constexpr float kDegToRad = kPi / 180.0f;         // :17 (folded in float)

struct M4 {
    double m[4][4];  // column-major, m[col][row] as GLSL
};

M4 ident() {
    M4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0;
    return r;
}

M4 mul(const M4 &a, const M4 &b) {
    M4 r{};
    for (int c = 0; c < 4; ++c)
        for (int row = 0; row < 4; ++row) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc += a.m[k][row] * b.m[c][k];
            r.m[c][row] = acc;
        }
    return r;
}

// Inverse via the 4x4 adjugate (float64).
M4 inverse(const M4 &a) {
    const double *s = &a.m[0][0];  // column-major linear
    double inv[16];
    inv[0] = s[5] * s[10] * s[15] - s[5] * s[11] * s[14] - s[9] * s[6] * s[15] + s[9] * s[7] * s[14] +
             s[13] * s[6] * s[11] - s[13] * s[7] * s[10];
    inv[4] = -s[4] * s[10] * s[15] + s[4] * s[11] * s[14] + s[8] * s[6] * s[15] - s[8] * s[7] * s[14] -
             s[12] * s[6] * s[11] + s[12] * s[7] * s[10];
    inv[8] = s[4] * s[9] * s[15] - s[4] * s[11] * s[13] - s[8] * s[5] * s[15] + s[8] * s[7] * s[13] +
             s[12] * s[5] * s[11] - s[12] * s[7] * s[9];
    inv[12] = -s[4] * s[9] * s[14] + s[4] * s[10] * s[13] + s[8] * s[5] * s[14] - s[8] * s[6] * s[13] -
              s[12] * s[5] * s[10] + s[12] * s[6] * s[9];
    inv[1] = -s[1] * s[10] * s[15] + s[1] * s[11] * s[14] + s[9] * s[2] * s[15] - s[9] * s[3] * s[14] -
             s[13] * s[2] * s[11] + s[13] * s[3] * s[10];
    inv[5] = s[0] * s[10] * s[15] - s[0] * s[11] * s[14] - s[8] * s[2] * s[15] + s[8] * s[3] * s[14] +
             s[12] * s[2] * s[11] - s[12] * s[3] * s[10];
    inv[9] = -s[0] * s[9] * s[15] + s[0] * s[11] * s[13] + s[8] * s[1] * s[15] - s[8] * s[3] * s[13] -
             s[12] * s[1] * s[11] + s[12] * s[3] * s[9];
    inv[13] = s[0] * s[9] * s[14] - s[0] * s[10] * s[13] - s[8] * s[1] * s[14] + s[8] * s[2] * s[13] +
              s[12] * s[1] * s[10] - s[12] * s[2] * s[9];
    inv[2] = s[1] * s[6] * s[15] - s[1] * s[7] * s[14] - s[5] * s[2] * s[15] + s[5] * s[3] * s[14] +
             s[13] * s[2] * s[7] - s[13] * s[3] * s[6];
    inv[6] = -s[0] * s[6] * s[15] + s[0] * s[7] * s[14] + s[4] * s[2] * s[15] - s[4] * s[3] * s[14] -
             s[12] * s[2] * s[7] + s[12] * s[3] * s[6];
    inv[10] = s[0] * s[5] * s[15] - s[0] * s[7] * s[13] - s[4] * s[1] * s[15] + s[4] * s[3] * s[13] +
              s[12] * s[1] * s[7] - s[12] * s[3] * s[5];
    inv[14] = -s[0] * s[5] * s[14] + s[0] * s[6] * s[13] + s[4] * s[1] * s[14] - s[4] * s[2] * s[13] -
              s[12] * s[1] * s[6] + s[12] * s[2] * s[5];
    inv[3] = -s[1] * s[6] * s[11] + s[1] * s[7] * s[10] + s[5] * s[2] * s[11] - s[5] * s[3] * s[10] -
             s[9] * s[2] * s[7] + s[9] * s[3] * s[6];
    inv[7] = s[0] * s[6] * s[11] - s[0] * s[7] * s[10] - s[4] * s[2] * s[11] + s[4] * s[3] * s[10] +
             s[8] * s[2] * s[7] - s[8] * s[3] * s[6];
    inv[11] = -s[0] * s[5] * s[11] + s[0] * s[7] * s[9] + s[4] * s[1] * s[11] - s[4] * s[3] * s[9] -
              s[8] * s[1] * s[7] + s[8] * s[3] * s[5];
    inv[15] = s[0] * s[5] * s[10] - s[0] * s[6] * s[9] - s[4] * s[1] * s[10] + s[4] * s[2] * s[9] +
              s[8] * s[1] * s[6] - s[8] * s[2] * s[5];
    double det = s[0] * inv[0] + s[1] * inv[4] + s[2] * inv[8] + s[3] * inv[12];
    M4 r;
    double *o = &r.m[0][0];
    for (int i = 0; i < 16; ++i) o[i] = inv[i] / det;
    return r;
}

// rotation_matrix_{x,y,z} (:444-486): the angle enters as the float
// DEG_TO_RAD * deg the shader forms, then cos/sin in float64.
M4 rot(int axis, float deg) {
    const double a = static_cast<double>(kDegToRad * deg);
    const double c = std::cos(a), s = std::sin(a);
    M4 r = ident();
    if (axis == 0) { r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = -s; r.m[2][2] = c; }
    if (axis == 1) { r.m[0][0] = c; r.m[0][2] = -s; r.m[2][0] = s; r.m[2][2] = c; }
    if (axis == 2) { r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = -s; r.m[1][1] = c; }
    return r;
}

// calc_transform_matrix (:529-532) = translation (:432) * rotation (:492-503:
// yaw about z, then pitch about x, then roll about y).
M4 transform(const float pos[3], const float ang[3]) {
    M4 t = ident();
    t.m[3][0] = pos[0];
    t.m[3][1] = pos[1];
    t.m[3][2] = pos[2];
    return mul(t, mul(mul(rot(2, ang[1]), rot(0, ang[0])), rot(1, ang[2])));
}

void set4(float *d, float a, float b, float c, float e) {
    d[0] = a; d[1] = b; d[2] = c; d[3] = e;
}
void set4s(float *d, float s) { set4(d, s, s, s, s); }

void set_material(rt_material &m, float amb, const float dif[4], float spe, float shin, float refl, float transp,
                  float ior) {
    set4s(m.ambient, amb);
    std::memcpy(m.diffuse, dif, 16);
    set4s(m.specular, spe);
    m.shininess = shin;
    set4s(m.emissive, 0.0f);
    m.reflectivity = refl;
    m.transparency = transp;
    m.refraction_index = ior;
}

void make_object(rt_object &o, float mn[3], float mx[3], float radius, float p0, float p1, float p2, float a0, float a1,
                 float a2, int mat) {
    std::memcpy(o.box_mins, mn, 12);
    std::memcpy(o.box_maxs, mx, 12);
    o.radius = radius;
    o.position[0] = p0; o.position[1] = p1; o.position[2] = p2;
    o.angles[0] = a0; o.angles[1] = a1; o.angles[2] = a2;
    o.material = mat;
}

// get_closest_collision's type test (:749-771).
int object_kind(const rt_object &o) {
    const bool box = !(o.box_mins[0] == 0.0f && o.box_mins[1] == 0.0f && o.box_mins[2] == 0.0f &&
                       o.box_maxs[0] == 0.0f && o.box_maxs[1] == 0.0f && o.box_maxs[2] == 0.0f);
    if (box) return 1;
    if (o.radius != -1.0f) return 2;
    return 0;
}

uint64_t splitmix64(uint64_t &state) {
    state += 0x9E3779B97F4A7C15ULL;
    uint64_t z = state;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

float uniform(uint64_t &state, double lo, double hi) {
    const double u = static_cast<double>(splitmix64(state) >> 11) * (1.0 / 9007199254740992.0);
    return static_cast<float>(lo + (hi - lo) * u);
}

}  // namespace

extern "C" {

// raytrace_compute.glsl:74-157
int rt_reference_materials(rt_material out[RT_REFERENCE_MATERIALS]) {
    if (!out) { set_error("rt_reference_materials: null out"); return RT_ERR_INVALID; }
    const float d1[4] = {0.5f, 0.0f, 0.0f, 1.0f}, d2[4] = {0.3f, 0.6f, 0.3f, 1.0f};
    const float dr[4] = {1, 0, 0, 1}, dg[4] = {0, 1, 0, 1}, db[4] = {0, 0, 1, 1};
    const float dm[4] = {0.6f, 0.6f, 0.6f, 1.0f}, dw[4] = {0.4f, 0.4f, 0.4f, 0.4f};
    set_material(out[RT_MAT_MATERIAL1], 1.0f, d1, 1.0f, 4.0f, 1.0f, 0.0f, 1.5f);
    set_material(out[RT_MAT_MATERIAL2], 1.0f, d2, 1.0f, 4.0f, 1.0f, 0.0f, 1.5f);
    set_material(out[RT_MAT_RED_GLASS], 1.0f, dr, 1.0f, 10.0f, 0.8f, 0.4f, 1.5f);
    set_material(out[RT_MAT_GREEN_GLASS], 1.0f, dg, 1.0f, 10.0f, 0.4f, 0.6f, 1.5f);
    set_material(out[RT_MAT_BLUE_GLASS], 1.0f, db, 1.0f, 10.0f, 0.4f, 0.6f, 1.5f);
    set_material(out[RT_MAT_MIRROR], 1.0f, dm, 1.0f, 4.0f, 1.0f, 0.0f, 1.0f);
    set_material(out[RT_MAT_WALL], 0.5f, dw, 0.3f, 3.0f, 0.3f, 0.0f, 1.0f);
    return RT_OK;
}

// raytrace_compute.glsl:199-224
int rt_reference_lights(rt_light out[RT_REFERENCE_LIGHTS]) {
    if (!out) { set_error("rt_reference_lights: null out"); return RT_ERR_INVALID; }
    const float pos[3][3] = {{0.1f, 0.1f, 0.1f}, {7.0f, 7.0f, 2.0f}, {3.0f, -3.0f, 4.0f}};
    for (int i = 0; i < 3; ++i) std::memcpy(out[i].position, pos[i], 12);
    set4s(out[0].ambient, 0.3f); set4s(out[0].diffuse, 0.0f); set4s(out[0].specular, 0.0f);
    set4s(out[1].ambient, 0.05f); set4s(out[1].diffuse, 1.0f); set4s(out[1].specular, 1.0f);
    set4s(out[2].ambient, 0.05f);
    set4(out[2].diffuse, 1.0f, 0.0f, 0.0f, 1.0f);
    set4(out[2].specular, 1.0f, 0.0f, 0.0f, 1.0f);
    return RT_OK;
}

int rt_object_transforms(const rt_object *obj, float l2w[16], float w2l[16], float nrm[9]) {
    if (!obj || !l2w || !w2l || !nrm) {
        set_error("rt_object_transforms: null argument");
        return RT_ERR_INVALID;
    }
    reference_box_transforms(obj->position, obj->angles, l2w, w2l, nrm);
    return RT_OK;
}

// raytrace_compute.glsl:236-237 (scaled_time), :261-321 (objects)
int rt_reference_objects(float time, rt_object out[RT_REFERENCE_OBJECTS]) {
    if (!out) { set_error("rt_reference_objects: null out"); return RT_ERR_INVALID; }
    // scaled_time * k = (time * time_scale) * k, which the reference's GL
    // compiles as time * (time_scale * k) (a product by a constant times
    // another constant folds; probed on llvmpipe)
    auto st = [time](float k) { return time * (0.4f * k); };
    float zero[3] = {0, 0, 0};
    float mn0[3] = {-11, -11, -11}, mx0[3] = {11, 11, 11};
    make_object(out[0], mn0, mx0, -1.0f, 0, 0, 0, 0, 0, 0, RT_MAT_WALL);
    // run-time sin as the reference's GL evaluates it (rt_camera.cpp)
    const float s = 0.5f * gl_sin(st(0.5f)) + 1.5f;
    float mn1[3] = {-1.0f * s, -1.0f * s, -1.0f * s}, mx1[3] = {1.0f * s, 1.0f * s, 1.0f * s};
    make_object(out[1], mn1, mx1, -1.0f, 0, 0, gl_sin(st(3.0f)), 0, st(90.0f), 0, RT_MAT_MIRROR);
    float mn2[3] = {-10, -10, -1}, mx2[3] = {10, 10, 1};
    make_object(out[2], mn2, mx2, -1.0f, 0, 0, -3, gl_sin(st(5.0f)) * 10.0f, 45.0f, 0, RT_MAT_GREEN_GLASS);
    float mn3[3] = {-1, -1, -2}, mx3[3] = {1, 1, 2};
    make_object(out[3], mn3, mx3, -1.0f, 3, 4, 1, 45.0f + st(45.0f), 0, 45.0f + st(180.0f), RT_MAT_BLUE_GLASS);
    make_object(out[4], zero, zero, 2.0f, -3, 4, 1, 0, 0, 0, RT_MAT_RED_GLASS);
    return RT_OK;
}

// raytrace_compute.glsl:334-364 (run-time sin / cos and mod() as the
// reference's GL evaluates them, rt_camera.cpp)
int rt_reference_camera(float time, rt_camera *out) {
    if (!out) { set_error("rt_reference_camera: null out"); return RT_ERR_INVALID; }
    float yaw;
    reference_orbit(time, nullptr, out->position, &yaw);
    out->angles[0] = 0.0f;
    out->angles[1] = yaw;
    out->angles[2] = 0.0f;
    out->near_plane = 0.1f;
    out->far_plane = 1000.0f;
    out->aspect = 16.0f / 9.0f;
    out->v_fov = 90.0f;
    return RT_OK;
}

int rt_bench_objects(int n_spheres, uint64_t seed, rt_object *out) {
    if (!out || n_spheres < 0 || n_spheres + 1 > RT_MAX_OBJECTS) {
        set_error("rt_bench_objects: bad arguments");
        return RT_ERR_INVALID;
    }
    float mn[3] = {-11, -11, -11}, mx[3] = {11, 11, 11}, zero[3] = {0, 0, 0};
    make_object(out[0], mn, mx, -1.0f, 0, 0, 0, 0, 0, 0, RT_MAT_WALL);
    static const int cycle[6] = {RT_MAT_MATERIAL1, RT_MAT_MATERIAL2, RT_MAT_RED_GLASS,
                                 RT_MAT_GREEN_GLASS, RT_MAT_BLUE_GLASS, RT_MAT_MIRROR};
    uint64_t st = seed;
    for (int i = 0; i < n_spheres; ++i) {
        const float cx = uniform(st, -8.0, 8.0);
        const float cy = uniform(st, -8.0, 8.0);
        const float cz = uniform(st, -4.0, 4.0);
        const float r = uniform(st, 0.3, 1.2);
        make_object(out[i + 1], zero, zero, r, cx, cy, cz, 0, 0, 0, cycle[i % 6]);
    }
    return RT_OK;
}

// main() :366-392 — P (:411-426) and V = inverse(T * R * Rx(90)) (:538-545),
// unprojection = inverse(P * V).
//  cam == NULL: the reference orbit camera at `time`, evaluated as the
//    reference's GL evaluates it (rt_camera.cpp) — bit-identical to llvmpipe;
//  an explicit camera (no counterpart in the reference, which hard-codes its
//    camera): float64, rounded once.
int rt_make_view(const rt_camera *cam_in, float time, rt_view *out) {
    if (!out) { set_error("rt_make_view: null out"); return RT_ERR_INVALID; }
    if (!cam_in) {
        float speed, yaw;
        reference_orbit(time, &speed, out->origin, &yaw);  // ray start = c.position (:391)
        reference_view_gl(time, out->unprojection, nullptr);
        return RT_OK;
    }
    const rt_camera cam = *cam_in;
    const double q = 1.0 / std::tan(static_cast<double>(kDegToRad * 0.5f * cam.v_fov));
    const double n = cam.near_plane, f = cam.far_plane;
    M4 P{};
    P.m[0][0] = q / cam.aspect;
    P.m[1][1] = q;
    P.m[2][2] = (n + f) / (n - f);
    P.m[2][3] = -1.0;
    P.m[3][2] = (2.0 * n * f) / (n - f);
    const M4 V = inverse(mul(transform(cam.position, cam.angles), rot(0, 90.0f)));
    const M4 U = inverse(mul(P, V));
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out->unprojection[c * 4 + r] = static_cast<float>(U.m[c][r]);
    std::memcpy(out->origin, cam.position, 12);
    return RT_OK;
}

}  // extern "C"

namespace rtamd {

namespace {

// Build a BVH over the spheres with finite centre and radius (the others can
// never produce a valid hit: their quadratic is NaN or its roots infinite),
// reordering `sph`/`smeta` into leaf order. Median split on the widest
// centroid axis, leaves of <= RT_BVH_LEAF spheres, depth-first layout with skip links.
struct BuildItem {
    SphereRec s;
    SphereMeta m;
    double lo[3], hi[3], c[3];
};

int build_node(std::vector<BuildItem> &items, int begin, int end, std::vector<BvhNode> &nodes,
               std::vector<int> &axes) {
    const int id = static_cast<int>(nodes.size());
    nodes.push_back(BvhNode{});
    axes.push_back(0);
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
    for (int i = begin; i < end; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], items[i].lo[a]);
            hi[a] = std::max(hi[a], items[i].hi[a]);
            clo[a] = std::min(clo[a], items[i].c[a]);
            chi[a] = std::max(chi[a], items[i].c[a]);
        }
    BvhNode &n = nodes[id];
    for (int a = 0; a < 3; ++a) {
        n.lo[a] = std::nextafter(static_cast<float>(lo[a]), -INFINITY);
        n.hi[a] = std::nextafter(static_cast<float>(hi[a]), INFINITY);
    }
#ifndef RT_BVH_LEAF  // leaves of up to 6 spheres: config 4 22.04 -> 21.82 ms against 4 (2: 24.7, 3: 22.3, 8: 21.8;
#define RT_BVH_LEAF 6  // SAH leaf termination at 6-8 spheres: 22.3-29.2 ms); config 3 within 0.5 %
#endif
    if (end - begin <= RT_BVH_LEAF) {
        n.leaf = ((end - begin) << 24) | begin;
        return id;
    }
    // surface-area heuristic: over every axis and every split of the
    // centroid-sorted items, minimise A(left) N(left) + A(right) N(right)
    // (a sphere test costs about one node test; ties keep the median split)
    const int cnt = end - begin;
    auto area = [](const double *l, const double *h) {
        const double dx = h[0] - l[0], dy = h[1] - l[1], dz = h[2] - l[2];
        return dx * dy + dy * dz + dz * dx;
    };
    int best_axis = -1, best_mid = (begin + end) / 2;
#ifndef RT_BVH_MEDIAN
    double best = 1e300;
    std::vector<double> left_area(cnt);
    for (int a = 0; a < 3; ++a) {
        std::sort(items.begin() + begin, items.begin() + end,
                  [a](const BuildItem &x, const BuildItem &y) { return x.c[a] < y.c[a]; });
        double l[3] = {1e300, 1e300, 1e300}, h[3] = {-1e300, -1e300, -1e300};
        for (int i = 0; i < cnt; ++i) {
            for (int k = 0; k < 3; ++k) {
                l[k] = std::min(l[k], items[begin + i].lo[k]);
                h[k] = std::max(h[k], items[begin + i].hi[k]);
            }
            left_area[i] = area(l, h);  // items [begin, begin + i]
        }
        double rl[3] = {1e300, 1e300, 1e300}, rh[3] = {-1e300, -1e300, -1e300};
        for (int i = cnt - 1; i >= 1; --i) {  // right = [begin + i, end)
            for (int k = 0; k < 3; ++k) {
                rl[k] = std::min(rl[k], items[begin + i].lo[k]);
                rh[k] = std::max(rh[k], items[begin + i].hi[k]);
            }
            const double cost = left_area[i - 1] * i + area(rl, rh) * (cnt - i);
            if (cost < best) {
                best = cost;
                best_axis = a;
                best_mid = begin + i;
            }
        }
    }
#endif
    int axis = best_axis;
    if (axis < 0) {  // median split on the widest centroid axis
        axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
    }
    const int mid = best_mid;
    std::sort(items.begin() + begin, items.begin() + end,
              [axis](const BuildItem &x, const BuildItem &y) { return x.c[axis] < y.c[axis]; });
    nodes[id].leaf = 0;
    axes[id] = axis;
    build_node(items, begin, mid, nodes, axes);
    build_node(items, mid, end, nodes, axes);
    return id;
}

// Subtree sizes make the skip links: in depth-first order a subtree rooted at
// id occupies [id, id + size).
int subtree_size(const std::vector<BvhNode> &nodes, int id) {
    if (nodes[id].leaf) return 1;
    const int left = subtree_size(nodes, id + 1);
    return 1 + left + subtree_size(nodes, id + 1 + left);
}

void set_skips(std::vector<BvhNode> &nodes, int id, int next) {
    nodes[id].skip = next;
    if (nodes[id].leaf) return;
    const int left = id + 1, left_size = subtree_size(nodes, left);
    const int right = left + left_size;
    set_skips(nodes, left, right);
    set_skips(nodes, right, next);
}

// The octant's depth-first order (rt_internal.h, kBvhOctants): the children
// of an inner node split on axis a (left: the lower centroids) are entered
// right first when the octant's d[a] < 0.
static_assert(2 * RT_MAX_OBJECTS < 0x8000, "BVH node indices fit the 16-bit links");
void set_links(const std::vector<BvhNode> &nodes, const std::vector<int> &axes, int id, int next, int oct,
               std::vector<uint32_t> &links) {
    auto enc = [](int n) { return static_cast<uint32_t>(n) & 0xFFFFu; };  // -1 -> 0xFFFF
    if (nodes[id].leaf) {
        links[static_cast<size_t>(id) * kBvhOctants + oct] = enc(next) | (enc(next) << 16);
        return;
    }
    const int left = id + 1, right = left + subtree_size(nodes, left);
    const bool flip = (oct >> axes[id]) & 1;
    const int first = flip ? right : left, second = flip ? left : right;
    links[static_cast<size_t>(id) * kBvhOctants + oct] = enc(first) | (enc(next) << 16);
    set_links(nodes, axes, first, second, oct, links);
    set_links(nodes, axes, second, next, oct, links);
}

// extent: a bound on |coordinate| of every finite object of the scene (the
// origins of the secondary rays that walk the BVH lie on their surfaces).
void build_bvh(std::vector<SphereRec> &sph, std::vector<SphereMeta> &smeta, std::vector<BvhNode> &nodes,
               std::vector<uint32_t> &links, double extent) {
    std::vector<BuildItem> finite, other;
    for (size_t i = 0; i < sph.size(); ++i) {
        BuildItem it{sph[i], smeta[i], {}, {}, {}};
        const double c[3] = {sph[i].cx, sph[i].cy, sph[i].cz};
        const double r = std::sqrt(static_cast<double>(sph[i].rr));  // |radius| as the test sees it
        bool ok = std::isfinite(r);
        double mag = 0.0;
        for (int a = 0; a < 3; ++a) {
            ok = ok && std::isfinite(c[a]);
            mag = std::max(mag, std::fabs(c[a]) + r);
        }
        // the kernel's node test (rt_kernel.hip, node_hit) has no slack of
        // its own: its error, ~2^-22 (|x| + |o|) / |d|, stays far below this
        // margin for every box coordinate x and ray origin o of the scene
        const double margin = 1e-3 + 1e-4 * std::max(mag, extent);
        for (int a = 0; a < 3; ++a) {
            it.c[a] = c[a];
            it.lo[a] = c[a] - r - margin;
            it.hi[a] = c[a] + r + margin;
        }
        (ok ? finite : other).push_back(it);
    }
    nodes.clear();
    links.clear();
    if (!finite.empty()) {
        std::vector<int> axes;
        build_node(finite, 0, static_cast<int>(finite.size()), nodes, axes);
        set_skips(nodes, 0, -1);
        links.assign(nodes.size() * kBvhOctants, 0u);
        for (int oct = 0; oct < kBvhOctants; ++oct) set_links(nodes, axes, 0, -1, oct, links);
    }
    // leaf order first, then the spheres that cannot be hit (linear loops only)
    sph.clear();
    smeta.clear();
    for (auto *v : {&finite, &other})
        for (const BuildItem &it : *v) {
            sph.push_back(it.s);
            smeta.push_back(it.m);
        }
}

}  // namespace

// proj*view for culling: the float64 inverse of the view's unprojection, and
// whether the view is a consistent pinhole (every pixel's ray, built as the
// kernel builds it, lies on the line through the origin and its NDC point,
// with positive homogeneous w) so that projected footprints bound ray hits.
bool view_projection(const rt_view &v, float proj[16]) {
    M4 U;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) U.m[c][r] = v.unprojection[c * 4 + r];
    const M4 P = inverse(U);
    bool ok = true;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            proj[c * 4 + r] = static_cast<float>(P.m[c][r]);
            ok = ok && std::isfinite(P.m[c][r]);
        }
    const double o[3] = {v.origin[0], v.origin[1], v.origin[2]};
    const double ndc[5][2] = {{-1, -1}, {1, -1}, {-1, 1}, {1, 1}, {0, 0}};
    for (int i = 0; i < 5 && ok; ++i) {
        double pt[2][3];
        for (int k = 0; k < 2; ++k) {
            const double z = k == 0 ? 0.5 : 1.0;
            double h[4];
            for (int r = 0; r < 4; ++r)
                h[r] = U.m[0][r] * ndc[i][0] + U.m[1][r] * ndc[i][1] + U.m[2][r] * z + U.m[3][r];
            ok = ok && h[3] > 0.0;
            for (int r = 0; r < 3; ++r) pt[k][r] = h[r] / h[3];
        }
        // distance of the origin from the line through the two points
        double d[3], w[3];
        for (int r = 0; r < 3; ++r) {
            d[r] = pt[1][r] - pt[0][r];
            w[r] = o[r] - pt[0][r];
        }
        const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double cx = d[1] * w[2] - d[2] * w[1], cy = d[2] * w[0] - d[0] * w[2], cz = d[0] * w[1] - d[1] * w[0];
        const double dist = std::sqrt((cx * cx + cy * cy + cz * cz) / dd);
        const double scale = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) + 1e-12;
        ok = ok && dd > 0.0 && dist <= 1e-5 * scale;
    }
    return ok;
}

// Whether the camera ray's six perspective divisions (raytrace_compute.glsl
// :383-390, ws[k] / ws[3] and we[k] / we[3]) may take the short form
// (rt_kernel.hip div_r: the refined reciprocal of the w component and one
// correction, correctly rounded for b normal in [2^-60, 2^60] and a = +0 or
// |a| in [2^-60, 2^60]) for EVERY pixel of a width x height frame, jittered
// samples included. Each component is ((M[k] vx + M[4+k] vy) + M[8+k] z) +
// M[12+k] in float32 with vx in [-1, (width - hw) / hw], vy likewise and z in
// {0.5, 1}:
//  * a numerator's last operation adds c = M[12+k] != 0 to a float y: a
//    nonzero result is at least 2^-26 |c| (if |y| >= |c| / 2 both are
//    multiples of ulp(c) / 2, else |y + c| > |c| / 2), and an exact
//    cancellation gives +0, never -0; so |c| >= 2^-34 keeps every nonzero
//    numerator at or above 2^-60;
//  * the denominators are the linear function w(vx, vy, z) up to rounding:
//    its extremes over the pixel box are at the corners (float64), and the
//    float32 evaluation differs from it by at most 8 * 2^-24 times the sum
//    of the terms' magnitudes; both sit in [2^-20, 2^20] or in the mirror
//    range, every pixel's w does.
bool camera_short_divisions(const float M[16], int width, int height) {
    const int hw = width / 2, hh = height / 2;
    if (hw <= 0 || hh <= 0) return false;
    for (int i = 0; i < 16; ++i)
        if (!std::isfinite(M[i]) || std::fabs(M[i]) > 0x1p40f) return false;
    for (int k = 0; k < 4; ++k)
        if (!(std::fabs(M[12 + k]) >= 0x1p-34f)) return false;
    const double vx[2] = {-1.0, static_cast<double>(width - hw) / hw};
    const double vy[2] = {-1.0, static_cast<double>(height - hh) / hh};
    for (const double z : {0.5, 1.0}) {
        const double mag = std::fabs(M[3]) * std::max(std::fabs(vx[0]), std::fabs(vx[1])) +
                           std::fabs(M[7]) * std::max(std::fabs(vy[0]), std::fabs(vy[1])) + std::fabs(M[11]) * z +
                           std::fabs(M[15]);
        const double err = 8.0 * 0x1p-24 * mag + 0x1p-100;
        double lo = INFINITY, hi = -INFINITY;
        for (const double x : vx)
            for (const double y : vy) {
                const double w = double(M[3]) * x + double(M[7]) * y + double(M[11]) * z + double(M[15]);
                lo = std::min(lo, w);
                hi = std::max(hi, w);
            }
        const bool pos = lo - err >= 0x1p-20 && hi + err <= 0x1p20;
        const bool neg = hi + err <= -0x1p-20 && lo - err >= -0x1p20;
        if (!pos && !neg) return false;
    }
    return true;
}

// The kernel's frame_setup (rt_kernel.hip) for a one-view launch, on the
// host: every work-group would otherwise derive the same constants (measured
// 7 % of a 1080p depth-0 frame). Camera terms in float32 with the kernel's
// operation order (dot = x*x + (y*y + z*z); xform_point left to right), so the
// LDS image is bit-identical; footprints in float64 with the same inflation
// and 2-pixel margin — closer to the exact projection than the kernel's
// approximate-reciprocal version, and as conservative.
static void view_frame_setup(const LaunchParams &p, const FrameView &V, const float4 *blob, float4 *out);

void host_frame_setup(LaunchParams &p, const float4 *const *blobs) {
    p.n_frame_consts = 0;
    const int ns = p.n_spheres, nb = p.n_boxes, per = 2 * ns + nb;
    if (per == 0 || per > kMaxViewConsts || p.n_views < 1 || p.n_views * per > kMaxFrameConsts) return;
    for (int k = 0; k < p.n_views; ++k)
        if (!blobs[k]) return;
    for (int k = 0; k < p.n_views; ++k) view_frame_setup(p, p.view[k], blobs[k], p.frame_consts + k * per);
    p.n_frame_consts = per;
}

int host_view_consts(const LaunchParams &p, const FrameView &V, const float4 *blob, float4 *out) {
    const int per = 2 * p.n_spheres + p.n_boxes;
    if (per == 0 || per > kMaxViewConsts || !blob) return 0;
    view_frame_setup(p, V, blob, out);
    return per;
}

// One view's records (host_frame_setup).
static void view_frame_setup(const LaunchParams &p, const FrameView &V, const float4 *blob, float4 *out) {
    const int ns = p.n_spheres, nb = p.n_boxes;
    const float ox = V.origin[0], oy = V.origin[1], oz = V.origin[2];
    const int hw = p.width / 2, hh = p.height / 2;
    const bool cull = V.cull && hw > 0 && hh > 0;
    const float *P = V.proj;
    const auto *sph = reinterpret_cast<const SphereRec *>(blob + p.off_spheres);
    const auto *meta = reinterpret_cast<const SphereMeta *>(blob + p.off_smeta);
    const auto *box = reinterpret_cast<const BoxRec *>(blob + p.off_boxes);
    float4 *cam = out, *px = out + ns, *bcam = out + 2 * ns;
    for (int s = 0; s < ns; ++s) {
        const SphereRec c = sph[s];
        const float ocx = ox - c.cx, ocy = oy - c.cy, ocz = oz - c.cz;
        const float dd = ocx * ocx + (ocy * ocy + ocz * ocz);
        cam[s] = make_float4(ocx, ocy, ocz, dd - c.rr);
        const float r = meta[s].radius * 1.001f + 1e-3f;
        bool ok = r == r && c.cx == c.cx && c.cy == c.cy && c.cz == c.cz;
        double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
        for (int i = 0; i < 8 && ok; ++i) {
            const double X = c.cx + ((i & 1) ? r : -r), Y = c.cy + ((i & 2) ? r : -r), Z = c.cz + ((i & 4) ? r : -r);
            const double cw = P[3] * X + P[7] * Y + P[11] * Z + P[15];
            const double cx = P[0] * X + P[4] * Y + P[8] * Z + P[12];
            const double cy = P[1] * X + P[5] * Y + P[9] * Z + P[13];
            ok = cw > 1e-4;
            x0 = std::min(x0, cx / cw);
            x1 = std::max(x1, cx / cw);
            y0 = std::min(y0, cy / cw);
            y1 = std::max(y1, cy / cw);
        }
        const double fx0 = std::floor(x0 * hw + hw) - 2.0, fx1 = std::ceil(x1 * hw + hw) + 2.0;
        const double fy0 = std::floor(y0 * hh + hh) - 2.0, fy1 = std::ceil(y1 * hh + hh) + 2.0;
        const double lim = 1.0e9;
        const bool fin = std::fabs(fx0) < lim && std::fabs(fx1) < lim && std::fabs(fy0) < lim && std::fabs(fy1) < lim;
        int32_t rect[4] = {INT32_MIN / 2, INT32_MAX / 2, INT32_MIN / 2, INT32_MAX / 2};
        if (cull && ok && fin) {
            rect[0] = static_cast<int32_t>(fx0);
            rect[1] = static_cast<int32_t>(fx1);
            rect[2] = static_cast<int32_t>(fy0);
            rect[3] = static_cast<int32_t>(fy1);
        }
        std::memcpy(&px[s], rect, sizeof rect);
    }
    for (int b = 0; b < nb; ++b) {
        const float *m = box[b].w2l;
        const float rx = m[0] * ox + m[1] * oy + m[2] * oz + m[3] * 1.0f;
        const float ry = m[4] * ox + m[5] * oy + m[6] * oz + m[7] * 1.0f;
        const float rz = m[8] * ox + m[9] * oy + m[10] * oz + m[11] * 1.0f;
        const BoxRec &B = box[b];
        const bool inside = B.mins[0] < rx && rx < B.maxs[0] && B.mins[1] < ry && ry < B.maxs[1] && B.mins[2] < rz &&
                            rz < B.maxs[2];
        bcam[b] = make_float4(rx, ry, rz, inside ? 1.0f : 0.0f);
    }
}

// The texel and block cones of an n x n cube map (geometry only: computed
// once per n and kept). Texels are grouped in blocks of kMaskBlock x
// kMaskBlock; a block's reach is its own cone's half-angle plus the largest
// half-angle of its texels.
constexpr int kMaskBlock = 8;
struct MaskCones {
    int n = 0;
    std::vector<double> w, ca, sa;  // per texel (face-major): centre direction, cos / sin of the half-angle
    struct Block {
        int face, r0, r1, c0, c1;
        double w[3], reach, cr, sr;  // centre direction, reach and its cos / sin
    };
    std::vector<Block> blocks;
    // per block, its kMaskSubBlock x kMaskSubBlock sub-blocks (same reach rule)
    std::vector<std::vector<Block>> subs;
};
constexpr int kMaskSubBlock = 2;

const MaskCones &mask_cones(int n) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<MaskCones>> cache;
    std::lock_guard<std::mutex> lock(mu);
    std::unique_ptr<MaskCones> &slot = cache[n];
    if (slot) return *slot;
    auto unit = [](double v[3]) {
        const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        for (int k = 0; k < 3; ++k) v[k] /= l;
    };
    auto angle = [](const double a[3], const double b[3]) {
        const double c = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
        return std::acos(std::max(-1.0, std::min(1.0, c)));
    };
    auto mc = std::make_unique<MaskCones>();
    mc->n = n;
    const size_t texels = static_cast<size_t>(6) * n * n;
    mc->w.resize(3 * texels);
    mc->ca.resize(texels);
    mc->sa.resize(texels);
    std::vector<double> alpha(texels);
    for (int f = 0; f < 6; ++f) {
        // face f's point (a, b) in the kernel's cube-map coordinates
        // (direction_texel: the cube instructions' sc / |major|, tc / |major|,
        // column from sc, row from tc), as a direction
        auto face_dir = [f](double a, double b, double q[3]) {
            switch (f) {
                case 0: q[0] = 1.0; q[1] = -b; q[2] = -a; break;   // +x: sc = -z, tc = -y
                case 1: q[0] = -1.0; q[1] = -b; q[2] = a; break;   // -x: sc = z, tc = -y
                case 2: q[0] = a; q[1] = 1.0; q[2] = b; break;     // +y: sc = x, tc = z
                case 3: q[0] = a; q[1] = -1.0; q[2] = -b; break;   // -y: sc = x, tc = -z
                case 4: q[0] = a; q[1] = -b; q[2] = 1.0; break;    // +z: sc = x, tc = -y
                default: q[0] = -a; q[1] = -b; q[2] = -1.0; break; // -z: sc = -x, tc = -y
            }
        };
        // a square [a0, a1] x [b0, b1] of the face: its centre direction and
        // the half-angle of the cone through its corners
        auto cone = [&](double a0, double a1, double b0, double b1, double w[3]) {
            face_dir(0.5 * (a0 + a1), 0.5 * (b0 + b1), w);
            unit(w);
            double al = 0.0;
            for (int k = 0; k < 4; ++k) {
                double q[3];
                face_dir((k & 1) ? a1 : a0, (k & 2) ? b1 : b0, q);
                unit(q);
                al = std::max(al, angle(w, q));
            }
            return al;
        };
        for (int row = 0; row < n; ++row)
            for (int col = 0; col < n; ++col) {
                const size_t t = (static_cast<size_t>(f) * n + row) * n + col;
                alpha[t] = cone(-1.0 + 2.0 * col / n, -1.0 + 2.0 * (col + 1) / n, -1.0 + 2.0 * row / n,
                                -1.0 + 2.0 * (row + 1) / n, &mc->w[3 * t]);
                mc->ca[t] = std::cos(alpha[t]);
                mc->sa[t] = std::sin(alpha[t]);
            }
        auto block = [&](int r0, int c0, int size) {
            MaskCones::Block bl;
            bl.face = f;
            bl.r0 = r0;
            bl.c0 = c0;
            bl.r1 = std::min(n, r0 + size);
            bl.c1 = std::min(n, c0 + size);
            bl.reach = cone(-1.0 + 2.0 * bl.c0 / n, -1.0 + 2.0 * bl.c1 / n, -1.0 + 2.0 * bl.r0 / n,
                            -1.0 + 2.0 * bl.r1 / n, bl.w);
            double amax = 0.0;
            for (int row = bl.r0; row < bl.r1; ++row)
                for (int col = bl.c0; col < bl.c1; ++col)
                    amax = std::max(amax, alpha[(static_cast<size_t>(f) * n + row) * n + col]);
            bl.reach += amax;
            bl.cr = std::cos(bl.reach);
            bl.sr = std::sin(bl.reach);
            return bl;
        };
        for (int r0 = 0; r0 < n; r0 += kMaskBlock)
            for (int c0 = 0; c0 < n; c0 += kMaskBlock) {
                mc->blocks.push_back(block(r0, c0, kMaskBlock));
                const MaskCones::Block &bl = mc->blocks.back();
                std::vector<MaskCones::Block> sub;
                for (int r = bl.r0; r < bl.r1; r += kMaskSubBlock)
                    for (int c = bl.c0; c < bl.c1; c += kMaskSubBlock) sub.push_back(block(r, c, kMaskSubBlock));
                mc->subs.push_back(std::move(sub));
            }
    }
    slot = std::move(mc);
    return *slot;
}

// Build the device blob: [spheres][sphere meta][boxes][materials][lights]
// [light x material products]; every section 16-B aligned.
// Shadow direction masks (rt_internal.h, kMaskMaxSpheres): float64 geometry.
// A shadow ray from shaded point p runs from p + 0.01 n towards the light L
// (:808-809): within 0.01 of the segment [L, p], i.e. of the ray from L in
// the direction of p - L. Sphere s (centre c, radius r, d = |c - L|) can
// block it only if that ray passes within rp = r + 0.021 + 1e-3 d of c (the
// ShadowCone inflation): its direction within asin(rp / d) of (c - L) / d,
// or any direction when d <= rp. A texel is the spherical image of a square
// of the cube face; it lies inside the cone around its centre direction
// whose half-angle is the largest angle to its four corners (a cone narrower
// than 90 degrees is convex, so holding the corners it holds the square).
// Spheres are tested texel by texel only in the blocks whose reach their
// cone comes within (a texel's centre lies in its block's cone, so every
// texel the texel test accepts lies in an accepted block): the bits set are
// those of the texel-by-texel test alone.
static void build_direction_masks(const std::vector<SphereRec> &sph, const std::vector<SphereMeta> &smeta,
                           const rt_light *lights, const std::vector<LightRec> &lrec, int n,
                           std::vector<uint64_t> &out, int words = 1) {
    const int n_lights = static_cast<int>(lrec.size());
    const MaskCones &mc = mask_cones(n);
    out.clear();
    for (int j = 0; j < n_lights; ++j) {
        if (lrec[j].dead != 0.0f) continue;
        // each sphere's cone from this light: axis, half-angle (or everywhere);
        // the texel test angle(w, axis) <= alpha + half + 1e-3 is evaluated on
        // cosines, dot(w, axis) >= cos(alpha + half + 1e-3) (both angles are
        // below pi; acos is decreasing), with cos / sin of half + 1e-3 per
        // sphere and of alpha per texel: no inverse cosine per (texel, sphere)
        std::vector<double> ax(3 * sph.size()), half(sph.size()), ch(sph.size()), sh(sph.size());
        std::vector<char> every(sph.size(), 0);
        for (size_t s = 0; s < sph.size(); ++s) {
            double v[3] = {double(sph[s].cx) - lights[j].position[0], double(sph[s].cy) - lights[j].position[1],
                           double(sph[s].cz) - lights[j].position[2]};
            const double d = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            const double rp = double(smeta[s].radius) + 0.021 + 1e-3 * d;
            if (!(std::isfinite(d) && std::isfinite(rp)) || d <= rp) {
                every[s] = 1;
                continue;
            }
            for (int k = 0; k < 3; ++k) ax[3 * s + k] = v[k] / d;
            half[s] = std::asin(std::min(1.0, rp / d));
            ch[s] = std::cos(half[s] + 1e-3);
            sh[s] = std::sin(half[s] + 1e-3);
        }
        const size_t base = out.size();
        out.resize(base + static_cast<size_t>(6) * n * n * words, 0u);
        for (const MaskCones::Block &bl : mc.blocks)
            for (size_t s = 0; s < sph.size(); ++s) {
                if (!every[s]) {
                    // cos(reach + half + 1e-3), less a margin for rounding
                    const double lim = bl.cr * ch[s] - bl.sr * sh[s] - 1e-9;
                    const double c = bl.w[0] * ax[3 * s] + bl.w[1] * ax[3 * s + 1] + bl.w[2] * ax[3 * s + 2];
                    if (bl.reach + half[s] + 1e-3 < 3.141592653589793 && c < lim) continue;
                }
                for (int row = bl.r0; row < bl.r1; ++row)
                    for (int col = bl.c0; col < bl.c1; ++col) {
                        const size_t t = (static_cast<size_t>(bl.face) * n + row) * n + col;
                        const double *w = &mc.w[3 * t];
                        // cos(alpha + half + 1e-3), less 1e-12 for rounding (far below the 1e-3 rad margin)
                        const double lim = mc.ca[t] * ch[s] - mc.sa[t] * sh[s] - 1e-12;
                        const double c = w[0] * ax[3 * s] + w[1] * ax[3 * s + 1] + w[2] * ax[3 * s + 2];
                        if (every[s] || c >= lim) out[base + t * words + s / 64] |= uint64_t{1} << (s % 64);
                    }
            }
    }
}

// Origin-sphere candidate lists of the secondary rays (rt_internal.h,
// kOListSlots): float64 geometry, the spheres in their final (BVH) slot order.
// Every reflection or refraction ray that leaves sphere s starts within
// 0.001 of its surface (:1010-1023: p +- 0.001 n), so inside the ball
// B(c_s, r_s + 0.001); it can hit sphere j only in a direction within
// asin(rin / d) of (c_j - c_s) / d, rin = r_j + r_s + 0.001 + margins, d =
// |c_j - c_s| (any direction when d <= rin) — the shadow masks' cone test
// with the origin ball folded into the target, texel by texel in the blocks
// the sphere's cone reaches. The margins (1e-3 + 1e-4 of the coordinates'
// magnitude, plus 1e-3 rad) dwarf the float32 error of the kernel's hit
// points, offsets and approximate texel lookup. A candidate's bound is a
// lower bound of the ray parameter of any hit on it from that ball: the
// distance between the balls, shrunk by the same margins and by 1e-5 for
// ray directions that are unit vectors only up to rounding; stored rounded
// down in 1/256 units, so a lane that stops on `best t < bound` drops only
// spheres whose hit would lie strictly farther (no tie can be lost).
static void origin_lists_range(const std::vector<SphereRec> &sph, const std::vector<SphereMeta> &smeta, int n,
                               std::vector<uint8_t> &out, size_t s_begin, size_t s_end) {
    const size_t ns = sph.size();
    const MaskCones &mc = mask_cones(n);
    const size_t texels = static_cast<size_t>(6) * n * n;
    std::vector<double> ax(3 * ns), ch(ns), sh(ns), lb(ns), reach(ns);
    std::vector<char> every(ns);
    // the spheres' cone data in list order (o*), a block's candidates (k*) and
    // a sub-block's (s*), contiguous
    std::vector<int> order(ns), kq(ns), sq(ns);
    std::vector<double> ox(ns), oy(ns), oz(ns), oc(ns), osn(ns), orc(ns);
    std::vector<double> kx(ns), ky(ns), kz(ns), kc(ns), ksn(ns), kr(ns);
    std::vector<double> sx(ns), sy(ns), sz(ns), sc(ns), ss(ns);
    std::vector<char> oe(ns), ke(ns), se(ns), keep(ns), hit(ns);
    std::vector<std::pair<double, int>> list;  // one texel's candidates: (bound, slot)
    auto quant = [](double x) -> uint16_t {  // rounded down, saturating (a smaller bound stays a bound)
        if (!(x > 0.0)) return 0;
        const double q = std::floor(x / static_cast<double>(kOListBoundUnit));
        return static_cast<uint16_t>(std::min(q, 65535.0));
    };
    for (size_t s = s_begin; s < s_end; ++s) {
        const double cs[3] = {sph[s].cx, sph[s].cy, sph[s].cz};
        const double rs = smeta[s].radius;
        const double ms = std::sqrt(cs[0] * cs[0] + cs[1] * cs[1] + cs[2] * cs[2]);
        for (size_t j = 0; j < ns; ++j) {
            const double v[3] = {double(sph[j].cx) - cs[0], double(sph[j].cy) - cs[1], double(sph[j].cz) - cs[2]};
            const double d = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            const double cj = std::sqrt(double(sph[j].cx) * sph[j].cx + double(sph[j].cy) * sph[j].cy +
                                        double(sph[j].cz) * sph[j].cz);
            const double rj = smeta[j].radius;
            const double margin = 1e-3 + 1e-4 * (d + ms + cj + rs + rj);
            const double rin = rj + rs + 0.001 + margin;
            const bool ok = std::isfinite(d) && std::isfinite(rin) && std::isfinite(margin);
            lb[j] = j == s ? -1.0 : (ok ? std::max(0.0, (d - rj - rs - 0.001 - 2.0 * margin) * (1.0 - 1e-5)) : 0.0);
            every[j] = !ok || d <= rin;
            if (every[j]) continue;
            for (int k = 0; k < 3; ++k) ax[3 * j + k] = v[k] / d;
            const double half = std::asin(std::min(1.0, rin / d));
            reach[j] = half + 1e-3;
            ch[j] = std::cos(reach[j]);
            sh[j] = std::sin(reach[j]);
        }
        // The spheres in list order, (bound, slot) ascending: every list
        // below is built by walking them in this order, so it comes out
        // sorted. A (sub-)block is skipped for sphere j when j's cone misses
        // the block's reach (every texel the texel test accepts lies in an
        // accepted block and sub-block); the tests run over contiguous
        // arrays of the candidates' cone data.
        for (size_t j = 0; j < ns; ++j) order[j] = static_cast<int>(j);
        std::sort(order.begin(), order.end(), [&](int x, int y) { return lb[x] < lb[y] || (lb[x] == lb[y] && x < y); });
        for (size_t q = 0; q < ns; ++q) {
            const int j = order[q];
            ox[q] = ax[3 * j];
            oy[q] = ax[3 * j + 1];
            oz[q] = ax[3 * j + 2];
            oc[q] = ch[j];
            osn[q] = sh[j];
            orc[q] = reach[j];
            oe[q] = every[j];
        }
        // reach test of a block against candidates [0, m) of (x, y, z, c, sn, r, e): keep[] = 1 if it may reach
        auto reach_test = [](const MaskCones::Block &bl, size_t m, const double *x, const double *y, const double *z,
                             const double *c, const double *sn, const double *r, const char *e, char *keep) {
            for (size_t q = 0; q < m; ++q)
                keep[q] = e[q] | static_cast<char>(bl.reach + r[q] >= 3.141592653589793) |
                          static_cast<char>(bl.w[0] * x[q] + bl.w[1] * y[q] + bl.w[2] * z[q] >=
                                            bl.cr * c[q] - bl.sr * sn[q] - 1e-9);
        };
        for (size_t k = 0; k < mc.blocks.size(); ++k) {
            reach_test(mc.blocks[k], ns, ox.data(), oy.data(), oz.data(), oc.data(), osn.data(), orc.data(), oe.data(),
                       keep.data());
            size_t mk = 0;  // the block's candidates, in list order
            for (size_t q = 0; q < ns; ++q)
                if (keep[q]) {
                    kq[mk] = static_cast<int>(q);
                    kx[mk] = ox[q];
                    ky[mk] = oy[q];
                    kz[mk] = oz[q];
                    kc[mk] = oc[q];
                    ksn[mk] = osn[q];
                    kr[mk] = orc[q];
                    ke[mk] = oe[q];
                    ++mk;
                }
            for (const MaskCones::Block &sb : mc.subs[k]) {
                reach_test(sb, mk, kx.data(), ky.data(), kz.data(), kc.data(), ksn.data(), kr.data(), ke.data(),
                           keep.data());
                size_t m = 0;  // the sub-block's candidates, in list order
                for (size_t q = 0; q < mk; ++q)
                    if (keep[q]) {
                        sq[m] = kq[q];
                        sx[m] = kx[q];
                        sy[m] = ky[q];
                        sz[m] = kz[q];
                        sc[m] = kc[q];
                        ss[m] = ksn[q];
                        se[m] = ke[q];
                        ++m;
                    }
                for (int row = sb.r0; row < sb.r1; ++row)
                    for (int col = sb.c0; col < sb.c1; ++col) {
                        const size_t t = (static_cast<size_t>(sb.face) * n + row) * n + col;
                        const double w0 = mc.w[3 * t], w1 = mc.w[3 * t + 1], w2 = mc.w[3 * t + 2];
                        const double ca = mc.ca[t], sa = mc.sa[t];
                        // (reach < pi / 2 + 1e-3 and a texel's half-angle is small: the summed
                        // angle stays below pi, where the cosine test is exact)
                        for (size_t q = 0; q < m; ++q)
                            hit[q] = se[q] | static_cast<char>(w0 * sx[q] + w1 * sy[q] + w2 * sz[q] >=
                                                               ca * sc[q] - sa * ss[q] - 1e-12);
                        list.clear();  // (list order already)
                        for (size_t q = 0; q < m; ++q)
                            if (hit[q]) list.push_back({lb[order[sq[q]]], order[sq[q]]});
                        uint8_t *rec = out.data() + (s * texels + t) * kOListRecordBytes;
                        const size_t cnt = list.size();
                        rec[0] = static_cast<uint8_t>(std::min<size_t>(cnt, 255));
                        for (size_t i = 0; i < cnt && i < static_cast<size_t>(kOListSlots); ++i)
                            rec[1 + i] = static_cast<uint8_t>(list[i].second);
                        const uint16_t bnd[3] = {cnt > 8 ? quant(list[8].first) : uint16_t{65535},
                                                 cnt > 16 ? quant(list[16].first) : uint16_t{65535},
                                                 cnt > static_cast<size_t>(kOListSlots)
                                                     ? quant(list[kOListSlots].first)
                                                     : uint16_t{65535}};
                        std::memcpy(rec + 1 + kOListSlots, bnd, sizeof bnd);
                    }
            }
        }
    }
}

// The lists of all spheres: independent per origin sphere, built on up to 16
// host threads (256 spheres: about 130 ms of host work on one thread). A
// thread that cannot be started (std::system_error, e.g. a process thread
// limit) leaves its range to the calling thread: nothing throws out of here.
static void build_origin_lists(const std::vector<SphereRec> &sph, const std::vector<SphereMeta> &smeta, int n,
                               std::vector<uint8_t> &out) {
    const size_t ns = sph.size();
    out.assign(ns * static_cast<size_t>(6) * n * n * kOListRecordBytes, 0);
    (void)mask_cones(n);  // (built once, before the workers share it)
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t n_thr = std::min<size_t>({16, hw, (ns + 15) / 16});
    if (n_thr <= 1) {
        origin_lists_range(sph, smeta, n, out, 0, ns);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(n_thr);
    const size_t per = (ns + n_thr - 1) / n_thr;
    size_t started = 0;  // [0, started) is covered by the running workers
    for (size_t k = 0; k < n_thr; ++k) {
        const size_t a = k * per, b = std::min(ns, a + per);
        if (a >= b) break;
        try {
            pool.emplace_back(origin_lists_range, std::cref(sph), std::cref(smeta), n, std::ref(out), a, b);
        } catch (const std::system_error &) {
            break;
        }
        started = b;
    }
    if (started < ns) origin_lists_range(sph, smeta, n, out, started, ns);
    for (std::thread &t : pool) t.join();
}

// The origin-sphere lists of a built scene, from its host blob (the sphere
// records the kernel stages): empty unless the scene has
// kOListMinSpheres..256 spheres (DeviceScene::olist_eligible).
int build_origin_lists_for(const std::vector<float4> &host, const DeviceScene &ds, std::vector<uint8_t> &olist) {
    olist.clear();
    if (!ds.olist_eligible) return RT_OK;
    const size_t ns = static_cast<size_t>(ds.n_spheres);
    if (host.size() * sizeof(float4) < (static_cast<size_t>(ds.off_smeta) * 16 + ns * sizeof(SphereMeta)) ||
        host.size() * sizeof(float4) < (static_cast<size_t>(ds.off_spheres) * 16 + ns * sizeof(SphereRec))) {
        set_error("origin lists: the scene's host copy is incomplete");
        return RT_ERR_INVALID;
    }
    std::vector<SphereRec> sph(ns);
    std::vector<SphereMeta> smeta(ns);
    const char *base = reinterpret_cast<const char *>(host.data());
    std::memcpy(sph.data(), base + static_cast<size_t>(ds.off_spheres) * 16, ns * sizeof(SphereRec));
    std::memcpy(smeta.data(), base + static_cast<size_t>(ds.off_smeta) * 16, ns * sizeof(SphereMeta));
    try {
        build_origin_lists(sph, smeta, kOListTexels, olist);
    } catch (const std::bad_alloc &) {
        olist.clear();
        set_error("origin lists: out of memory");
        return RT_ERR_NOMEM;
    }
    return RT_OK;
}

int build_scene(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats, const rt_light *lights,
                int n_lights, std::vector<float4> &blob, DeviceScene &ds, bool with_origin_lists) {
    std::vector<SphereRec> sph;
    std::vector<SphereMeta> smeta;
    std::vector<BoxRec> boxes;
    for (int i = 0; i < n_objs; ++i) {
        const rt_object &o = objs[i];
        const int kind = object_kind(o);
        if (kind == 0) continue;
        if (o.material < 0 || o.material >= n_mats) {
            set_error("rt_scene_create: object " + std::to_string(i) + " has material index out of range");
            return RT_ERR_INVALID;
        }
        if (kind == 2) {
            sph.push_back({o.position[0], o.position[1], o.position[2], o.radius * o.radius});
            // |radius| for the culling bounds (a negative radius other than -1
            // is a sphere of radius |r|: the test only sees r*r, :588)
            smeta.push_back({i, o.material, std::fabs(o.radius), 0});
        } else {
            // the transforms as the reference's GL evaluates them per ray (rt_camera.cpp)
            float L[16], W[16], N[9];
            reference_box_transforms(o.position, o.angles, L, W, N);
            BoxRec b{};
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) {  // stored row-major
                    b.w2l[r * 4 + c] = W[c * 4 + r];
                    b.l2w[r * 4 + c] = L[c * 4 + r];
                }
            // the normal matrix transpose(inverse(mat3(L))), stored row-major
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) b.nrm[r * 3 + c] = N[c * 3 + r];
            std::memcpy(b.mins, o.box_mins, 12);
            std::memcpy(b.maxs, o.box_maxs, 12);
            b.obj_index = i;
            b.material = o.material;
            for (int r = 0; r < 3; ++r) b.w2l_w0[r] = b.w2l[r * 4 + 3] * 0.0f;  // the kernel adds it as is
            b.translate_only = 1;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    if (b.w2l[r * 4 + c] != (r == c ? 1.0f : 0.0f)) b.translate_only = 0;
            // Lights strictly inside the box by a margin (float64): a shadow
            // segment that starts inside the box then ends inside it too (its
            // end is the light + 0.01 n, :808-809), so the box cannot occlude.
            const M4 Wd = inverse(transform(o.position, o.angles));  // culling only (float64)
            for (int j = 0; j < n_lights && j < 32; ++j) {
                double lp[3];
                bool in = true;
                for (int r = 0; r < 3; ++r) {
                    lp[r] = Wd.m[0][r] * lights[j].position[0] + Wd.m[1][r] * lights[j].position[1] +
                            Wd.m[2][r] * lights[j].position[2] + Wd.m[3][r];
                    const double m = 0.05 + 1e-4 * (std::fabs(o.box_mins[r]) + std::fabs(o.box_maxs[r]) +
                                                    std::fabs(lp[r]));
                    in = in && std::isfinite(lp[r]) && o.box_mins[r] + m < lp[r] && lp[r] < o.box_maxs[r] - m;
                }
                if (in) b.light_inside |= 1u << j;
            }
            boxes.push_back(b);
        }
    }
    double extent = 0.0;  // |coordinate| bound of the finite objects (BVH margins)
    for (int i = 0; i < n_objs; ++i) {
        const rt_object &o = objs[i];
        double e = std::sqrt(static_cast<double>(o.position[0]) * o.position[0] +
                             static_cast<double>(o.position[1]) * o.position[1] +
                             static_cast<double>(o.position[2]) * o.position[2]);
        double corner = std::fabs(static_cast<double>(o.radius));
        for (int a = 0; a < 3; ++a)
            corner = std::max(corner, std::max(std::fabs(static_cast<double>(o.box_mins[a])),
                                               std::fabs(static_cast<double>(o.box_maxs[a]))));
        e += corner * std::sqrt(3.0);
        if (std::isfinite(e)) extent = std::max(extent, e);
    }
    std::vector<BvhNode> bvh;
    std::vector<uint32_t> blink;
    build_bvh(sph, smeta, bvh, blink, extent);
    std::vector<MatRec> mrec(n_mats);
    std::vector<LightMatRec> lm(static_cast<size_t>(n_mats) * n_lights);
    for (int m = 0; m < n_mats; ++m) {
        MatRec &r = mrec[m];
        for (int k = 0; k < 4; ++k) {
            float acc = 0.0f;  // ambient = vec4(0.0); ambient += La * Ma (:793, :801)
            for (int j = 0; j < n_lights; ++j) acc = acc + lights[j].ambient[k] * mats[m].ambient[k];
            r.amb_sum[k] = acc;
            r.emissive[k] = mats[m].emissive[k];
        }
        r.shininess = mats[m].shininess;
        r.reflectivity = mats[m].reflectivity;
        r.transparency = mats[m].transparency;
        r.refraction_index = mats[m].refraction_index;
        r.eta_in = 1.0f / r.refraction_index;  // the ratio of a ray entering (IEEE division, as the kernel's)
        r.eta_out = 1.0f / r.eta_in;           // and of one leaving the object
        // tame: every product finite and shininess in (0, 1e6): then the
        // diffuse factor max(cos, 0) <= 1 + 2^-20 and pow(max(cos, 0),
        // shininess) are finite (pow is skipped for a zero base; its exp2
        // argument stays below 128 for such bases and exponents) and a light
        // whose products are zero, or whose factor is zero, adds only +-0 to
        // the sums (which start at +0 and so are never -0): its shadow ray
        // cannot change the colour.
        bool tame = mats[m].shininess > 0.0f && mats[m].shininess < 1e6f;
        for (int j = 0; j < n_lights; ++j) {
            LightMatRec &q = lm[m * n_lights + j];
            for (int k = 0; k < 4; ++k) {
                q.ld_md[k] = lights[j].diffuse[k] * mats[m].diffuse[k];   // :830
                q.ls_ms[k] = lights[j].specular[k] * mats[m].specular[k];  // :832
                q.d_nz |= q.ld_md[k] != 0.0f;
                q.s_nz |= q.ls_ms[k] != 0.0f;
                tame = tame && std::isfinite(q.ld_md[k]) && std::isfinite(q.ls_ms[k]);
            }
        }
        for (int j = 0; j < n_lights; ++j) lm[m * n_lights + j].always = tame ? 0 : 1;
    }
    // Shadow culling cones of every (light, sphere) pair (float64; culling
    // only, the margins dwarf the float32 rounding of the stored values).
    std::vector<ShadowCone> cones(static_cast<size_t>(n_lights) * sph.size());
    for (int j = 0; j < n_lights; ++j)
        for (size_t s = 0; s < sph.size(); ++s) {
            ShadowCone &c = cones[j * sph.size() + s];
            const double v[3] = {double(sph[s].cx) - lights[j].position[0], double(sph[s].cy) - lights[j].position[1],
                                 double(sph[s].cz) - lights[j].position[2]};
            const double d = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            const double rp = double(smeta[s].radius) + 0.021 + 1e-3 * d;
            if (!(std::isfinite(d) && std::isfinite(rp)) || d <= rp) {
                c.near = 1.0f;  // always a candidate
                continue;
            }
            for (int r = 0; r < 3; ++r) c.v[r] = static_cast<float>(v[r] / d);
            c.far = static_cast<float>(d - rp);
            const double sp = rp / d;
            c.sph = static_cast<float>(sp);
            c.cph = static_cast<float>(std::sqrt(std::max(0.0, 1.0 - sp * sp)));
        }
    // A light with zero diffuse and specular colour (the reference's ambient
    // light, :202-207) adds +-0 to the sums for every finite material with
    // shininess >= 0 (pow then stays finite), so lit and shadowed agree and
    // the kernel may skip it; its ambient term is in amb_sum.
    bool materials_tame = true;
    for (int m = 0; m < n_mats; ++m) {
        // (shininess below 1e6 keeps pow's exp2 argument below 128: finite)
        materials_tame = materials_tame && mats[m].shininess >= 0.0f && mats[m].shininess < 1e6f;
        for (int k = 0; k < 4; ++k)
            materials_tame = materials_tame && std::isfinite(mats[m].diffuse[k]) && std::isfinite(mats[m].specular[k]);
    }
    std::vector<LightRec> lrec(n_lights);
    for (int j = 0; j < n_lights; ++j) {
        std::memcpy(lrec[j].pos, lights[j].position, 12);
        bool zero = true;
        for (int k = 0; k < 4; ++k) zero = zero && lights[j].diffuse[k] == 0.0f && lights[j].specular[k] == 0.0f;
        lrec[j].dead = (zero && materials_tame) ? 1.0f : 0.0f;
    }
    auto units = [](size_t bytes) { return static_cast<int32_t>((bytes + 15) / 16); };
    int32_t off = 0;
    ds.off_spheres = off; off += units(sph.size() * sizeof(SphereRec));
    ds.off_smeta = off;   off += units(smeta.size() * sizeof(SphereMeta));
    ds.off_boxes = off;   off += units(boxes.size() * sizeof(BoxRec));
    ds.off_mats = off;    off += units(mrec.size() * sizeof(MatRec));
    ds.off_lights = off;  off += units(lrec.size() * sizeof(LightRec));
    ds.off_lightmat = off; off += units(lm.size() * sizeof(LightMatRec));
    // Round 6: in a scene of several boxes (chosen by the object kinds alone,
    // as the mask bits), per (box, light) the face plane of the box (in the
    // float32 transform the kernel uses) with the light farthest beyond it:
    // a shadow segment whose start lies beyond that plane too cannot be
    // occluded by the box (both of its ends beyond the plane of a face; the
    // exact slab test then sees that axis' entry at t > 1 or a miss). Stored
    // as (n, w) with the margin m folded into w (a start counts as beyond
    // when n . start + w > 0), m = 1e-3 + 1e-5 (scene extent + |w|), far
    // above the float32 rounding of n . start and of the kernel's transform;
    // kept only if the light lies beyond by more than 0.01 (the segment ends
    // at L + 0.01 n, :808-809) + 2 m; else w = -inf (never beyond).
    std::vector<float4> bplane;
    ds.off_bplane = -1;
    if (boxes.size() >= 2) {
        bool finite = true;  // (a non-finite object: no planes; shaded points are bounded by `extent` otherwise)
        for (int i = 0; i < n_objs; ++i)
            for (int k = 0; k < 3; ++k)
                finite = finite && std::isfinite(objs[i].position[k]) && std::isfinite(objs[i].box_mins[k]) &&
                         std::isfinite(objs[i].box_maxs[k]) && std::isfinite(objs[i].radius);
        bplane.assign(boxes.size() * static_cast<size_t>(n_lights), float4{0.0f, 0.0f, 0.0f, -HUGE_VALF});
        for (size_t b = 0; b < boxes.size() && finite; ++b) {
            const BoxRec &B = boxes[b];
            for (int j = 0; j < n_lights; ++j) {
                const double L[3] = {lights[j].position[0], lights[j].position[1], lights[j].position[2]};
                double best = -HUGE_VAL, bn[3] = {0, 0, 0}, bw = 0, bm = 0;
                for (int a = 0; a < 3; ++a)
                    for (int sgn = -1; sgn <= 1; sgn += 2) {
                        const double face = sgn > 0 ? B.maxs[a] : B.mins[a];
                        const double r[4] = {B.w2l[4 * a], B.w2l[4 * a + 1], B.w2l[4 * a + 2], B.w2l[4 * a + 3]};
                        const double sl = sgn * (r[0] * L[0] + r[1] * L[1] + r[2] * L[2] + r[3] - face);
                        if (sl > best) {
                            best = sl;
                            for (int k = 0; k < 3; ++k) bn[k] = sgn * r[k];
                            bw = sgn * (r[3] - face);
                            bm = 1e-3 + 1e-5 * (extent + std::fabs(r[3]) + std::fabs(face));
                        }
                    }
                if (std::isfinite(best) && std::isfinite(bw) && best > 0.01 + 2.0 * bm)
                    bplane[b * n_lights + j] = float4{static_cast<float>(bn[0]), static_cast<float>(bn[1]),
                                                      static_cast<float>(bn[2]), static_cast<float>(bw - bm)};
            }
        }
        ds.off_bplane = off;
        off += units(bplane.size() * sizeof(float4));
    }
    ds.off_bvh = off;     off += units(bvh.size() * sizeof(BvhNode));
    ds.off_blink = off;   off += units(blink.size() * sizeof(uint32_t));
    // The cone table rides in LDS only while the work-group's LDS stays small
    // enough for full occupancy (config 4's 256 spheres x 3 lights would add
    // 24 KB and cut the resident work-groups per CU); without it the kernel
    // derives the cones per wave (off_cone = -1).
    const size_t per_frame = sph.size() * 32 + boxes.size() * 16;
    // Direction masks replace the cone table where they fit (finest texels first).
    int n_live = 0;
    for (int j = 0; j < n_lights; ++j) n_live += lrec[j].dead == 0.0f;
    std::vector<uint64_t> dmask;
    ds.off_dmask = -1;
    ds.dmask_n = 0;
    // Round 6: in a scene of several boxes the boxes get mask bits too (bit
    // n_spheres + b), from their bounding spheres. A box that can occlude a
    // shadow segment holds a point of it, and so does its bounding sphere: the
    // spheres' cone test is conservative for it. The sphere's radius carries
    // 1e-3 relative + 1e-3 (1 + |centre|) of margin over the float64 half
    // diagonal, far above the float32 transforms' error. The choice depends
    // on the object kinds alone (the blob layout rt_render_batch_scenes
    // requires to be shared by the frames of an animated scene): a one-box
    // scene — the room of configs 2-5 — keeps its box's shortcuts instead.
    const bool box_bits = boxes.size() >= 2;
    const size_t mask_bits = sph.size() + (box_bits ? boxes.size() : 0);
    ds.dmask_box = 0;
    if (!sph.empty() && mask_bits <= static_cast<size_t>(kMaskMaxSpheres) && n_live > 0) {
        ds.dmask_bytes = mask_bits <= 16 ? 2 : (mask_bits <= 32 ? 4 : 8);
#ifndef RT_DMASK_MAXN
#define RT_DMASK_MAXN 12
#endif
        for (int n : {32, 24, 16, 12, 8}) {
            if (n > RT_DMASK_MAXN) continue;
            const size_t bytes = static_cast<size_t>(n_live) * 6 * n * n * ds.dmask_bytes;
            if ((static_cast<size_t>(off) + units(bytes)) * 16 + per_frame <= kMaskLdsBudget) {
                ds.dmask_n = n;
                break;
            }
        }
    }
    std::vector<char> dmask_bytes;
    if (ds.dmask_n > 0) {
        if (box_bits) {
            std::vector<SphereRec> bsph(sph);
            std::vector<SphereMeta> bmeta(smeta);
            for (int i = 0; i < n_objs; ++i) {
                const rt_object &o = objs[i];
                if (object_kind(o) != 1) continue;
                const M4 T = transform(o.position, o.angles);
                double c[3], h2 = 0.0;
                for (int r = 0; r < 3; ++r) {
                    const double lc = 0.5 * (double(o.box_mins[r]) + double(o.box_maxs[r]));
                    const double e = 0.5 * (double(o.box_maxs[r]) - double(o.box_mins[r]));
                    h2 += e * e;
                    c[r] = lc;
                }
                double w[3];
                for (int r = 0; r < 3; ++r) w[r] = T.m[0][r] * c[0] + T.m[1][r] * c[1] + T.m[2][r] * c[2] + T.m[3][r];
                const double wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                const double rad = std::sqrt(h2) * 1.001 + 1e-3 * (1.0 + wl);
                bsph.push_back({static_cast<float>(w[0]), static_cast<float>(w[1]), static_cast<float>(w[2]), 0.0f});
                // (a non-finite box: a non-finite radius, the bit set everywhere)
                bmeta.push_back({i, o.material, std::isfinite(rad) ? static_cast<float>(rad * (1.0 + 1e-6))
                                                                   : HUGE_VALF, 0});
            }
            build_direction_masks(bsph, bmeta, lights, lrec, ds.dmask_n, dmask);
            ds.dmask_box = 1;
        } else {
            build_direction_masks(sph, smeta, lights, lrec, ds.dmask_n, dmask);
        }
        ds.off_dmask = off;
        dmask_bytes.resize(dmask.size() * ds.dmask_bytes);
        for (size_t i = 0; i < dmask.size(); ++i)  // little-endian: the low bytes of each mask
            std::memcpy(dmask_bytes.data() + i * ds.dmask_bytes, &dmask[i], ds.dmask_bytes);
        off += units(dmask_bytes.size());
        cones.clear();
    }
    const size_t with_cones = (static_cast<size_t>(off) + units(cones.size() * sizeof(ShadowCone))) * 16 + per_frame;
    if (ds.dmask_n == 0 && with_cones <= kConeLdsBudget) {
        ds.off_cone = off;
        off += units(cones.size() * sizeof(ShadowCone));
    } else {
        ds.off_cone = -1;
        cones.clear();
    }
    ds.n_bvh = static_cast<int32_t>(bvh.size());
    ds.blob_units = off;  // the part every work-group stages into LDS
    // Scenes above RT_GMASK_FROM spheres: wide direction masks (kGMaskMaxSpheres),
    // also beside the LDS masks (depth 0-1 keep those; depth >= 2 reads these),
    // kept in the device blob past the staged part and read through L2.
    std::vector<uint64_t> gmask;
    std::vector<uint8_t> glist;
    ds.off_gmask = -1;
    ds.off_glist = -1;
    ds.gmask_words = 0;
#ifndef RT_GMASK_FROM
#define RT_GMASK_FROM 32  // wide masks above this many spheres at depth >= 2 (tools/ablate.sh flags; config 3, 64 spheres: 1.15 -> 1.11 ms)
#endif
    if (sph.size() > static_cast<size_t>(RT_GMASK_FROM) &&
        sph.size() <= static_cast<size_t>(kGMaskMaxSpheres) && n_live > 0) {
        ds.gmask_words = static_cast<int32_t>((sph.size() + 63) / 64);
        build_direction_masks(sph, smeta, lights, lrec, kGMaskTexels, gmask, ds.gmask_words);
        ds.off_gmask = off;
        off += units(gmask.size() * 8);
        // the candidate lists of the same texels (rt_internal.h kGListMax)
        const size_t n_texels = gmask.size() / static_cast<size_t>(ds.gmask_words);
        glist.assign(n_texels * 16, 0);
        // each live light's order of the spheres: largest angular size seen
        // from the light first (a light inside a sphere's inflated bound, or
        // a non-finite sphere, first of all), so a shadowed query meets its
        // occluder early and its any-hit walk ends (the result is
        // order-independent). CPU model (tools/model/shadow_model.py): the
        // wave's candidate passes per shadow call 2.34 -> 1.47 on config 4,
        // 0.95 -> 0.73 on config 3.
        std::vector<int> live;
        for (int j = 0; j < n_lights; ++j)
            if (lrec[j].dead == 0.0f) live.push_back(j);
        std::vector<std::vector<int>> rank_of(live.size(), std::vector<int>(sph.size()));
        for (size_t k = 0; k < live.size(); ++k) {
            const rt_light &L = lights[live[k]];
            std::vector<double> key(sph.size());
            for (size_t q = 0; q < sph.size(); ++q) {
                const double v[3] = {double(sph[q].cx) - L.position[0], double(sph[q].cy) - L.position[1],
                                     double(sph[q].cz) - L.position[2]};
                const double d = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                const double r = double(smeta[q].radius);
                key[q] = (std::isfinite(d) && std::isfinite(r) && d > r + 0.021 + 1e-3 * d) ? r / d : HUGE_VAL;
            }
            std::vector<int> order(sph.size());
            for (size_t q = 0; q < sph.size(); ++q) order[q] = static_cast<int>(q);
            std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] > key[y]; });
            for (size_t q = 0; q < order.size(); ++q) rank_of[k][order[q]] = static_cast<int>(q);
        }
        const size_t per_light = n_texels / (live.empty() ? 1 : live.size());
        for (size_t t = 0; t < n_texels; ++t) {
            uint8_t *rec = glist.data() + t * 16;
            const std::vector<int> &rk = rank_of[t / per_light];
            int n = 0;
            // the same truncation as the kernel's word walk (occluded: the
            // last word masked to the `rest` = ns - 64 w live slots)
            const int ns = static_cast<int>(sph.size());
            for (int w = 0; w < ds.gmask_words; ++w) {
                uint64_t bits = gmask[t * ds.gmask_words + w];
                const int rest = ns - 64 * w;
                if (rest < 64) bits &= (uint64_t{1} << rest) - 1u;
                for (; bits; bits &= bits - 1) {
                    if (n < kGListMax) rec[1 + n] = static_cast<uint8_t>(64 * w + __builtin_ctzll(bits));
                    ++n;
                }
            }
            rec[0] = n <= kGListMax ? static_cast<uint8_t>(n) : static_cast<uint8_t>(kGListOverflow);
            if (n <= kGListMax)
                std::sort(rec + 1, rec + 1 + n, [&](uint8_t x, uint8_t y) { return rk[x] < rk[y]; });
        }
        ds.off_glist = off;
        off += units(glist.size());
    }
    // The secondary rays' origin-sphere candidate lists (rt_internal.h
    // kOListSlots), past the staged part like the wide masks. Only depth >= 2
    // renders read them, and they cost tens of ms of host work and up to
    // 12.6 MB at 256 spheres: a scene is created without them, and the first
    // render that reads them appends them to the device blob
    // (ensure_origin_lists, rt_api.cpp; never to the host copy).
    // with_origin_lists: built here, at the blob's end (the CPU models'
    // rt_debug_scene_blob).
    std::vector<uint8_t> olist;
    ds.off_olist = -1;
    ds.olist_eligible = sph.size() >= static_cast<size_t>(kOListMinSpheres) && sph.size() <= 256;
    if (ds.olist_eligible && with_origin_lists) {
        build_origin_lists(sph, smeta, kOListTexels, olist);
        ds.off_olist = off;
        off += units(olist.size());
    }
    ds.n_spheres = static_cast<int32_t>(sph.size());
    ds.n_boxes = static_cast<int32_t>(boxes.size());
    ds.room = boxes.size() == 1 && boxes[0].translate_only;
    for (int j = 0; j < n_lights && ds.room; ++j)
        if (lrec[j].dead == 0.0f && (j >= 32 || !((boxes[0].light_inside >> j) & 1u))) ds.room = 0;
    ds.n_mats = n_mats;
    ds.n_lights = n_lights;
    blob.assign(static_cast<size_t>(off > 0 ? off : 1), float4{0, 0, 0, 0});
    auto put = [&](int32_t at, const void *src, size_t bytes) {
        if (bytes) std::memcpy(reinterpret_cast<char *>(blob.data()) + static_cast<size_t>(at) * 16, src, bytes);
    };
    put(ds.off_spheres, sph.data(), sph.size() * sizeof(SphereRec));
    put(ds.off_smeta, smeta.data(), smeta.size() * sizeof(SphereMeta));
    put(ds.off_boxes, boxes.data(), boxes.size() * sizeof(BoxRec));
    put(ds.off_mats, mrec.data(), mrec.size() * sizeof(MatRec));
    put(ds.off_lights, lrec.data(), lrec.size() * sizeof(LightRec));
    put(ds.off_lightmat, lm.data(), lm.size() * sizeof(LightMatRec));
    if (ds.off_bplane >= 0) put(ds.off_bplane, bplane.data(), bplane.size() * sizeof(float4));
    put(ds.off_bvh, bvh.data(), bvh.size() * sizeof(BvhNode));
    put(ds.off_blink, blink.data(), blink.size() * sizeof(uint32_t));
    if (ds.off_cone >= 0) put(ds.off_cone, cones.data(), cones.size() * sizeof(ShadowCone));
    if (ds.off_dmask >= 0) put(ds.off_dmask, dmask_bytes.data(), dmask_bytes.size());
    if (ds.off_gmask >= 0) put(ds.off_gmask, gmask.data(), gmask.size() * 8);
    if (ds.off_glist >= 0) put(ds.off_glist, glist.data(), glist.size());
    if (ds.off_olist >= 0) put(ds.off_olist, olist.data(), olist.size());
    return RT_OK;
}

}  // namespace rtamd
