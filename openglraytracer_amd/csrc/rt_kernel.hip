// rt_kernel.hip — the hot path of raytrace_compute.glsl as one CDNA4 kernel.
//
// One ray per lane; a 256-thread work-group renders a 16x16 pixel tile as
// four wave64s of 8x8 pixels each (square wave footprints keep the lanes of a
// wave coherent: they hit the same objects, take the same shading branches and
// tend to exit the shadow loops together). The whole scene (spheres, boxes,
// materials, lights) is staged into LDS once per work-group; every lane then
// reads object records as LDS broadcasts. The frame constants for the camera
// origin (sphere offset / qc terms, box-local camera position) are computed
// once per work-group during staging. Each lane ends with one float4 store:
// a wave writes eight fully-used 128-B lines.
//
// Arithmetic: float32, GLSL operation order, compiled with -ffp-contract=off
// and IEEE division / sqrt so every per-pixel value matches the reference's
// llvmpipe evaluation bit-for-bit given the same frame constants
// (tests/test_gpu_parity.py). Cited line numbers are raytrace_compute.glsl.
//
// Work the reference does that cannot change the result is skipped:
//  * only the closest hit's collision record is built (the reference builds
//    one per intersected object and keeps the nearest, :744-779);
//  * a shadow ray stops at its first occluder with 0 < t < 1 (the reference
//    finds the closest hit and then tests t < 1, :813-816);
//  * a light whose unshadowed diffuse+specular contribution leaves the sums
//    bit-identical (e.g. a light with no diffuse/specular colour, or a
//    surface facing away) casts no shadow ray — lit and shadowed agree.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "rt_internal.h"

namespace rtamd {
namespace {

constexpr int kTile = 16;  // pixels per tile edge
constexpr int kThreads = 256;

struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 muls(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
// dot(vec3) as llvmpipe associates it: x + (y + z)
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
// normalize(v) = v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt (IEEE)
__device__ __forceinline__ v3 normalize(v3 a) { return muls(a, 1.0f / sqrtf(dot(a, a))); }
__device__ __forceinline__ float gmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float gmax(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float comp(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
// reflect(I, N) = I - 2 * dot(N, I) * N
__device__ __forceinline__ v3 reflect(v3 i, v3 n) { return sub(i, muls(n, 2.0f * dot(n, i))); }
// refract(I, N, eta) with k = 1 - eta * (eta * (1 - dot^2)) (Mesa's builtin)
__device__ __forceinline__ v3 refract(v3 i, v3 n, float eta) {
    const float d = dot(n, i);
    const float k = 1.0f - eta * (eta * (1.0f - d * d));
    if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    return sub(muls(i, eta), muls(n, eta * d + sqrtf(k)));
}
// mix(x, y, a) evaluated as x + a * (y - x)
__device__ __forceinline__ v3 mix(v3 x, v3 y, float a) { return add(x, muls(sub(y, x), a)); }

// pow(x, y) = exp2(log2(x) * y) with the polynomial log2 / exp2 the reference's
// GL (llvmpipe) uses for a run-time exponent: even/odd-split polynomials with
// fused multiply-adds (bit-exact, oracle/rt_oracle.c glsl_pow).
__device__ __forceinline__ float poly_log2(float z) {
    const float z2 = z * z;
    float even = __builtin_fmaf(z2, 0.406718052498846252698f, 0.577440339438736392009f);
    even = __builtin_fmaf(z2, even, 2.88539009343309178325f);
    const float odd = __builtin_fmaf(z2, 0.403343858251329912514f, 0.961791550404184197881f);
    return __builtin_fmaf(odd, z, even);
}
__device__ __forceinline__ float poly_exp2(float x) {
    const float x2 = x * x;
    float even = __builtin_fmaf(x2, 0.00898934009049466391101f, 0.240153617044375388211f);
    even = __builtin_fmaf(x2, even, 1.0f);
    float odd = __builtin_fmaf(x2, 0.00187757667519147912699f, 0.0558263180532956664775f);
    odd = __builtin_fmaf(x2, odd, 0.693153073200168932794f);
    return __builtin_fmaf(odd, x, even);
}
__device__ __forceinline__ float glsl_log2(float x) {
    if (x == 0.0f) return -__builtin_inff();
    if (!(x >= 0.0f)) return __builtin_nanf("");
    if (x == __builtin_inff()) return x;
    const uint32_t i = __float_as_uint(x);
    const float e = static_cast<float>(static_cast<int>((i >> 23) & 0xffu) - 127);
    const float mant = __uint_as_float((i & 0x007fffffu) | 0x3f800000u);
    const float y = (mant - 1.0f) / (mant + 1.0f);
    return __builtin_fmaf(y, poly_log2(y * y), e);
}
__device__ __forceinline__ float glsl_exp2(float x) {
    x = x < 129.0f ? x : 129.0f;
    x = x > -126.99999f ? x : -126.99999f;
    const float ip = floorf(x);
    const float fp = x - ip;
    const float ex = __uint_as_float(static_cast<uint32_t>(static_cast<int>(ip) + 127) << 23);
    return ex * poly_exp2(fp);
}
__device__ __forceinline__ float glsl_pow(float x, float y) { return glsl_exp2(glsl_log2(x) * y); }

struct Ray {
    v3 start, dir;
};

// LDS-resident scene view.
struct Scene {
    const float4 *sph;         // cx, cy, cz, r*r
    const int4 *smeta;         // obj_index, material, radius bits, 0
    const float4 *sph_cam;     // camera-origin terms: oc = origin - centre, qc (:587-588)
    const BoxRec *box;
    const float4 *box_cam;     // box-local camera origin (:655 for the primary ray)
    const MatRec *mat;
    const LightRec *light;
    const LightMatRec *lm;
    int ns, nb, nl;
};

// Hit = the closest object so far: t and reference object index (tie-break).
struct Hit {
    float t;
    int obj;     // reference index, -1 = none
    int slot;    // sphere slot (>= 0) or ~box slot (< 0)
    bool inside; // sphere: t_near < 0 (:621)
};

__device__ __forceinline__ bool closer(float t, int obj, const Hit &h) {
    // get_closest_collision (:753, :763, :773): valid when t > 0 and strictly
    // below the running closest (initially 10000); objects are scanned in
    // index order, so an equal t keeps the lower index.
    return t > 0.0f && (t < h.t || (t == h.t && h.obj >= 0 && obj < h.obj));
}

// Box slab test (:655-666): local ray, t1 = min(tmin, tmax), t2 = max(...).
struct Slab {
    v3 rs, rd, t1, t2;
    float t_near, t_far;
};
__device__ __forceinline__ v3 xform_dir(const float *m, v3 d) {
    // (M * vec4(d, 0)).xyz, GLSL order including the * 0.0 of the w column
    return mk(m[0] * d.x + m[1] * d.y + m[2] * d.z + m[3] * 0.0f,
              m[4] * d.x + m[5] * d.y + m[6] * d.z + m[7] * 0.0f,
              m[8] * d.x + m[9] * d.y + m[10] * d.z + m[11] * 0.0f);
}
__device__ __forceinline__ v3 xform_point(const float *m, v3 p) {
    return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3] * 1.0f, m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7] * 1.0f,
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11] * 1.0f);
}
__device__ __forceinline__ Slab slab(const BoxRec &b, v3 rs, v3 rd) {
    Slab s;
    s.rs = rs;
    s.rd = rd;
    const v3 tmn = mk((b.mins[0] - rs.x) / rd.x, (b.mins[1] - rs.y) / rd.y, (b.mins[2] - rs.z) / rd.z);
    const v3 tmx = mk((b.maxs[0] - rs.x) / rd.x, (b.maxs[1] - rs.y) / rd.y, (b.maxs[2] - rs.z) / rd.z);
    s.t1 = mk(gmin(tmn.x, tmx.x), gmin(tmn.y, tmx.y), gmin(tmn.z, tmx.z));
    s.t2 = mk(gmax(tmn.x, tmx.x), gmax(tmn.y, tmx.y), gmax(tmn.z, tmx.z));
    s.t_near = gmax(gmax(s.t1.x, s.t1.y), s.t1.z);
    s.t_far = gmin(gmin(s.t2.x, s.t2.y), s.t2.z);
    return s;
}
// intersect_box_object's t (:680-696); -1 on a miss.
__device__ __forceinline__ float slab_t(const Slab &s) {
    if (s.t_near >= s.t_far || s.t_far <= 0.0f) return -1.0f;
    return s.t_near < 0.0f ? s.t_far : s.t_near;
}

// intersect_sphere_object's t (:586-625) from the ray-invariant terms.
__device__ __forceinline__ float sphere_t(float qb, float qc, float qa2, float qa4, bool &inside) {
    const float qd = qb * qb - qa4 * qc;
    if (qd < 0.0f) return -1.0f;
    const float sq = sqrtf(qd);
    const float t1 = (-qb + sq) / qa2;
    const float t2 = (-qb - sq) / qa2;
    const float tn = gmin(t1, t2), tf = gmax(t1, t2);
    if (tf < 0.0f) return -1.0f;
    inside = tn < 0.0f;
    return inside ? tf : tn;
}

template <bool kPrimary>
__device__ __forceinline__ Hit closest(const Scene &S, const Ray &r) {
    Hit h{10000.0f, -1, 0, false};
    for (int b = 0; b < S.nb; ++b) {
        const BoxRec &B = S.box[b];
        v3 rs;
        if (kPrimary) {
            const float4 c = S.box_cam[b];
            rs = mk(c.x, c.y, c.z);
        } else {
            rs = xform_point(B.w2l, r.start);
        }
        const float t = slab_t(slab(B, rs, xform_dir(B.w2l, r.dir)));
        if (closer(t, B.obj_index, h)) h = {t, B.obj_index, ~b, false};
    }
    const v3 d2 = muls(r.dir, 2.0f);
    const float qa = dot(r.dir, r.dir);
    const float qa2 = 2.0f * qa, qa4 = 4.0f * qa;
    for (int s = 0; s < S.ns; ++s) {
        float qb, qc;
        if (kPrimary) {
            const float4 c = S.sph_cam[s];
            qb = dot(d2, mk(c.x, c.y, c.z));
            qc = c.w;
        } else {
            const float4 c = S.sph[s];
            const v3 oc = sub(r.start, mk(c.x, c.y, c.z));
            qb = dot(d2, oc);
            qc = dot(oc, oc) - c.w;
        }
        const float qd = qb * qb - qa4 * qc;
        if (qd >= 0.0f) {  // rare per sphere: keep the divisions off the common path
            bool inside = false;
            const float t = sphere_t(qb, qc, qa2, qa4, inside);
            const int obj = S.smeta[s].x;
            if (closer(t, obj, h)) h = {t, obj, s, inside};
        }
    }
    return h;
}

// Shadow query (:807-819): is there any object with 0 < t < 1 along
// start + t * dir? (equivalent to closest-hit t < 1.)
__device__ __forceinline__ bool occluded(const Scene &S, v3 start, v3 dir) {
    bool hit = false;
    for (int b = 0; b < S.nb && !hit; ++b) {
        const BoxRec &B = S.box[b];
        const float t = slab_t(slab(B, xform_point(B.w2l, start), xform_dir(B.w2l, dir)));
        hit = t > 0.0f && t < 1.0f;
    }
    const v3 d2 = muls(dir, 2.0f);
    const float qa = dot(dir, dir);
    const float qa2 = 2.0f * qa, qa4 = 4.0f * qa;
    for (int s = 0; s < S.ns; ++s) {
        if (__all(hit)) break;  // wave-uniform exit once every lane is decided
        if (!hit) {
            const float4 c = S.sph[s];
            const v3 oc = sub(start, mk(c.x, c.y, c.z));
            const float qb = dot(d2, oc);
            const float qc = dot(oc, oc) - c.w;
            const float qd = qb * qb - qa4 * qc;
            if (qd >= 0.0f) {
                bool inside;
                const float t = sphere_t(qb, qc, qa2, qa4, inside);
                hit = t > 0.0f && t < 1.0f;
            }
        }
    }
    return hit;
}

struct Collision {
    v3 p, n;
    bool inside;
    int material;
};

// Build the collision record of the winning object (:628-637, :686-721).
__device__ __forceinline__ Collision resolve(const Scene &S, const Ray &r, const Hit &h) {
    Collision c;
    if (h.slot >= 0) {
        const float4 sp = S.sph[h.slot];
        const v3 pos = mk(sp.x, sp.y, sp.z);
        c.material = S.smeta[h.slot].y;
        c.p = add(r.start, muls(r.dir, h.t));
        c.n = normalize(sub(c.p, pos));
        c.inside = h.inside;
        if (c.inside) c.n = muls(c.n, -1.0f);  // leaving the sphere: flip (:634-637)
    } else {
        const BoxRec &B = S.box[~h.slot];
        c.material = B.material;
        const Slab s = slab(B, xform_point(B.w2l, r.start), xform_dir(B.w2l, r.dir));
        float isect = s.t_near;
        v3 boundary = s.t1;
        c.inside = false;
        if (s.t_near < 0.0f) {
            isect = s.t_far;
            boundary = s.t2;
            c.inside = true;
        }
        int face = 0;
        if (isect == boundary.y) face = 1;
        else if (isect == boundary.z) face = 2;
        v3 n = mk(face == 0 ? 1.0f : 0.0f, face == 1 ? 1.0f : 0.0f, face == 2 ? 1.0f : 0.0f);
        if (comp(s.rd, face) > 0.0f) n = muls(n, -1.0f);
        const float *N = B.nrm;
        c.n = mk(N[0] * n.x + N[1] * n.y + N[2] * n.z, N[3] * n.x + N[4] * n.y + N[5] * n.z,
                 N[6] * n.x + N[7] * n.y + N[8] * n.z);
        const v3 lp = add(s.rs, muls(s.rd, h.t));
        c.p = xform_point(B.l2w, lp);
    }
    return c;
}

// ads_phong_lighting (:789-840).
__device__ __forceinline__ v3 phong(const Scene &S, const Ray &r, const Collision &c) {
    const MatRec &m = S.mat[c.material];
    float4 dif = make_float4(0.0f, 0.0f, 0.0f, 0.0f), spe = dif;
    const v3 view = normalize(muls(r.dir, -1.0f));
    for (int j = 0; j < S.nl; ++j) {
        const v3 lpos = mk(S.light[j].pos[0], S.light[j].pos[1], S.light[j].pos[2]);
        const v3 ldir = normalize(sub(lpos, c.p));
        const v3 lref = normalize(reflect(muls(ldir, -1.0f), c.n));
        const float cos_theta = dot(ldir, c.n);
        const float cos_phi = dot(view, lref);
        const LightMatRec &q = S.lm[c.material * S.nl + j];
        const float kd = gmax(cos_theta, 0.0f);
        const float ks = glsl_pow(gmax(cos_phi, 0.0f), m.shininess);
        const float4 nd = make_float4(dif.x + q.ld_md[0] * kd, dif.y + q.ld_md[1] * kd, dif.z + q.ld_md[2] * kd,
                                      dif.w + q.ld_md[3] * kd);
        const float4 ns = make_float4(spe.x + q.ls_ms[0] * ks, spe.y + q.ls_ms[1] * ks, spe.z + q.ls_ms[2] * ks,
                                      spe.w + q.ls_ms[3] * ks);
        const bool changes =
            __float_as_uint(nd.x) != __float_as_uint(dif.x) || __float_as_uint(nd.y) != __float_as_uint(dif.y) ||
            __float_as_uint(nd.z) != __float_as_uint(dif.z) || __float_as_uint(nd.w) != __float_as_uint(dif.w) ||
            __float_as_uint(ns.x) != __float_as_uint(spe.x) || __float_as_uint(ns.y) != __float_as_uint(spe.y) ||
            __float_as_uint(ns.z) != __float_as_uint(spe.z) || __float_as_uint(ns.w) != __float_as_uint(spe.w);
        if (changes && !occluded(S, add(c.p, muls(c.n, 0.01f)), sub(lpos, c.p))) {
            dif = nd;
            spe = ns;
        }
    }
    // phong = ambient + diffuse + specular + emissive; return rgb * a (:837-839)
    const float px = ((m.amb_sum[0] + dif.x) + spe.x) + m.emissive[0];
    const float py = ((m.amb_sum[1] + dif.y) + spe.y) + m.emissive[1];
    const float pz = ((m.amb_sum[2] + dif.z) + spe.z) + m.emissive[2];
    const float pw = ((m.amb_sum[3] + dif.w) + spe.w) + m.emissive[3];
    return mk(px * pw, py * pw, pz * pw);
}

// recursive_raytrace (:1071-1105) as real recursion on a compile-time depth:
// the stack machine's order (reflection subtree, then refraction subtree,
// then mix(mix(phong, R, refl), T, transp)) and its flags (:994, :1027).
template <int kDepth, bool kPrimary>
__device__ v3 trace(const Scene &S, const Ray &r);

template <int kDepth, bool kPrimary>
__device__ __forceinline__ v3 trace_body(const Scene &S, const Ray &r) {
    const Hit h = closest<kPrimary>(S, r);
    if (kPrimary && !__any(h.obj >= 0)) return mk(0.0f, 0.0f, 0.0f);  // per-wave early out
    if (h.obj < 0) return mk(0.0f, 0.0f, 0.0f);                        // miss -> black (:962-963)
    const Collision c = resolve(S, r, h);
    v3 col = phong(S, r, c);
    if constexpr (kDepth > 0) {
        const MatRec &m = S.mat[c.material];
#pragma unroll 1
        for (int k = 0; k < 2; ++k) {
            const float w = k == 0 ? m.reflectivity : m.transparency;
            if (w > 0.0f) {
                Ray cr;
                if (k == 0) {
                    cr.start = add(c.p, muls(c.n, 0.001f));
                    cr.dir = reflect(r.dir, c.n);
                } else {
                    cr.start = sub(c.p, muls(c.n, 0.001f));
                    float ratio = 1.0f / m.refraction_index;
                    if (c.inside) ratio = 1.0f / ratio;
                    cr.dir = refract(r.dir, c.n, ratio);
                }
                const v3 cc = trace<kDepth - 1, false>(S, cr);
                col = mix(col, cc, w);
            }
        }
    }
    return col;
}

template <int kDepth, bool kPrimary>
__device__ __noinline__ v3 trace_call(const Scene &S, const Ray &r) {
    return trace_body<kDepth, kPrimary>(S, r);
}

template <int kDepth, bool kPrimary>
__device__ __forceinline__ v3 trace(const Scene &S, const Ray &r) {
    if constexpr (kPrimary || kDepth == 0) return trace_body<kDepth, kPrimary>(S, r);
    else return trace_call<kDepth, kPrimary>(S, r);
}

__device__ __forceinline__ int output_row(const LaunchParams &p, int local) {
    if (p.n_shards <= 0) return p.row_begin + local;
    const int blk = local / p.block_rows;
    return (blk * p.n_shards + p.shard) * p.block_rows + (local - blk * p.block_rows);
}

template <int kDepth>
__global__ __launch_bounds__(kThreads) void render_kernel(LaunchParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    // ---- stage the scene blob into LDS (one pass per work-group) ----
    const float4 *blob = static_cast<const float4 *>(p.scene);
    for (int i = threadIdx.x; i < p.blob_units; i += kThreads) lds[i] = blob[i];
    float4 *sph_cam = lds + p.blob_units;
    float4 *box_cam = sph_cam + p.n_spheres;
    __syncthreads();
    const v3 origin = mk(p.origin[0], p.origin[1], p.origin[2]);
    {
        const float4 *sph = lds + p.off_spheres;
        for (int s = threadIdx.x; s < p.n_spheres; s += kThreads) {
            const float4 c = sph[s];
            const v3 oc = sub(origin, mk(c.x, c.y, c.z));
            sph_cam[s] = make_float4(oc.x, oc.y, oc.z, dot(oc, oc) - c.w);
        }
        const BoxRec *box = reinterpret_cast<const BoxRec *>(lds + p.off_boxes);
        for (int b = threadIdx.x; b < p.n_boxes; b += kThreads) {
            const v3 rs = xform_point(box[b].w2l, origin);
            box_cam[b] = make_float4(rs.x, rs.y, rs.z, 0.0f);
        }
    }
    __syncthreads();
    Scene S;
    S.sph = lds + p.off_spheres;
    S.smeta = reinterpret_cast<const int4 *>(lds + p.off_smeta);
    S.sph_cam = sph_cam;
    S.box = reinterpret_cast<const BoxRec *>(lds + p.off_boxes);
    S.box_cam = box_cam;
    S.mat = reinterpret_cast<const MatRec *>(lds + p.off_mats);
    S.light = reinterpret_cast<const LightRec *>(lds + p.off_lights);
    S.lm = reinterpret_cast<const LightMatRec *>(lds + p.off_lightmat);
    S.ns = p.n_spheres;
    S.nb = p.n_boxes;
    S.nl = p.n_lights;

    // ---- this lane's pixel: wave w covers the 8x8 quadrant w of the tile ----
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = blockIdx.x * kTile + (wave & 1) * 8 + (lane & 7);
    const int local_row = blockIdx.y * kTile + (wave >> 1) * 8 + (lane >> 3);
    const bool active = x < p.width && local_row < p.n_rows;
    if (!__any(active)) return;
    const int y = output_row(p, active ? local_row : 0);

    // ---- camera ray (:377-392) ----
    const int hw = p.width / 2, hh = p.height / 2;
    const float vx = static_cast<float>(x - hw) / static_cast<float>(hw);
    const float vy = static_cast<float>(y - hh) / static_cast<float>(hh);
    const float *M = p.unproj;  // column-major
    float ws[4], we[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ws[k] = M[k] * vx + M[4 + k] * vy + M[8 + k] * 0.5f + M[12 + k] * 1.0f;
        we[k] = M[k] * vx + M[4 + k] * vy + M[8 + k] * 1.0f + M[12 + k] * 1.0f;
    }
    const v3 s3 = mk(ws[0] / ws[3], ws[1] / ws[3], ws[2] / ws[3]);
    const v3 e3 = mk(we[0] / we[3], we[1] / we[3], we[2] / we[3]);
    Ray ray;
    ray.start = origin;
    ray.dir = normalize(sub(e3, s3));

    v3 col = mk(0.0f, 0.0f, 0.0f);
    if (active) col = trace<kDepth, true>(S, ray);
    if (active) p.out[static_cast<size_t>(local_row) * p.width + x] = make_float4(col.x, col.y, col.z, 0.0f);
}

template <int kDepth>
hipError_t launch_depth(const LaunchParams &p, hipStream_t stream) {
    const dim3 grid((p.width + kTile - 1) / kTile, (p.n_rows + kTile - 1) / kTile);
    hipLaunchKernelGGL(render_kernel<kDepth>, grid, dim3(kThreads), lds_bytes(p), stream, p);
    return hipGetLastError();
}

}  // namespace

size_t lds_bytes(const LaunchParams &p) {
    return (static_cast<size_t>(p.blob_units) + p.n_spheres + p.n_boxes) * sizeof(float4);
}

hipError_t launch_render(const LaunchParams &p, int max_depth, hipStream_t stream) {
    switch (max_depth) {
        case 0: return launch_depth<0>(p, stream);
        case 1: return launch_depth<1>(p, stream);
        case 2: return launch_depth<2>(p, stream);
        case 3: return launch_depth<3>(p, stream);
        case 4: return launch_depth<4>(p, stream);
        case 5: return launch_depth<5>(p, stream);
        case 6: return launch_depth<6>(p, stream);
        case 7: return launch_depth<7>(p, stream);
        case 8: return launch_depth<8>(p, stream);
        case 9: return launch_depth<9>(p, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rtamd

namespace rtamd {

// Allow dynamic LDS above the 64 KiB default for every depth instantiation
// (gfx950 has 160 KiB per CU). Best effort: a failure only lowers the largest
// scene that fits, which rt_scene_create checks.
hipError_t allow_large_lds(size_t bytes) {
    const void *fns[] = {
        reinterpret_cast<const void *>(&render_kernel<0>), reinterpret_cast<const void *>(&render_kernel<1>),
        reinterpret_cast<const void *>(&render_kernel<2>), reinterpret_cast<const void *>(&render_kernel<3>),
        reinterpret_cast<const void *>(&render_kernel<4>), reinterpret_cast<const void *>(&render_kernel<5>),
        reinterpret_cast<const void *>(&render_kernel<6>), reinterpret_cast<const void *>(&render_kernel<7>),
        reinterpret_cast<const void *>(&render_kernel<8>), reinterpret_cast<const void *>(&render_kernel<9>)};
    for (const void *f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
    (void)hipGetLastError();  // do not leak a sticky error into the next launch check
    return hipSuccess;
}

}  // namespace rtamd
