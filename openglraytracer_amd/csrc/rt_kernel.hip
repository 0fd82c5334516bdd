// rt_kernel.hip — the hot path of raytrace_compute.glsl as one CDNA4 kernel.
//
// One ray per lane; a 256-thread work-group renders a 16x16 pixel tile as
// four wave64s of 8x8 pixels each (square wave footprints keep the lanes of a
// wave coherent: they hit the same objects, take the same shading branches and
// cull the same spheres). The whole scene (spheres, boxes, materials, lights)
// is staged into LDS once per work-group, together with per-frame constants
// computed there once: the camera-origin terms of every sphere / box and every
// sphere's conservative screen-space footprint. Each lane ends with one float4
// store: a wave writes eight fully-used 128-B lines.
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
//    surface facing away) casts no shadow ray — lit and shadowed agree;
//  * culling (conservative, with margins far above float error): a primary
//    ray skips spheres whose projected footprint misses its wave's 8x8 tile;
//    a shadow ray skips spheres outside its wave's cone from the light;
//  * a box whose interior holds the ray origin needs only its three exit
//    distances (the slab test's t_far), and a shadow ray compares them with 1
//    without dividing unless the comparison is within 2^-16 of 1.
// Control flow at function level is wave-uniform (per-lane `valid` masks
// instead of early returns), so the ballot-based culling always sees all 64
// lanes; divergence is confined to the innermost exact tests.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <string>

#include "rt_internal.h"

namespace rtamd {
namespace {

// A work-group renders a tile of kWavesX x kWavesY wave footprints of 8x8
// pixels (2 x 2; 32x8 and 16x32 work-group tiles measured no gain, r01).
constexpr int kWavesX = 2, kWavesY = 2;
constexpr int kTileX = 8 * kWavesX, kTileY = 8 * kWavesY;
constexpr int kThreads = 64 * kWavesX * kWavesY;

struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 muls(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ v3 sel(bool c, v3 a, v3 b) { return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z}; }
// dot(vec3) as llvmpipe associates it: x + (y + z)
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }

// Price-of-exactness ablation (timing and accuracy probes, never the product
// build: tools/ab.py, tools/ab_accuracy.py): RT_FAST_DIV (a * v_rcp(b) for
// every division), RT_FAST_RSQ (v_rsq in normalize), RT_FAST_SQRT (v_sqrt in
// the sphere tests and refract), RT_FAST_POW (v_log / v_exp in the specular
// pow); RT_FAST_MATH sets all four.
#ifdef RT_FAST_MATH
#define RT_FAST_DIV
#define RT_FAST_RSQ
#define RT_FAST_SQRT
#define RT_FAST_POW
#endif

// Wave votes on the lane masks themselves: the ballot of the condition (its
// compare's lane mask, without HIP's __any/__all round trip of the predicate
// through a 0/1 vector register and a second compare) against zero / exec.
__device__ __forceinline__ bool wave_any(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }
__device__ __forceinline__ bool wave_all(bool c) { return __builtin_amdgcn_ballot_w64(c) == __builtin_amdgcn_read_exec(); }
__device__ __forceinline__ uint64_t wave_ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// ---- correctly rounded division and square root, short forms -------------
// hipcc lowers a / b (IEEE) to div_scale(b), rcp, 2 fma (the refined
// reciprocal r), div_scale(a), mul, 3 fma, div_fmas, div_fixup; and sqrtf(x)
// to a scale-up of tiny x, v_sqrt, two one-ulp probes with fma, the
// scale-down and a class fix-up. For operands of moderate magnitude the scale
// steps are identities and the fix-ups return their input, so the arithmetic
// that remains is the same correctly rounded result in fewer instructions:
//  * the refined reciprocal r = rcp + one fma step IS the correctly rounded
//    1 / b (on gfx950, for every significand: tools/probes/arith_probe.hip,
//    exhaustive over three binade pairs, profiles/r02k_arith_probe.log);
//  * so one correction of q = a r gives the correctly rounded quotient
//    (Markstein: r correctly rounded and q faithful => q + (a - b q) r,
//    rounded once, is RN(a / b); also 3.2e9 random pairs, 0 mismatches);
//  * a reciprocal shared by several quotients is refined once.
// (v_sqrt errs both ways — 1 ulp low on 15 % of significands, 1 ulp high on
// 982 of 2^24 — so sqrt_short keeps both one-ulp probes.)
// Valid ranges: div_r needs b normal with |b| in [2^-60, 2^60] and a = +0 or
// |a| in [2^-60, 2^60]; sqrt_short needs x >= 2^-96 (or +inf). Callers prove
// the range or check it per wave.
struct Rcp {
    float b, r;
};
__device__ __forceinline__ Rcp rcp_refined(float b) {
    float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    return {b, r};
}
__device__ __forceinline__ float div_r(float a, Rcp d) {
#ifdef RT_FAST_DIV
    return a * __builtin_amdgcn_rcpf(d.b);
#endif
    const float q = a * d.r;
    return __builtin_fmaf(__builtin_fmaf(-d.b, q, a), d.r, q);
}
__device__ __forceinline__ float sqrt_short(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u), up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
    return __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
}
// a / b: the IEEE division (RT_FAST_DIV ablation builds: a * v_rcp(b))
__device__ __forceinline__ float fdiv(float a, float b) {
#ifdef RT_FAST_DIV
    return a * __builtin_amdgcn_rcpf(b);
#else
    return a / b;
#endif
}
// 1 / sqrt(d), both correctly rounded (GLSL inversesqrt as llvmpipe evaluates
// it): the refined reciprocal of the short square root
__device__ __forceinline__ float inv_sqrt(float d) {
#ifdef RT_FAST_RSQ
    return __builtin_amdgcn_rsqf(d);
#endif
    // d in [2^-96, 2^100] as one unsigned compare of the bit pattern (NaN and
    // negative d fall outside), so the vote takes the compare's lane mask
    if (wave_all(__float_as_uint(d) - __float_as_uint(0x1p-96f) <=
                 __float_as_uint(0x1p100f) - __float_as_uint(0x1p-96f)))
        return rcp_refined(sqrt_short(d)).r;
    return 1.0f / sqrtf(d);
}
// normalize(v) = v * inversesqrt(dot(v, v))
__device__ __forceinline__ v3 normalize(v3 a) { return muls(a, inv_sqrt(dot(a, a))); }
// inversesqrt of d = 1 + k ulp(1) (|k| <= 2048 float steps of d's bit pattern):
// fl(1 / fl(sqrt(d))) in closed form. Above 1, fl(sqrt(1 + k 2^-23)) =
// 1 + floor(k/2) 2^-23 and its reciprocal rounds to 1 - floor(k/2) 2^-23;
// below 1, d = 1 - m 2^-24 gives 1 - ceil(m/2) 2^-24 and then
// 1 + ceil(m/4) 2^-23 (the neglected higher-order terms stay far below the
// rounding boundaries: exhaustively equal to the IEEE pair for k in
// [-8190, 2897], tests/test_host.py::test_inv_sqrt_near_one).
__device__ __forceinline__ bool near_one(float d) { return __float_as_uint(d) - 0x3f7ff800u <= 0x1000u; }
__device__ __forceinline__ float inv_sqrt_near_one(float d) {
    const uint32_t b = __float_as_uint(d);
    // both arms computed, then one select (as a ternary the compiler made
    // this a divergent branch)
    const uint32_t above = 0x3f800000u - ((b - 0x3f800000u) & ~1u);  // k >= 0
    const uint32_t below = 0x3f800000u + ((0x3f800003u - b) >> 2);    // k < 0: (3 - k) >> 2
    return __uint_as_float(b >= 0x3f800000u ? above : below);
}
// normalize() of a vector that is a unit vector up to rounding (a reflected
// or negated unit vector): the closed form when every lane's squared length
// is within 2048 ulps of 1, else the general path; bit-identical either way
__device__ __forceinline__ v3 normalize_unit(v3 a) {
    const float d = dot(a, a);
#ifdef RT_FAST_RSQ
    return muls(a, __builtin_amdgcn_rsqf(d));
#endif
    if (wave_all(near_one(d))) return muls(a, inv_sqrt_near_one(d));
    return muls(a, inv_sqrt(d));
}
__device__ __forceinline__ float gmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float gmax(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float comp(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
// reflect(I, N) = I - 2 * dot(N, I) * N
__device__ __forceinline__ v3 reflect(v3 i, v3 n) { return sub(i, muls(n, 2.0f * dot(n, i))); }
// refract(I, N, eta) with k = 1 - eta * (eta * (1 - dot^2)) (Mesa's builtin)
__device__ __forceinline__ float sphere_sqrt(float qd);
__device__ __forceinline__ v3 refract(v3 i, v3 n, float eta) {
    const float d = dot(n, i);
    const float k = 1.0f - eta * (eta * (1.0f - d * d));
    // every lane computes the ray (the short square root when every lane's
    // operand allows it; a total internal reflection lane takes any operand)
    // and total internal reflection selects the zero vector
    const bool tir = k < 0.0f;
    const v3 r = sub(muls(i, eta), muls(n, eta * d + sphere_sqrt(tir ? 1.0f : k)));
    return tir ? mk(0.0f, 0.0f, 0.0f) : r;
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
    // mant - 1 is +0 or at least 2^-23, mant + 1 in [2, 3): the short division is exact
    const float y = div_r(mant - 1.0f, rcp_refined(mant + 1.0f));
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
// pow(x, y) for x = max(cos_phi, 0) as the shading computes it: gmax never
// returns NaN or a negative value, and a dot product of two normalize()d
// vectors is at most about 3 or NaN, so glsl_log2's NaN and +inf cases are
// never reached; its zero case becomes a select
__device__ __forceinline__ float glsl_pow_cos(float x, float y) {
#ifdef RT_FAST_POW
    return x == 0.0f ? 0.0f : __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#endif
    const uint32_t i = __float_as_uint(x);
    const float e = static_cast<float>(static_cast<int>((i >> 23) & 0xffu) - 127);
    const float mant = __uint_as_float((i & 0x007fffffu) | 0x3f800000u);
    const float q = div_r(mant - 1.0f, rcp_refined(mant + 1.0f));
    // computed in every lane (the empty asm pins the value): left to itself
    // the compiler sank the polynomial into a divergent branch around the
    // zero case (configs 3-4 -2 %, config 2 -1 % as a select)
    float lr = __builtin_fmaf(q, poly_log2(q * q), e);
    asm volatile("" : "+v"(lr));
    const float l = x == 0.0f ? -__builtin_inff() : lr;
    return glsl_exp2(l * y);
}

// Hardware sqrt (about 1 ulp, no correction steps): culling arithmetic only,
// whose margins exceed its error by orders of magnitude.
__device__ __forceinline__ float fsqrt_approx(float x) { return __builtin_amdgcn_sqrtf(x); }

// ---- wave-wide reductions (called with all 64 lanes active) -------------
// DPP butterfly within each 16-lane row, then row broadcasts; lane 63 holds
// the result, read back as a wave-uniform value.
template <bool kMax>
__device__ __forceinline__ float dpp_step(float v, float t) { return kMax ? fmaxf(v, t) : fminf(v, t); }
template <int kCtrl, int kRows>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), kCtrl, kRows, 0xF, false));
}
template <bool kMax>
__device__ __forceinline__ float wave_minmax(float v) {
    v = dpp_step<kMax>(v, dpp<0xB1, 0xF>(v));   // quad_perm [1,0,3,2]
    v = dpp_step<kMax>(v, dpp<0x4E, 0xF>(v));   // quad_perm [2,3,0,1]
    v = dpp_step<kMax>(v, dpp<0x141, 0xF>(v));  // row_half_mirror
    v = dpp_step<kMax>(v, dpp<0x140, 0xF>(v));  // row_mirror
    v = dpp_step<kMax>(v, dpp<0x142, 0xA>(v));  // row_bcast:15 into rows 1, 3
    v = dpp_step<kMax>(v, dpp<0x143, 0xC>(v));  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_min(float v) { return wave_minmax<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_minmax<true>(v); }
__device__ __forceinline__ float lane_value(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

struct Ray {
    v3 start, dir;
};

// Development probe (RT_STATS builds only, tools/stats.py): event counts per
// launch, accumulated per wave in LDS and flushed once per wave.
#ifdef RT_STATS
constexpr int kStats = 16;
__device__ unsigned long long rt_stats[kStats];
__shared__ unsigned rt_stats_lds[16][kStats];
// lanes for which `c` holds (active lanes only)
#define RT_STAT(k, c)                                                                          \
    do {                                                                                       \
        const uint64_t b_ = __ballot(c);                                                       \
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1)))                                \
            atomicAdd(&rt_stats_lds[threadIdx.x >> 6][k], static_cast<unsigned>(__popcll(b_))); \
    } while (0)
#else
#define RT_STAT(k, c) \
    do {              \
    } while (0)
#endif

// Development probe (RT_CYCLES builds only, tools/cycles.py): wave time per
// phase. At every phase switch the first active lane of the wave adds the
// shader-clock cycles since the previous switch to the phase being left
// (per-wave slots in LDS, flushed once per wave), so the sums are wave-time
// — issue and stalls alike — attributed to where the wave was.
enum CycPhase {
    kCycPrologue, kCycRaygen, kCycClosest1, kCycClosest2, kCycResolve, kCycPhong, kCycShadow, kCycWalk,
    kCycStore, kCycPhases
};
#ifdef RT_CYCLES
__device__ unsigned long long rt_cycles[16];
__shared__ unsigned long long rt_cyc_lds[16][kCycPhases + 1];  // [wave][phase], [kCycPhases]: last switch
__shared__ int rt_cyc_cur[16];
#define RT_CYC(next)                                                                     \
    do {                                                                                 \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();                    \
        const int w_ = threadIdx.x >> 6;                                                 \
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {                         \
            rt_cyc_lds[w_][rt_cyc_cur[w_]] += now_ - rt_cyc_lds[w_][kCycPhases];         \
            rt_cyc_lds[w_][kCycPhases] = now_;                                           \
            rt_cyc_cur[w_] = (next);                                                     \
        }                                                                                \
    } while (0)
// the switch after `v` is computed
#define RT_CYC_AFTER(next, v)                   \
    do {                                        \
        asm volatile("" ::"v"(v));              \
        RT_CYC(next);                           \
    } while (0)
#else
#define RT_CYC(next) \
    do {             \
    } while (0)
#define RT_CYC_AFTER(next, v) \
    do {                      \
    } while (0)
#endif

// A record read through the constant address space, dword by dword (scalar
// loads when the address is wave-uniform).
template <class T>
__device__ __forceinline__ T cload(const __attribute__((address_space(4))) T *p) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    T r;
    const __attribute__((address_space(4))) uint32_t *src = (const __attribute__((address_space(4))) uint32_t *)p;
    uint32_t *dst = reinterpret_cast<uint32_t *>(&r);
#pragma unroll
    for (int i = 0; i < static_cast<int>(sizeof(T) / 4); ++i) dst[i] = src[i];
    return r;
}

// LDS-resident scene view.
struct Scene {
    const float4 *sph;      // cx, cy, cz, r*r
    const int4 *smeta;      // obj_index, material, radius bits, 0
    const float4 *sph_cam;  // camera-origin terms: oc = origin - centre, qc (:587-588)
    int cam_terms;          // sph_cam present (a constant per kernel: not with lean views)
    const int4 *sph_px;     // conservative pixel footprint x0, x1, y0, y1 (culling)
    const BoxRec *box;
    const float4 *box_cam;  // box-local camera origin (:655), w = origin strictly inside
    const MatRec *mat;
    const LightRec *light;
    const LightMatRec *lm;
    const float4 *bvh;  // BvhNode pairs (lo, hi)
    const uint32_t *blink;  // per node, kBvhOctants traversal links
    const ShadowCone *cone;  // [light][sphere] shadow culling cones
    const char *dmask;  // [live light][face][row][col] shadow direction masks (nullptr: none)
    int dmask_n, dmask_bytes;
    int dmask_box;  // the masks carry a bit per box (bit ns + b)
    // per (box, light) the plane separating the box from the light's end of
    // every shadow segment (rt_scene.cpp; nullptr: none, or culling off)
    const __attribute__((address_space(4))) float4 *cbplane;
    const uint64_t *gmask;  // wide masks in global memory: [live light][texel][word] (nullptr: none)
    const uint4 *glist;     // their candidate lists: [live light][texel] (nullptr: none)
    int gwords;
    // secondary rays' origin-sphere candidate lists, 32-B records
    // [sphere][texel] (rt_internal.h kOListSlots; nullptr: none)
    const uint4 *olist;
    // The same box and light records in the device blob through the constant
    // address space: a wave-uniform record index becomes scalar loads into
    // SGPRs (no LDS round trip, no VGPRs) — used where the index is uniform.
    const __attribute__((address_space(4))) BoxRec *cbox;
    const __attribute__((address_space(4))) LightRec *clight;
#ifdef RT_UNIFORM_MAT
    const __attribute__((address_space(4))) MatRec *cmat;
    const __attribute__((address_space(4))) LightMatRec *clm;
#endif
    int ns, nb, nl, nm, nbvh;
    int cull;
    int room;  // the one box is a room (kShapeRoom): its shadow shortcut always applies
    int tx0, tx1, ty0, ty1;  // this wave's pixel rectangle (frame coordinates)
};

// Hit = the closest object so far: t and reference object index (tie-break).
// A box's hit face is decided when the box becomes the closest (from the
// slab distances t is the minimum / maximum of, :690-721), so the three slab
// distances are not carried through the rest of the scan (3 VGPRs less
// live across the sphere tests and the BVH walk).
struct Hit {
    float t;
    int obj;   // reference index, -1 = none
    int slot;  // sphere slot (>= 0) or ~box slot (< 0)
    int info;  // bit 0: t_near < 0, the ray leaves the object (:621, :693-696); bits 1-2: box face
};
// The collision record's face (:699-705): x unless t equals the y, then the
// z slab distance.
__device__ __forceinline__ int box_face(float t, v3 bnd) { return t == bnd.y ? 1 : (t == bnd.z ? 2 : 0); }

__device__ __forceinline__ bool closer(float t, int obj, const Hit &h) {
    // get_closest_collision (:753, :763, :773): valid when t > 0 and strictly
    // below the running closest (initially 10000); objects are scanned in
    // index order, so an equal t keeps the lower index.
    return t > 0.0f && (t < h.t || (t == h.t && h.obj >= 0 && obj < h.obj));
}

// ---- boxes (:647-724) ----------------------------------------------------
struct Slab {
    v3 rs, rd, t1, t2;
    float t_near, t_far;
};
// (w2l * vec4(d, 0.0)).xyz of a box: the w column's products with 0.0 come
// precomputed with the record (each is the same float product, +-0 or NaN)
__device__ __forceinline__ v3 box_dir(const BoxRec &b, v3 d) {
    const float *m = b.w2l;
    return mk(m[0] * d.x + m[1] * d.y + m[2] * d.z + b.w2l_w0[0], m[4] * d.x + m[5] * d.y + m[6] * d.z + b.w2l_w0[1],
              m[8] * d.x + m[9] * d.y + m[10] * d.z + b.w2l_w0[2]);
}
__device__ __forceinline__ v3 xform_point(const float *m, v3 p) {
    return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3] * 1.0f, m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7] * 1.0f,
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11] * 1.0f);
}
__device__ __forceinline__ Slab slab(const BoxRec &b, v3 rs, v3 rd) {
    Slab s;
    s.rs = rs;
    s.rd = rd;
    const v3 tmn = mk(fdiv(b.mins[0] - rs.x, rd.x), fdiv(b.mins[1] - rs.y, rd.y), fdiv(b.mins[2] - rs.z, rd.z));
    const v3 tmx = mk(fdiv(b.maxs[0] - rs.x, rd.x), fdiv(b.maxs[1] - rs.y, rd.y), fdiv(b.maxs[2] - rs.z, rd.z));
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
// Origin strictly inside the box on every axis (local coordinates).
__device__ __forceinline__ bool strictly_inside(const BoxRec &b, v3 rs) {
    return b.mins[0] < rs.x && rs.x < b.maxs[0] && b.mins[1] < rs.y && rs.y < b.maxs[1] && b.mins[2] < rs.z &&
           rs.z < b.maxs[2];
}
__device__ __forceinline__ bool not_nan(v3 v) { return v.x == v.x && v.y == v.y && v.z == v.z; }
// Inside the box the slab's t2 on an axis is the exit boundary chosen by the
// sign of the direction: max((mins-s)/d, (maxs-s)/d) with one division. For
// d = +-0 the sign bit picks the +inf quotient, exactly as max() does.
__device__ __forceinline__ float exit_num(float mn, float mx, float s, float d) {
    return (__float_as_uint(d) >> 31) ? (mn - s) : (mx - s);
}
__device__ __forceinline__ v3 exits(const BoxRec &b, v3 rs, v3 rd) {
    const float ex = exit_num(b.mins[0], b.maxs[0], rs.x, rd.x), ey = exit_num(b.mins[1], b.maxs[1], rs.y, rd.y),
                ez = exit_num(b.mins[2], b.maxs[2], rs.z, rd.z);
    return mk(fdiv(ex, rd.x), fdiv(ey, rd.y), fdiv(ez, rd.z));
}
// Box t for the closest-hit loop (-1 on a miss), with the slab distances the
// collision record's face test needs (bnd: t1 when entering, t2 when leaving)
// and whether the ray leaves the box. With the origin strictly inside and no
// NaN in the direction: t_near < 0 < t_far, so t = t_far (:690-696).
// (One correctly rounded division for the nearest exit, chosen by the
// approximate quotients when they are apart by more than their error,
// bit-identical, measured slower: config 2 +4.2 %, config 5 +4.9 %, config 4
// +3.8 %, round 5, profiles/r05d_ab.log: the three v_rcp and the selects cost
// more than the two divisions they save.)
__device__ __forceinline__ float box_t(const BoxRec &b, v3 rs, v3 rd, bool inside, v3 &bnd, bool &leaving) {
    if (inside && not_nan(rd)) {
        bnd = exits(b, rs, rd);
        leaving = true;
        return gmin(gmin(bnd.x, bnd.y), bnd.z);
    }
    const Slab sl = slab(b, rs, rd);
    leaving = sl.t_near < 0.0f;
    bnd = sel(leaving, sl.t2, sl.t1);
    return slab_t(sl);
}
// Conservative slab pre-test of a box (local ray rs, rd): false only when the
// exact slab test (slab(): six correctly rounded quotients q = fl(n / d) of
// the same numerators n = fl(mins - rs), fl(maxs - rs)) provably misses —
// t_near >= t_far, t_far <= 0 — or provably gives t_near > t_max >= 0.
// Here q' = fl(n * v_rcp(d)): v_rcp is within 1 ulp, so |q' - q| <= 2^-21 |q|
// for |d| >= 2^-60 and finite operands; min and max are monotone, so t_near'
// and t_far' keep that relative bound, and the decisions below carry a margin
// of 2^-19 of the magnitudes (4x the bound, the subtraction's rounding
// included). Anything else — a tiny or non-finite direction component, a
// non-finite distance — is "may hit", and the exact test decides. So a culled
// lane is one whose exact test misses: bit-identical results.
__device__ __forceinline__ bool slab_may_hit(const BoxRec &b, v3 rs, v3 rd, float t_max) {
    const bool ok = fabsf(rd.x) >= 0x1p-60f && fabsf(rd.y) >= 0x1p-60f && fabsf(rd.z) >= 0x1p-60f;
    const float ix = __builtin_amdgcn_rcpf(rd.x), iy = __builtin_amdgcn_rcpf(rd.y), iz = __builtin_amdgcn_rcpf(rd.z);
    const float ax = (b.mins[0] - rs.x) * ix, bx = (b.maxs[0] - rs.x) * ix;
    const float ay = (b.mins[1] - rs.y) * iy, by = (b.maxs[1] - rs.y) * iy;
    const float az = (b.mins[2] - rs.z) * iz, bz = (b.maxs[2] - rs.z) * iz;
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    const float an = fabsf(tn), af = fabsf(tf);
    const bool finite = an < 1e30f && af < 1e30f;  // (NaN fails)
    const float m = 0x1p-19f;
    const bool miss = (tn - tf > m * (an + af)) | (tf < -m * af) | (tn > t_max + m * an);
    return !(ok & finite & miss);
}

// fl(num / d) < 1 for a non-negative quotient, dividing only when |num| is
// within 2^-16 of |d| (correctly rounded division is monotonic).
__device__ __forceinline__ bool quotient_below_one(float num, float d) {
    const float an = fabsf(num), ad = fabsf(d);
    if (an > 1e-30f && ad > 1e-30f) {
        if (an > ad * 1.0000153f) return false;
        if (an < ad * 0.9999847f) return true;
    }
    return fdiv(num, d) < 1.0f;
}
// Does the box hold an occluder with 0 < t < 1 (:813-816)? light_bit: the
// light is inside the box with a margin (host, float64), so a segment that
// starts inside ends inside too and exits past t = 1.
// pretest: slab_may_hit first (RT_OPT_CULLING; never for the room)
__device__ __forceinline__ bool box_occludes(const BoxRec &b, v3 start, v3 dir, uint32_t light_bit, bool room,
                                             bool pretest) {
    if (room || ((b.light_inside & light_bit) && b.translate_only)) {
        // identity rotation: xform_point is ((1 x + 0 y) + 0 z) + w, which for
        // finite start equals x + w up to the sign of a zero (comparisons
        // alike); a non-finite component stays non-finite here and fails
        // strictly_inside, so a pass implies the full transform passes too
        const v3 rq = mk(start.x + b.w2l[3], start.y + b.w2l[7], start.z + b.w2l[11]);
        if (strictly_inside(b, rq)) return false;
    }
    const v3 rs = xform_point(b.w2l, start);
    const bool inside = strictly_inside(b, rs);
    if (inside && (b.light_inside & light_bit)) return false;
    const v3 rd = box_dir(b, dir);
    if (inside && not_nan(rd)) {
        // t = t_far > 0; occluded iff some exit distance is below 1
        return quotient_below_one(exit_num(b.mins[0], b.maxs[0], rs.x, rd.x), rd.x) ||
               quotient_below_one(exit_num(b.mins[1], b.maxs[1], rs.y, rd.y), rd.y) ||
               quotient_below_one(exit_num(b.mins[2], b.maxs[2], rs.z, rd.z), rd.z);
    }
    if (pretest && !room) {
        // the exact slab test (six divisions) only where the pre-test
        // cannot rule out an occluder with 0 < t < 1 (round 6: the shipped
        // scene's rotated boxes)
        const bool may = slab_may_hit(b, rs, rd, 1.0f);
        if (!wave_any(may)) return false;
        if (!may) return false;
    }
    const float t = slab_t(slab(b, rs, rd));
    return t > 0.0f && t < 1.0f;
}

// ---- spheres (:583-640) --------------------------------------------------
// The shader divides both roots' numerators n1 = -qb + sq >= n2 = -qb - sq by
// qa2 and then picks one by the quotients' signs. For qa2 a normal float in
// [2^-100, 2^100] and |n1|, |n2| >= qa2 * 2^-100 (`floor`, per ray) neither
// quotient underflows, so each has its numerator's sign, t1 >= t2 (correctly
// rounded division is monotonic), and the choice can be made on the
// numerators: one division instead of two, bit-identical. Otherwise (zero or
// tiny numerators, qa2 zero or huge; floor = NaN) the shader's arithmetic runs
// as written. NaN numerators pass the check only towards a NaN or a -1 result,
// both misses, as in the shader.
__device__ __forceinline__ float root_floor(float qa2) {
    return (qa2 >= 0x1p-100f && qa2 <= 0x1p100f) ? qa2 * 0x1p-100f : __builtin_nanf("");
}
// (Short divisions behind the same kind of per-wave range check measured
// slower for the box exits, config 4 +1 %, and again with one-correction
// quotients: config 2 +2.5 %, config 3 +2.6 %, config 4 +1.7 %; for this
// division of the sphere test, configs 3-4 +2-3 %; for the camera ray's six
// perspective divisions, config 2 +1.5 % / +3.5 %: the per-wave check and
// its branch cost more than the instructions saved.)
// sqrt(qd) of the sphere tests, correctly rounded: the short form when every
// active lane's operand is in its range (qd >= 2^-96; +inf included), else
// the IEEE sequence (config 4 18.20 -> 17.94 ms, config 3 1.030 -> 1.001 ms)
__device__ __forceinline__ float sphere_sqrt(float qd) {
#ifdef RT_FAST_SQRT
    return __builtin_amdgcn_sqrtf(qd);
#endif
    if (wave_all(qd >= 0x1p-96f)) return sqrt_short(qd);
    return sqrtf(qd);
}
// intersect_sphere_object's t (:586-625) from the ray-invariant terms.
__device__ __forceinline__ float sphere_t(float qb, float qc, float qa2, float qa4, float floor, bool &inside) {
    const float qd = qb * qb - qa4 * qc;
    if (qd < 0.0f) return -1.0f;
    const float sq = sphere_sqrt(qd);
    const float n1 = -qb + sq, n2 = -qb - sq;
    if (fminf(fabsf(n1), fabsf(n2)) >= floor) {
        // (the quotient in every lane and a select for t_far < 0 measured
        // slower: config 4 16.57 -> 16.79 ms)
        if (n1 < 0.0f) return -1.0f;  // t_far < 0
        inside = n2 < 0.0f;           // t_near < 0
        return fdiv(inside ? n1 : n2, qa2);
    }
    const float t1 = fdiv(n1, qa2);
    const float t2 = fdiv(n2, qa2);
    const float tn = gmin(t1, t2), tf = gmax(t1, t2);
    if (tf < 0.0f) return -1.0f;
    inside = tn < 0.0f;
    return inside ? tf : tn;
}
// Shadow test of one sphere: sphere_t's t in (0, 1), deciding fl(n / qa2) < 1
// without the division unless n is within 2^-16 of qa2 (quotient_below_one).
// (The same decision as predicated arithmetic, with only undecided lanes
// branching to this code, measured slower: config 2 37.9 -> 40.2 us per frame,
// configs 3-4 even.)
__device__ __forceinline__ bool sphere_blocks(float qb, float qc, float qa2, float qa4, float floor) {
    const float qd = qb * qb - qa4 * qc;
    if (!(qd >= 0.0f)) return false;
    const float sq = sphere_sqrt(qd);
    const float n1 = -qb + sq, n2 = -qb - sq;
    if (fminf(fabsf(n1), fabsf(n2)) >= floor) {
        if (n1 < 0.0f) return false;
        const float n = n2 < 0.0f ? n1 : n2;
        return n > 0.0f && quotient_below_one(n, qa2);
    }
    bool inside;
    const float t = sphere_t(qb, qc, qa2, qa4, __builtin_nanf(""), inside);
    return t > 0.0f && t < 1.0f;
}

__device__ __forceinline__ void test_sphere(const Scene &S, int s, v3 start, v3 d2, float qa2, float qa4, float floor,
                                            bool primary, Hit &h) {
    float qb, qc;
    if (primary) {
        const float4 c = S.sph_cam[s];
        qb = dot(d2, mk(c.x, c.y, c.z));
        qc = c.w;
    } else {
        const float4 c = S.sph[s];
        const v3 oc = sub(start, mk(c.x, c.y, c.z));
        qb = dot(d2, oc);
        qc = dot(oc, oc) - c.w;
    }
    const float qd = qb * qb - qa4 * qc;
    if (qd >= 0.0f) {  // rare per sphere: keep the divisions off the common path
        bool inside = false;
        const float t = sphere_t(qb, qc, qa2, qa4, floor, inside);
        const int obj = S.smeta[s].x;
        if (closer(t, obj, h)) {
            h.t = t;
            h.obj = obj;
            h.slot = s;
            h.info = inside ? 1 : 0;
        }
    }
}

// Conservative ray / inflated-box overlap for the BVH. Every node box is
// its spheres' bounding box grown by m = 1e-3 + 1e-4 |x| (host, rounded
// outward), so a ray through any point of a sphere's box spends a t-interval
// of at least m / |d_axis| around it inside the node's slabs. The slab
// distances here — approximate reciprocal direction, lo * id - o * id as one
// fma — are off by about 2^-22 |t| + 2^-24 |o| / |d_axis|, under 2e-3 of
// that margin for origins within 20 units of the centre, so no extra slack
// is needed: a node whose spheres the exact test could hit before t_limit
// always passes (tn <= t of the hit < t_limit, tf >= it > 0).
struct RayInv {
    v3 oid, id;  // o * id, 1 / d (approximate)
};
__device__ __forceinline__ float safe_rcp(float d) {
    return fabsf(d) > 1e-30f ? __builtin_amdgcn_rcpf(d) : (__float_as_uint(d) >> 31 ? -1e30f : 1e30f);
}
__device__ __forceinline__ RayInv ray_inv(const Ray &r) {
    const v3 id = mk(safe_rcp(r.dir.x), safe_rcp(r.dir.y), safe_rcp(r.dir.z));
    return {mk(r.start.x * id.x, r.start.y * id.y, r.start.z * id.z), id};
}
__device__ __forceinline__ bool node_hit(const RayInv &q, float4 lo, float4 hi, float t_limit) {
    const float x0 = __builtin_fmaf(lo.x, q.id.x, -q.oid.x), x1 = __builtin_fmaf(hi.x, q.id.x, -q.oid.x);
    const float y0 = __builtin_fmaf(lo.y, q.id.y, -q.oid.y), y1 = __builtin_fmaf(hi.y, q.id.y, -q.oid.y);
    const float z0 = __builtin_fmaf(lo.z, q.id.z, -q.oid.z), z1 = __builtin_fmaf(hi.z, q.id.z, -q.oid.z);
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return tn <= tf && tf >= 0.0f && tn <= t_limit;
}

// direction_texel, defined below
__device__ __forceinline__ int direction_texel(int n, v3 u);

// get_closest_collision (:738-782). Called with all lanes active. origin:
// the sphere slot a secondary ray starts on (-1: the camera or a box).
template <bool kPrimary>
__device__ __forceinline__ Hit closest_impl(const Scene &S, const Ray &r, bool valid, int origin) {
    Hit h{10000.0f, -1, 0, 0};
    RT_STAT(kPrimary ? 0 : 1, valid);
    RT_STAT(kPrimary ? 13 : 2, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
    for (int b = 0; b < S.nb; ++b) {
        const BoxRec B = cload(S.cbox + b);
        v3 rs;
        bool inside;
        if (kPrimary) {
            const float4 c = S.box_cam[b];
            rs = mk(c.x, c.y, c.z);
            inside = c.w != 0.0f;
        } else {
            rs = xform_point(B.w2l, r.start);
            inside = strictly_inside(B, rs);
        }
        v3 bnd;
        bool leaving;
        const v3 rd = box_dir(B, r.dir);
#ifdef RT_ABLATE_BOX_PRIMARY
        if (kPrimary && !S.room && !inside) continue;  // (timing probe: wrong images by design)
#endif
        if (!S.room && S.cull) {
            // boxes the ray may enter from outside: the exact slab test only
            // for lanes whose pre-test cannot rule the box out (a ruled-out
            // lane's exact t is a miss: slab_may_hit), and not at all in a wave
            // where none can (round 6: the shipped scene's rotated boxes)
            const bool may = valid && (inside || slab_may_hit(B, rs, rd, 1e30f));
            if (!wave_any(may)) continue;
            const float t = box_t(B, rs, rd, inside, bnd, leaving);
            if (may && closer(t, B.obj_index, h)) h = {t, B.obj_index, ~b, (leaving ? 1 : 0) | (box_face(t, bnd) << 1)};
            continue;
        }
        const float t = box_t(B, rs, rd, inside, bnd, leaving);
        if (closer(t, B.obj_index, h)) h = {t, B.obj_index, ~b, (leaving ? 1 : 0) | (box_face(t, bnd) << 1)};
    }
    const v3 d2 = muls(r.dir, 2.0f);
    const float qa = dot(r.dir, r.dir);
    const float qa2 = 2.0f * qa, qa4 = 4.0f * qa;
    const float floor = root_floor(qa2);
    if (kPrimary && S.cull) {
        // spheres whose conservative footprint overlaps this wave's tile
        const int lane = threadIdx.x & 63;
        for (int base = 0; base < S.ns; base += 64) {
            const int k = base + lane;
            bool cand = false;
            if (k < S.ns) {
                const int4 bb = S.sph_px[k];
                cand = !(bb.y < S.tx0 || bb.x > S.tx1 || bb.w < S.ty0 || bb.z > S.ty1);
            }
            uint64_t mask = wave_ballot(cand);
            while (mask) {
                const int s = base + __builtin_ctzll(mask);
                mask &= mask - 1;
                RT_STAT(6, true);
                // (lean views: the camera terms computed here, as for secondary rays)
                test_sphere(S, s, r.start, d2, qa2, qa4, floor, S.cam_terms != 0, h);
            }
        }
    } else if (!kPrimary && S.cull && S.nbvh > 0) {
        bool walk = valid;  // lanes that walk the BVH below
        if (S.olist) {
            // A ray that starts on sphere `origin` tests the candidates of its
            // direction's texel in that sphere's list (rt_internal.h
            // kOListSlots: every sphere it can hit, its own first, then by a
            // lower bound of the hit distance) instead of walking the BVH; it
            // stops once its closest hit lies below the next stored bound. A
            // lane whose list goes on past the record (and whose hit lies
            // above the next bound), or without an origin sphere or a usable
            // direction, walks the BVH. The candidates are a superset of the
            // spheres the ray can hit and the closest hit is order-independent
            // (explicit index tie-break): the result is the walk's, bit for
            // bit. CPU model (tools/model/origin_list_model.py, config 4):
            // 30.3 BVH node iterations + sphere passes per wave call become
            // 4.9 list passes + 7.1 for the lanes left to the BVH.
            const int tex = (valid && origin >= 0) ? direction_texel(kOListTexels, r.dir) : -1;
            uint4 ra = make_uint4(0u, 0u, 0u, 0u), rb = ra;
            if (tex >= 0) {
                const uint4 *rec =
                    S.olist + 2 * (static_cast<size_t>(origin) * (6 * kOListTexels * kOListTexels) + tex);
                ra = rec[0];
                rb = rec[1];
            }
            const uint32_t cnt = ra.x & 0xFFu;
            uint32_t n = cnt < static_cast<uint32_t>(kOListSlots) ? cnt : static_cast<uint32_t>(kOListSlots);
#pragma unroll
            for (int i = 0; i < kOListSlots; ++i) {  // i: a constant after unrolling (byte i + 1 of the record)
                if (!wave_any(static_cast<uint32_t>(i) < n)) break;
                RT_STAT(14, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                if (i == 8 || i == 16) {  // the stored bounds of candidates 8 and 16
                    const uint32_t q = i == 8 ? (rb.z >> 16) : (rb.w & 0xFFFFu);
                    if (h.t < static_cast<float>(q) * kOListBoundUnit) n = 0;
                }
                if (static_cast<uint32_t>(i) < n) {
                    RT_STAT(15, true);
                    const uint32_t word = (i + 1) < 4 ? ra.x : (i + 1) < 8 ? ra.y : (i + 1) < 12 ? ra.z
                                        : (i + 1) < 16 ? ra.w : (i + 1) < 20 ? rb.x : (i + 1) < 24 ? rb.y : rb.z;
                    const int sl = static_cast<int>((word >> (8 * ((i + 1) & 3))) & 0xFFu);
                    test_sphere(S, sl, r.start, d2, qa2, qa4, floor, false, h);
                }
            }
            const float bend = static_cast<float>(rb.w >> 16) * kOListBoundUnit;
            walk = valid && (tex < 0 || (cnt > static_cast<uint32_t>(kOListSlots) && !(h.t < bend)));
        }
        // secondary rays: stackless depth-first BVH walk (skip links)
        // (testing first the sphere a secondary ray starts inside — a
        // refraction into or a reflection inside a sphere — changed no node
        // test: the ordered walk reaches its leaf first anyway; config 4
        // +1.3 %, config 3 +1.6 %, r03c)
        const RayInv q = ray_inv(r);
        int node = walk ? 0 : -1;
        // while-while: each lane walks nodes until it holds a leaf (or its
        // walk ends); then the wave tests the spheres of every held leaf
        // together, so the sphere tests of lanes that reach leaves on
        // different iterations do not each cost the whole wave a pass.
        // Tried and measured slower (r02, tools/ab.py; the extra registers
        // spill at the 80-VGPR cap): reading both successors' records before
        // the node test (config 4 22.0 -> 24.7 ms, config 3 1.058 -> 1.128 ms);
        // loading the wide-mask words in phong ahead of the shading math
        // (22.0 -> 23.6 ms, 1.058 -> 1.149 ms); a speculative second leaf per
        // lane while other lanes look for their first (config 4 18.0 -> 19.0
        // ms, config 3 1.018 -> 1.060 ms).
        int held = 0;  // (count << 24) | first sphere of the held leaf
        // the ray's octant picks its traversal order (nearer child first)
        const int oct = (r.dir.x < 0.0f ? 1 : 0) | (r.dir.y < 0.0f ? 2 : 0) | (r.dir.z < 0.0f ? 4 : 0);
        while (wave_any(node >= 0)) {
            while (node >= 0 && held == 0) {
                RT_STAT(3, true);
                RT_STAT(4, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                const float4 lo = S.bvh[2 * node], hi = S.bvh[2 * node + 1];
                const int leaf = __float_as_int(hi.w);
                const uint32_t link = S.blink[node * kBvhOctants + oct];
                if (node_hit(q, lo, hi, h.t)) {
                    held = leaf;
                    node = static_cast<int16_t>(link & 0xFFFFu);
                } else {
                    node = static_cast<int16_t>(link >> 16);
                }
            }
            if (held) {
                RT_STAT(5, true);
                const int first = held & 0xFFFFFF, count = held >> 24;
                for (int s = first; s < first + count; ++s) test_sphere(S, s, r.start, d2, qa2, qa4, floor, false, h);
                held = 0;
            }
        }
    } else {
        for (int s = 0; s < S.ns; ++s) test_sphere(S, s, r.start, d2, qa2, qa4, floor, kPrimary && S.cam_terms != 0, h);
    }
    if (!valid) h.obj = -1;
    return h;
}
template <bool kPrimary>
__device__ __forceinline__ Hit closest(const Scene &S, const Ray &r, bool valid, int origin = -1) {
    RT_CYC(kPrimary ? kCycClosest1 : kCycClosest2);
    const Hit h = closest_impl<kPrimary>(S, r, valid, origin);
    RT_CYC_AFTER(kCycWalk, h.t);
    return h;
}

// Mask of the texel of direction u in a light's cube map (rt_internal.h,
// kMaskMaxSpheres): face = the largest |component| (ties to z, then y), column
// / row from the hardware's face coordinates over it. Approximate
// arithmetic: the host's texel cones carry a margin far above its error. A
// direction without a usable largest component gets every sphere.
// Texel of direction u, or -1.
__device__ __forceinline__ int direction_texel(int n, v3 u) {
    // the cube-map instructions: face id (+x, -x, +y, -y, +z, -z; z, then y
    // wins a tie), the face coordinates sc, tc and twice the major component
    // (rt_scene.cpp mask_cones lays the texels out in the same coordinates)
    const float face = __builtin_amdgcn_cubeid(u.x, u.y, u.z);
    const float sc = __builtin_amdgcn_cubesc(u.x, u.y, u.z), tc = __builtin_amdgcn_cubetc(u.x, u.y, u.z);
    const float ma = fabsf(__builtin_amdgcn_cubema(u.x, u.y, u.z));  // 2 |major|
    // (computed in every lane and selected instead of the early return:
    // measured even, r02k)
    if (!(ma > 2e-20f && ma < 2e30f)) return -1;
    const float h = static_cast<float>(n) * __builtin_amdgcn_rcpf(ma);
    const int col = min(max(static_cast<int>(floorf(sc * h + 0.5f * n)), 0), n - 1);
    const int row = min(max(static_cast<int>(floorf(tc * h + 0.5f * n)), 0), n - 1);
    return (static_cast<int>(face) * n + row) * n + col;
}
// (nbits: the mask's sphere and box bits)
__device__ __forceinline__ uint64_t direction_mask(const void *tab, int n, int bytes, v3 u, int nbits) {
    const int at = direction_texel(n, u);
    if (at < 0) return nbits >= 64 ? ~uint64_t{0} : (uint64_t{1} << nbits) - 1u;
    if (bytes == 8) return static_cast<const uint64_t *>(tab)[at];
    return bytes == 2 ? static_cast<const uint16_t *>(tab)[at] : static_cast<const uint32_t *>(tab)[at];
}

// Shadow query (:807-819) for the lanes with `need`: is there an object with
// 0 < t < 1 along start + t * dir? (equivalent to the closest hit's t < 1).
// Tried and measured no gain (r02, tools/ab.py): dropping the lane's own
// sphere from its mask when the segment provably starts outside it and
// leads away from it (config 2 +1-4 %, configs 3-4 +6-12 %, also after the
// frames shrank: the extra registers spill), and skipping the square root
// for spheres behind an outside origin (within 0.5 %), also as a separate
// first pass over the LDS mask that drops such candidates before the exact
// walk (config 2 even).
// p = the shaded point, L = the light. Called with all lanes active.
__device__ __forceinline__ bool occluded_impl(const Scene &S, v3 start, v3 dir, v3 p, v3 L, int light, int slot,
                                              uint64_t mask, bool need, const uint4 *pre) {
    bool hit = false;
    const uint32_t light_bit = light < 32 ? 1u << light : 0u;
    RT_STAT(7, need);
    RT_STAT(10, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
    // the LDS masks' box bits (round 6; `mask` is the lane's LDS mask where
    // there are no wide masks): a lane whose bit of box b is clear cannot be
    // occluded by it (its bounding sphere's cone from the light, the spheres'
    // test), and a wave none of whose lanes has the bit skips the box
    const bool box_bits = S.dmask_box != 0 && S.cull && S.dmask != nullptr && S.gmask == nullptr;
    for (int b = 0; b < S.nb; ++b) {
#ifdef RT_ABLATE_BOX_SHADOW
        if (!S.room && b > 0) continue;  // (timing probe: wrong images by design)
#endif
        if (box_bits || S.cbplane) {
            bool cand = need && !hit;
            if (box_bits) cand = cand && ((mask >> (S.ns + b)) & 1u) != 0u;
            if (S.cbplane) {
                // the segment's start beyond the plane of the box's face that
                // the light lies beyond: both ends beyond, no occluder (the
                // host's margins cover this float evaluation, rt_scene.cpp)
                const float4 pl = cload(S.cbplane + (b * S.nl + light));
                cand = cand && !(start.x * pl.x + start.y * pl.y + start.z * pl.z + pl.w > 0.0f);
            }
            if (!wave_any(cand)) continue;
            const bool occ = box_occludes(cload(S.cbox + b), start, dir, light_bit, S.room != 0, S.cull != 0);
            hit = hit | (cand & occ);
            continue;
        }
        // every lane tests (no divergent branch around the test; lanes
        // without the query or already shadowed keep their flag)
        const bool occ = box_occludes(cload(S.cbox + b), start, dir, light_bit, S.room != 0, S.cull != 0);
        hit = hit | (need & occ);
    }
    if (!wave_any(need && !hit)) return hit;
    if (S.cull && !S.gmask && S.dmask) {
        // the LDS-mask walk (see below) with the ray's quadratic terms
        // computed only when some lane of the wave has a candidate (most
        // shadow queries of a wave have none: config 2 -1 %)
        // (the sphere bits: the box bits above them dropped)
        const uint64_t m64 = (need && !hit ? mask : 0u) & (box_bits ? (uint64_t{1} << (S.ns & 63)) - 1u : ~uint64_t{0});
        if (!wave_any(m64 != 0u)) return hit;
        const v3 d2 = muls(dir, 2.0f);
        const float qa = dot(dir, dir);
        const float qa2 = 2.0f * qa, qa4 = 4.0f * qa;
        const float floor = root_floor(qa2);
        const auto test = [&](int s) {
            RT_STAT(8, true);
            const float4 c = S.sph[s];
            const v3 oc = sub(start, mk(c.x, c.y, c.z));
            hit = sphere_blocks(dot(d2, oc), dot(oc, oc) - c.w, qa2, qa4, floor);
        };
        if (S.dmask_bytes == 8) {
            uint64_t cand = m64;
            while (wave_any(cand != 0u)) {
                if (cand) {
                    test(__builtin_ctzll(cand));
                    cand = hit ? 0u : cand & (cand - 1u);
                }
            }
        } else {  // 32-bit masks: half the bit arithmetic
            uint32_t cand = static_cast<uint32_t>(m64);
            while (wave_any(cand != 0u)) {
                RT_STAT(12, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                if (cand) {
                    test(__builtin_ctz(cand));
                    cand = hit ? 0u : cand & (cand - 1u);
                }
            }
        }
        return hit;
    }
    const v3 d2 = muls(dir, 2.0f);
    const float qa = dot(dir, dir);
    const float qa2 = 2.0f * qa, qa4 = 4.0f * qa;
    const float floor = root_floor(qa2);
    auto exact = [&](int s) {
        if (need && !hit) {
            RT_STAT(8, true);
            const float4 c = S.sph[s];
            const v3 oc = sub(start, mk(c.x, c.y, c.z));
            const float qb = dot(d2, oc);
            const float qc = dot(oc, oc) - c.w;
            hit = sphere_blocks(qb, qc, qa2, qa4, floor);
        }
    };
    // the same test for the mask walks, whose candidate words are already
    // empty for lanes without the query or with a hit
    auto exact_cand = [&](int s) {
        RT_STAT(8, true);
        const float4 c = S.sph[s];
        const v3 oc = sub(start, mk(c.x, c.y, c.z));
        const float qb = dot(d2, oc);
        const float qc = dot(oc, oc) - c.w;
        hit = sphere_blocks(qb, qc, qa2, qa4, floor);
    };
    if (!S.cull) {
        for (int s = 0; s < S.ns; ++s) {
            if (!wave_any(need && !hit)) break;
            exact(s);
        }
        return hit;
    }
    if (S.gmask) {
        // wide masks from L2: `mask` holds the texel (-1: every sphere)
        const int texel = static_cast<int>(static_cast<int64_t>(mask));
        const int per_light = 6 * kGMaskTexels * kGMaskTexels;
        bool ask = need;  // lanes that walk the mask words below
        if (S.glist) {
            // the texel's candidate list (rt_internal.h kGListMax): one 16-B
            // load, then one pass per candidate of the longest list — a
            // wave no longer pays, per mask word, for the lane with the most
            // candidates in that word (against the words alone: config 4
            // 16.63 -> 14.83 ms, config 3 0.940 -> 0.896 ms, r03c; the
            // wave's candidate passes per tile 68.8 -> 52.5)
            uint4 rec = make_uint4(0u, 0u, 0u, 0u);
            if (pre) {
                if (need && !hit && texel >= 0) rec = *pre;
            } else if (need && !hit && texel >= 0) {
                rec = S.glist[static_cast<size_t>(slot) * per_light + texel];
            }
            uint32_t cnt = rec.x & 0xFFu;
            const bool wide = need && !hit && (texel < 0 || cnt == kGListOverflow);
            if (wide) cnt = 0u;
            for (uint32_t i = 1; wave_any(i <= cnt); ++i) {  // i: wave-uniform
                RT_STAT(9, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                if (i <= cnt) {
                    const uint32_t word = i < 4 ? rec.x : (i < 8 ? rec.y : (i < 12 ? rec.z : rec.w));
                    exact_cand(static_cast<int>((word >> (8 * (i & 3u))) & 0xFFu));
                    if (hit) cnt = 0u;
                }
            }
            if (!wave_any(wide)) return hit;
            ask = wide;  // more than kGListMax candidates, or every sphere: the words
        }
        // every word of the texel requested up front (independent L2 loads
        // in flight together), then walked word by word (one walk over all
        // words at once measured slower: config 3 +7 %, config 4 even)
        constexpr int kMaxWords = kGMaskMaxSpheres / 64;
        uint64_t words[kMaxWords];
        const uint64_t *row = S.gmask + (static_cast<size_t>(slot) * per_light + (texel >= 0 ? texel : 0)) * S.gwords;
#pragma unroll
        for (int w = 0; w < kMaxWords; ++w) {
            // (loading in every lane and selecting measured slower: config 4
            // 16.57 -> 17.16 ms, config 3 +2 %)
            words[w] = (w < S.gwords && ask && !hit && texel >= 0) ? row[w] : ~uint64_t{0};
        }
#pragma unroll
        for (int w = 0; w < kMaxWords; ++w) {
            if (w >= S.gwords) break;
            uint64_t cand = 0u;
            if (ask && !hit) {
                cand = words[w];
                const int rest = S.ns - 64 * w;
                if (rest < 64) cand &= (uint64_t{1} << rest) - 1u;
            }
            while (wave_any(cand != 0u)) {
                RT_STAT(9, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                if (cand) {
                    exact_cand(64 * w + __builtin_ctzll(cand));
                    cand = hit ? 0u : cand & (cand - 1u);
                }
            }
            if (!wave_any(ask && !hit)) break;
        }
        return hit;
    }
    if (S.dmask) {
        // the spheres that may block this lane's ray: `mask`, the texel mask
        // of its direction from the light (looked up by the caller); each
        // lane walks its own mask (usually empty)
        if (S.dmask_bytes == 8) {
            uint64_t cand = need && !hit ? mask : 0u;
            while (wave_any(cand != 0u)) {
                if (cand) {
                    exact_cand(__builtin_ctzll(cand));
                    cand = hit ? 0u : cand & (cand - 1u);
                }
            }
        } else {  // 32-bit masks: half the bit arithmetic
            uint32_t cand = need && !hit ? static_cast<uint32_t>(mask) : 0u;
            while (wave_any(cand != 0u)) {
                RT_STAT(12, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
                if (cand) {
                    exact_cand(__builtin_ctz(cand));
                    cand = hit ? 0u : cand & (cand - 1u);
                }
            }
        }
        return hit;
    }
    // The wave's shadow segments lie within 0.01 (the start offset, :808) of
    // the segments [L, p_i]: all inside the cone from L with axis `ax` and
    // half-angle acos(cmin), within distance `maxlen` of L. A sphere that
    // misses that cone by more than the margins cannot occlude any of them.
    const bool act = need && !hit;
    const v3 u = sub(p, L);
    const float ul = fsqrt_approx(dot(u, u));
    const v3 uh = ul > 0.0f ? muls(u, __builtin_amdgcn_rcpf(ul)) : mk(0.0f, 0.0f, 0.0f);
    // cone axis: the direction of the first active lane
    const int lead = __builtin_ctzll(wave_ballot(act));
    const v3 ax = mk(lane_value(uh.x, lead), lane_value(uh.y, lead), lane_value(uh.z, lead));
    const float cmin = wave_min(act ? dot(ax, uh) : 1.0f);
    const float maxlen = wave_max(act ? ul : 0.0f);
    const float al = dot(ax, ax);
    const bool angular = cmin > 0.0f && al > 0.5f;  // cone narrower than 90 degrees, axis a unit vector
    if (!angular && S.nbvh > 0) {
        // incoherent shadow rays (no useful common cone): per-lane any-hit
        // walk of the sphere BVH over the segment t in (0, 1)
        const RayInv q = ray_inv({start, dir});
        int node = act ? 0 : -1;
        while (node >= 0) {
            const float4 lo = S.bvh[2 * node], hi = S.bvh[2 * node + 1];
            const int leaf = __float_as_int(hi.w);
            if (node_hit(q, lo, hi, 1.0f)) {
                if (leaf) {
                    const int first = leaf & 0xFFFFFF, count = leaf >> 24;
                    for (int s = first; s < first + count; ++s) exact(s);
                    node = hit ? -1 : __float_as_int(lo.w);
                } else {
                    node = node + 1;
                }
            } else {
                node = __float_as_int(lo.w);
            }
        }
        return hit;
    }
    const float sth = fsqrt_approx(fmaxf(0.0f, 1.0f - cmin * cmin));
    const int lane = threadIdx.x & 63;
    const ShadowCone *cones = S.cone ? S.cone + light * S.ns : nullptr;
    for (int base = 0; base < S.ns; base += 64) {
        const int k = base + lane;
        bool cand = false;
        if (k < S.ns) {
            // the sphere's cone from the light: precomputed (host, float64) or
            // derived here with approximate sqrt / rcp (same margins)
            float far, sph, cph;
            v3 v;
            bool near;
            if (cones) {
                const ShadowCone &sc = cones[k];
                v = mk(sc.v[0], sc.v[1], sc.v[2]);
                far = sc.far;
                sph = sc.sph;
                cph = sc.cph;
                near = sc.near != 0.0f;
            } else {
                const float4 c = S.sph[k];
                const float rad = __int_as_float(S.smeta[k].z);
                v = sub(mk(c.x, c.y, c.z), L);
                const float d = fsqrt_approx(dot(v, v));
                const float rp = rad + 0.021f + 1e-3f * d;  // 0.01 start offset + margins
                near = d <= rp;
                far = d - rp;
                const float id = __builtin_amdgcn_rcpf(d);
                v = muls(v, id);
                sph = rp * id;
                cph = fsqrt_approx(fmaxf(0.0f, 1.0f - sph * sph));
            }
            if (near) {
                cand = true;  // light inside the inflated sphere
            } else if (far > maxlen) {
                cand = false;  // beyond every shaded point
            } else if (!angular) {
                cand = true;
            } else {
                const float cos_lim = cmin * cph - sth * sph;  // cos(theta + phi)
                cand = !(dot(ax, v) < cos_lim - 1e-3f);
            }
        }
        uint64_t mask = wave_ballot(cand);
        while (mask) {
            const int s = base + __builtin_ctzll(mask);
            mask &= mask - 1;
            exact(s);
            if (!wave_any(need && !hit)) return hit;
        }
    }
    return hit;
}

__device__ __forceinline__ bool occluded(const Scene &S, v3 start, v3 dir, v3 p, v3 L, int light, int slot,
                                         uint64_t mask, bool need, const uint4 *pre = nullptr) {
    RT_CYC(kCycShadow);
    const bool hit = occluded_impl(S, start, dir, p, L, light, slot, mask, need, pre);
    RT_CYC_AFTER(kCycPhong, hit ? 1 : 0);
    return hit;
}

struct Collision {
    v3 p, n;
    bool inside;
    int material;
};

// Build the collision record of the winning object (:628-637, :686-721).
// A box's slab distances come with the hit (the closest-hit loop computed
// them); its t is the slab test's intersection distance.
template <bool kPrimary>
__device__ __forceinline__ Collision resolve_impl(const Scene &S, const Ray &r, const Hit &h, bool valid) {
    Collision c;
    c.p = mk(0.0f, 0.0f, 0.0f);
    c.n = mk(0.0f, 0.0f, 1.0f);
    c.inside = false;
    c.material = 0;
    if (!valid) return c;
    if (h.slot >= 0) {
        const float4 sp = S.sph[h.slot];
        const v3 pos = mk(sp.x, sp.y, sp.z);
        c.material = S.smeta[h.slot].y;
        c.p = add(r.start, muls(r.dir, h.t));
        c.n = normalize(sub(c.p, pos));
        c.inside = h.info & 1;
        if (c.inside) c.n = muls(c.n, -1.0f);  // leaving the sphere: flip (:634-637)
    } else {
        const BoxRec &B = S.box[~h.slot];
        c.material = B.material;
        v3 rs;
        if (kPrimary) {
            const float4 bc = S.box_cam[~h.slot];
            rs = mk(bc.x, bc.y, bc.z);
        } else {
            rs = xform_point(B.w2l, r.start);
        }
        const v3 rd = box_dir(B, r.dir);
        c.inside = h.info & 1;
        const int face = h.info >> 1;  // box_face, decided in the scan
        v3 n = mk(face == 0 ? 1.0f : 0.0f, face == 1 ? 1.0f : 0.0f, face == 2 ? 1.0f : 0.0f);
        if (comp(rd, face) > 0.0f) n = muls(n, -1.0f);
        const float *N = B.nrm;
        c.n = mk(N[0] * n.x + N[1] * n.y + N[2] * n.z, N[3] * n.x + N[4] * n.y + N[5] * n.z,
                 N[6] * n.x + N[7] * n.y + N[8] * n.z);
        const v3 lp = add(rs, muls(rd, h.t));
        c.p = xform_point(B.l2w, lp);
    }
    return c;
}
template <bool kPrimary>
__device__ __forceinline__ Collision resolve(const Scene &S, const Ray &r, const Hit &h, bool valid) {
    RT_CYC(kCycResolve);
    const Collision c = resolve_impl<kPrimary>(S, r, h, valid);
    RT_CYC_AFTER(kCycWalk, c.p.x);
    return c;
}

// Development probe (timing builds only, tools/phase_trace.py): lane 0 of
// every wave of a depth-0 tiled launch records the 100 MHz real-time clock
// at fixed points of its life.
#ifdef RT_PHASE_TRACE
constexpr unsigned kPhaseWaves = 1u << 17;
__device__ unsigned long long rt_phase_buf[kPhaseWaves * 16];
#define RT_PHASE(k)                                                                                        \
    do {                                                                                                    \
        const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();                                   \
        const unsigned wg_ = (blockIdx.y * gridDim.x + blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); \
        if ((threadIdx.x & 63) == 0 && wg_ < kPhaseWaves) rt_phase_buf[wg_ * 16 + (k)] = now_;              \
    } while (0)
// the clock read after `v` is available (a branch on it orders the read)
#define RT_PHASE_AFTER(k, v)                     \
    do {                                         \
        if ((v) != -12345) RT_PHASE(k);      \
    } while (0)
#else
#define RT_PHASE_AFTER(k, v) \
    do {                     \
    } while (0)
#define RT_PHASE(k) \
    do {            \
    } while (0)
#endif

// ads_phong_lighting (:789-840). Called with all lanes active.
// kUni (RT_UNIFORM_MAT probe, depth 0): every lane with a hit has material
// `umat`, and the material and light x material records come by scalar
// loads (SGPRs) instead of per-lane LDS gathers.
template <bool kUni = false>
__device__ __forceinline__ v3 phong_impl(const Scene &S, const Ray &r, const Collision &c, bool valid, int umat = 0) {
#if defined(RT_UNIFORM_MAT) && !defined(RT_UNIFORM_MAT_LM_ONLY)
    const MatRec m = kUni ? cload(S.cmat + umat) : S.mat[c.material];
#else
    const MatRec &m = S.mat[c.material];
#endif
    float4 dif = make_float4(0.0f, 0.0f, 0.0f, 0.0f), spe = dif;
    const v3 view = normalize_unit(muls(r.dir, -1.0f));  // ray directions are unit vectors up to rounding
    int slot = -1;  // index among the live lights (direction masks)
    for (int j = 0; j < S.nl; ++j) {
        const LightRec L = cload(S.clight + j);
        if (L.dead != 0.0f) continue;  // no direct term for any material (host-checked)
        ++slot;
        const v3 lpos = mk(L.pos[0], L.pos[1], L.pos[2]);
        const v3 sdir = sub(lpos, c.p);  // the shadow ray's direction (:809)
        // wide masks: the texel's candidate list requested before the shading
        // math, for every lane with a hit, so its L2 latency overlaps the
        // math (config 4 14.92 -> 14.77 ms, config 3 0.893 -> 0.889 ms, r03b)
        int ptexel = -1;
        uint4 pre = make_uint4(0u, 0u, 0u, 0u);
        if (S.glist) {
            ptexel = valid ? direction_texel(kGMaskTexels, muls(sdir, -1.0f)) : -1;
            if (ptexel >= 0) pre = S.glist[static_cast<size_t>(slot) * 6 * kGMaskTexels * kGMaskTexels + ptexel];
        }
        const v3 ldir = normalize(sdir);
        const float cos_theta = dot(ldir, c.n);
        // reflect(-ldir, n) needs dot(n, -ldir), which is -cos_theta (exact
        // negation, commuted products) except that an exactly-zero dot may
        // differ in the sign of its zero; that only flips signs of zero
        // components of lref, which change cos_phi at most by the sign of a
        // zero, and max(cos_phi, 0) is +0 for both: the result is identical
        const v3 nl = muls(ldir, -1.0f);
        const v3 lref = normalize_unit(sub(nl, muls(c.n, 2.0f * -cos_theta)));
        const float cos_phi = dot(view, lref);
#ifdef RT_UNIFORM_MAT
        const LightMatRec q = kUni ? cload(S.clm + (umat * S.nl + j)) : S.lm[c.material * S.nl + j];
#else
        const LightMatRec &q = S.lm[c.material * S.nl + j];
#endif
        const float kd = gmax(cos_theta, 0.0f);
        // pow(0, s) is +0 for s > 0 (log2 = -inf, exp2 clamps to 2^-127
        // scaled to 0): skip the polynomials when no lane needs them
        const float xs = gmax(cos_phi, 0.0f);
        // flags combined with & and |, not && and ||: short-circuit evaluation
        // of LDS-loaded operands compiled to nested divergent branches
        const bool need_pow = !((xs == 0.0f) & (m.shininess > 0.0f));
        float ks = 0.0f;
        if (wave_any(need_pow && valid)) ks = need_pow ? glsl_pow_cos(xs, m.shininess) : 0.0f;
        const float4 nd = make_float4(dif.x + q.ld_md[0] * kd, dif.y + q.ld_md[1] * kd, dif.z + q.ld_md[2] * kd,
                                      dif.w + q.ld_md[3] * kd);
        const float4 ns = make_float4(spe.x + q.ls_ms[0] * ks, spe.y + q.ls_ms[1] * ks, spe.z + q.ls_ms[2] * ks,
                                      spe.w + q.ls_ms[3] * ks);
        // the shadow ray matters only if the light's term can change the sums
        // (host flags, rt_scene.cpp: with a tame material a zero factor or a
        // zero product adds +-0 to sums that are never -0)
        const bool changes = (q.always != 0) | ((kd != 0.0f) & (q.d_nz != 0)) | ((ks != 0.0f) & (q.s_nz != 0));
        const bool need = valid && changes;
        if (j == 1) RT_PHASE(5);
#ifdef RT_ABLATE_SHADOW
        if (need) { dif = nd; spe = ns; }
        continue;
#endif
        if (wave_any(need)) {
            // its direction-mask texel (p - L = -sdir), looked up only where
            // some lane casts the shadow ray (ahead of the shading math, to
            // overlap the LDS read, it measured slower: config 3 0.978 vs 0.960
            // ms, config 2 39.0 vs 38.6 us per frame, config 4 +0.5 %)
            uint64_t smask = 0u;  // LDS masks: the mask; wide masks: the texel
            // the LDS mask for every lane of the wave (occluded ignores the
            // mask of a lane without the query): no divergent branch around
            // the lookup (config 2 -1 %); the wide-mask texel only where the
            // query is cast (unguarded, config 3 +0.7 %)
            if (S.glist)
                smask = static_cast<uint64_t>(static_cast<int64_t>(ptexel));
            else if (S.gmask && need)  // wide masks win where both exist (as in occluded)
                smask = static_cast<uint64_t>(static_cast<int64_t>(direction_texel(kGMaskTexels, muls(sdir, -1.0f))));
            else if (S.dmask && !S.gmask)
                smask = direction_mask(S.dmask + slot * 6 * S.dmask_n * S.dmask_n * S.dmask_bytes, S.dmask_n,
                                       S.dmask_bytes, muls(sdir, -1.0f), S.ns + (S.dmask_box ? S.nb : 0));
            const bool shadowed = occluded(S, add(c.p, muls(c.n, 0.01f)), sdir, c.p, lpos, j, slot, smask, need,
                                           S.glist ? &pre : nullptr);
            if (need && !shadowed) {
                dif = nd;
                spe = ns;
            }
        }
    }
    RT_PHASE(6);
    // phong = ambient + diffuse + specular + emissive; return rgb * a (:837-839)
    const float px = ((m.amb_sum[0] + dif.x) + spe.x) + m.emissive[0];
    const float py = ((m.amb_sum[1] + dif.y) + spe.y) + m.emissive[1];
    const float pz = ((m.amb_sum[2] + dif.z) + spe.z) + m.emissive[2];
    const float pw = ((m.amb_sum[3] + dif.w) + spe.w) + m.emissive[3];
    return mk(px * pw, py * pw, pz * pw);
}
__device__ __forceinline__ v3 phong(const Scene &S, const Ray &r, const Collision &c, bool valid) {
    RT_CYC(kCycPhong);
    const v3 col = phong_impl(S, r, c, valid);
    RT_CYC_AFTER(kCycWalk, col.x);
    return col;
}

// ---- recursive_raytrace (:1071-1105) -----------------------------------
// The stack machine (:848-1065) evaluates, per ray: closest hit; Phong; if
// depth remains, the reflection subtree, then the refraction subtree; then
// mix(mix(phong, R, reflectivity), T, transparency), with a missed ray black
// (:962-963) and each mix only when that child was spawned (:994, :1027).
//
// Depth 0 is one ray (trace0). Deeper trees run as an explicit depth-first
// walk (trace_tree): every loop iteration traces ONE ray per lane — all lanes
// execute the same closest-hit + shading code whatever their position in
// their own tree — with per-level frames (partial colour and flags, 16 B; the
// pending refraction ray, 24 B, only where both children exist) indexed by
// the lane's own level, which the compiler keeps in scratch (Frames). Lanes
// whose tree is finished ride along with valid = false.
__device__ __forceinline__ v3 trace0(const Scene &S, const Ray &r, bool valid) {
    const v3 black = mk(0.0f, 0.0f, 0.0f);
    RT_PHASE(2);
    const Hit h = closest<true>(S, r, valid);
    RT_PHASE(3);
    const bool hit = valid && h.obj >= 0;
    if (!wave_any(hit)) return black;  // per-wave early out
    const Collision c = resolve<true>(S, r, h, hit);
    RT_PHASE(4);
#ifdef RT_ABLATE_PHONG
    const v3 col = add(c.p, c.n);
#elif defined(RT_UNIFORM_MAT)
    // the first hit lane's material; the scalar-record instance when every
    // hit lane shares it (97 % of config 2's wave tiles)
    const uint64_t hb = wave_ballot(hit);
    const int umat = __builtin_amdgcn_readlane(c.material, static_cast<int>(__builtin_ctzll(hb)));
    v3 col;
    if (wave_all(!hit || c.material == umat)) col = phong_impl<true>(S, r, c, hit, umat);
    else col = phong(S, r, c, hit);
#else
    const v3 col = phong(S, r, c, hit);
#endif
    return sel(hit, col, black);
}

struct Frame {
    v3 col;       // phong, then mix(phong, R, rho) once the reflection returned
    v3 rs, rd;    // pending refraction ray (:1010-1023)
    int flags;    // 1: refraction spawned; 2: waiting for the reflection; 4: for the refraction;
                  // | (the hit sphere's slot + 1) << 11 (the refraction child's origin sphere)
                  // | material << 3 (rho and tau read back from it: a 40-B frame instead of
                  // 48, config 4 18.68 -> 18.26 ms, config 3 1.022 -> 1.000 ms; the flags
                  // beside the colour, so a pop reads one 16-B word, measured even, r03h)
};

#ifdef RT_ABLATE_FRAMES
// Timing-only ablation (wrong images by design): only the walk's flags are
// kept (4 bits per level in one register); colours and pending rays are not
// stored, so the scratch traffic of the frames disappears while the walk
// visits the same nodes.
template <int N>
struct Frames {
    uint32_t bits = 0;
    __device__ __forceinline__ Frame get(int level) const {
        Frame f;
        f.col = mk(0.0f, 0.0f, 0.0f);
        f.rs = mk(0.0f, 0.0f, 0.0f);
        f.rd = mk(0.0f, 0.0f, 1.0f);
        f.flags = static_cast<int>((bits >> (4 * level)) & 7u);
        return f;
    }
    __device__ __forceinline__ void set(int level, const Frame &v) {
        bits = (bits & ~(15u << (4 * level))) | ((static_cast<uint32_t>(v.flags) & 7u) << (4 * level));
    }
    __device__ __forceinline__ void set_pending(int, const Frame &) {}
    __device__ __forceinline__ void pending(int, Ray &r) const { r.start = mk(0.0f, 0.0f, 0.0f); r.dir = mk(0.0f, 0.0f, 1.0f); }
};
template <int N>
struct FramesReal {
#else
template <int N>
struct Frames {
#endif
    // Per-level frames, indexed by the lane's level (the compiler keeps them in
    // scratch): the colour and flags (16 B) of every node with children, and
    // the pending refraction ray (24 B) only for a node whose refraction child
    // waits behind its reflection child, read back when that child starts.
    // Round 6: against one 40-B frame per level (a push storing, a pop loading
    // all of it), config 4 10.59 -> 10.32 ms, config 3 0.701 -> 0.692 ms, 7
    // views 0.660 -> 0.643 ms per frame, bit-identical (profiles/r06b_ab.log);
    // walk_model: 888 -> 521 frame bytes per config-4 pixel. (Round 2 had
    // measured this split slower, config 4 16.93 -> 17.12 ms, on a walk with
    // per-level select chains.) Earlier: per-level selects read every level's
    // frame (config 4 18.80 vs 19.08 ms, depth-4 scratch 292 vs 400 B per
    // lane); what the frames cost at most: RT_ABLATE_FRAMES, which keeps only
    // the flags, rendered config 4 in 11.4 instead of 16.6 ms (round 2); the top
    // levels in LDS, in 768-thread queued groups, measured config 3 -1 %,
    // config 4 +2 %.
    struct Head {
        v3 col;
        int flags;
    };
    Head h[N];
    Ray q[N];
    __device__ __forceinline__ Frame get(int level) const {
        Frame f;
        f.col = h[level].col;
        f.flags = h[level].flags;
        return f;
    }
    __device__ __forceinline__ void set(int level, const Frame &v) { h[level] = Head{v.col, v.flags}; }
    __device__ __forceinline__ void set_pending(int level, const Frame &v) { q[level] = Ray{v.rs, v.rd}; }
    __device__ __forceinline__ void pending(int level, Ray &r) const { r = q[level]; }
};

// `emit(value)` receives each lane's colour when its tree is finished (the
// lane then rides along with valid = false): the caller stores the pixel
// there, so no result registers stay live through the rest of the walk.
template <int kDepth, class Emit>
__device__ __forceinline__ void trace_tree(const Scene &S, Ray ray, bool active, Emit &&emit) {
    const v3 black = mk(0.0f, 0.0f, 0.0f);
    Frames<kDepth> F;
    // the lane's level in its tree (bits 0-7) and, from depth 2, the sphere
    // slot + 1 its ray starts on (bits 8-: 0 for the camera or a box), in one
    // register (a separate origin register spilled 8 B more per lane at the
    // 80-VGPR cap)
    int lv = 0;
    bool done = !active;
    bool first = true;
    while (wave_any(!done)) {
        RT_STAT(11, (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)));
        const bool valid = !done;
        const bool primary = first;
        // (origin lists: depth >= 2 only, S.olist)
        const Hit h = first ? closest<true>(S, ray, valid) : closest<false>(S, ray, valid, kDepth >= 2 ? (lv >> 8) - 1 : -1);
        first = false;
        const bool hit = valid && h.obj >= 0;
        const Collision c = primary ? resolve<true>(S, ray, h, hit) : resolve<false>(S, ray, h, hit);
#ifdef RT_ABLATE_PHONG
        const v3 col = add(c.p, c.n);
#else
        const v3 col = phong(S, ray, c, hit);
#endif
        if (!valid) continue;
        const MatRec &m = S.mat[c.material];
        const int level = lv & 0xFF;
        const bool sr = hit && level < kDepth && m.reflectivity > 0.0f;
        const bool st = hit && level < kDepth && m.transparency > 0.0f;
        if (sr || st) {  // push this node, descend into its first child
            Frame fr;
            fr.col = col;
            fr.rs = sub(c.p, muls(c.n, 0.001f));
            fr.rd = ray.dir;  // (no refraction child: never read)
            // only in waves with a refraction child (every surface of the
            // bench scenes reflects, few refract: config 4 14.68 -> 14.62 ms,
            // config 3 0.881 -> 0.878 ms, r03d)
            if (wave_any(st)) {
                const float ratio = c.inside ? m.eta_out : m.eta_in;  // (:1013-1016, host-divided)
                fr.rd = refract(ray.dir, c.n, ratio);
            }
            // (with the sphere its children start on, + 1, from bit 11: the
            // refraction child's origin when the walk comes back to it)
            const int here = h.slot >= 0 ? h.slot : -1;
            fr.flags = (st ? 1 : 0) | (sr ? 2 : 4) | (c.material << 3) | (kDepth >= 2 ? (here + 1) << 11 : 0);
            F.set(level, fr);
            if (sr && st) F.set_pending(level, fr);  // (read back when the refraction child starts)
            if (sr) {
                ray.start = add(c.p, muls(c.n, 0.001f));
                ray.dir = reflect(ray.dir, c.n);
            } else {
                ray.start = fr.rs;
                ray.dir = fr.rd;
            }
            lv = kDepth >= 2 ? ((here + 1) << 8) | (level + 1) : level + 1;
            continue;
        }
        // this node is finished: fold its colour into its ancestors
        v3 value = hit ? col : black;
        bool next_child = false;
        while ((lv & 0xFF) > 0 && !next_child) {
            Frame fr = F.get((lv & 0xFF) - 1);
            const MatRec &fm = S.mat[(fr.flags >> 3) & 0xFF];
            const float rho = fm.reflectivity, tau = fm.transparency;
            if (fr.flags & 2) {
                fr.col = mix(fr.col, value, rho);
                if (fr.flags & 1) {  // the refraction child comes next
                    fr.flags = (fr.flags & ~7) | 4;
                    F.set((lv & 0xFF) - 1, fr);
                    F.pending((lv & 0xFF) - 1, ray);
                    if constexpr (kDepth >= 2) lv = (lv & 0xFF) | ((fr.flags >> 11) << 8);
                    next_child = true;
                } else {
                    value = fr.col;
                    --lv;
                }
            } else {
                value = mix(fr.col, value, tau);
                --lv;
            }
        }
        if (!next_child) {
            emit(value);
            done = true;
        }
    }
}

// Frame row of a launch's local row: the interleaved shard mapping (block
// `blk` of this shard is block blk * n_shards + shard of the frame). A
// power-of-two block (the bench's 8) takes shifts: the integer division it
// replaces expands to a long VALU / SALU sequence, once per lane and eight
// times per wave tile.
__device__ __forceinline__ int output_row(const LaunchParams &p, int local) {
    if (p.n_shards <= 0) return p.row_begin + local;
    const int b = p.block_rows;
    if ((b & (b - 1)) == 0) {
        const int sh = __builtin_ctz(static_cast<unsigned>(b));
        return (((local >> sh) * p.n_shards + p.shard) << sh) + (local & (b - 1));
    }
    const int blk = local / b;
    return (blk * p.n_shards + p.shard) * b + (local - blk * b);
}

// GL_RGBA8 unorm conversion as the reference's GL applies it: NaN -> 0,
// clamp, v * 255 rounded to nearest even (rt_pack_rgba8)
__device__ __forceinline__ uint32_t unorm8(float v) {
    v = v != v ? 0.0f : gmin(gmax(v, 0.0f), 1.0f);
    return static_cast<uint32_t>(__builtin_rintf(v * 255.0f));
}

// One pixel's colour into the launch's surface (float4 or GL_RGBA8 bytes);
// idx = local_row * width + x (< 2^32: 65536 x 65536 frames at most).
__device__ __forceinline__ void store_pixel(const LaunchParams &p, int z, uint32_t idx, v3 col) {
    const size_t at = static_cast<size_t>(z) * p.n_rows * p.width + idx;
    if (p.out_format == RT_OUTPUT_RGBA8) {  // GL_RGBA8 unorm store of vec4(rgb, 0.0) (main.cpp:223, :404): rt_pack_rgba8
        reinterpret_cast<uint32_t *>(p.out)[at] = unorm8(col.x) | (unorm8(col.y) << 8) | (unorm8(col.z) << 16);
    } else if (p.out_format == RT_OUTPUT_RGB32F) {  // packed float3, the constant alpha dropped
        float *o = reinterpret_cast<float *>(p.out) + 3 * at;
        o[0] = col.x;
        o[1] = col.y;
        o[2] = col.z;
    } else
        p.out[at] = make_float4(col.x, col.y, col.z, 0.0f);
}

// Counter-based sample jitter (Monte-Carlo extension):
// a 32-bit integer hash of (seed, sample, pixel, axis); u in [0, 1) with 24
// bits. Integer-only, so the oracle reproduces it exactly.
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ float jitter_u(uint32_t seed, uint32_t sample, uint32_t pixel, uint32_t axis) {
    uint32_t h = mix32(seed * 0x9E3779B1u + 0x7F4A7C15u);
    h = mix32(h ^ (sample * 0x85EBCA77u));
    h = mix32(h ^ (pixel * 0xC2B2AE3Du + axis));
    return static_cast<float>(h >> 8) * (1.0f / 16777216.0f);
}


// Occupancy target per depth: the recursive kernels (depth >= 2) keep the
// tree walk's frames in scratch either way and hide its latency best at 6
// (the general kernels) or 7 (the wide shapes, round 6) waves per SIMD
// (config 4: 58 -> 37 ms from the uncapped build to 6; config 3: 1.52 ->
// 1.37 ms); depth 0/1 need fewer registers than that anyway.
#ifndef RT_WAVES_PER_EU
#ifndef RT_WPE0
#define RT_WPE0 8  // depth 0 at 64 VGPRs (measured equal to the unconstrained 70: 42.9 us per 1080p frame either way)
#endif
#ifndef RT_WPE_DEEP
#define RT_WPE_DEEP 6
#endif
#ifndef RT_WPE2
// depth 2, general kernel: 7 waves had raised round 3's HBM traffic 2.4 ->
// 4.1 GB per frame and its sustained bench kernel to 1.03 ms against 0.98 (r03c)
#define RT_WPE2 6
#endif
#ifndef RT_WPE_WIDE
// the wide-shape recursive kernels (configs 3-4) at 7 waves (72 VGPRs),
// re-measured on round 6's walk (split frames, origin lists, lean views):
// config 3 (depth 2; 176 B of scratch per lane against 152) 4.538 ->
// 4.418-4.428 ms per 7-frame step in interleaved bench lines (-2.6 %,
// profiles/r06v/), its queued launch then holding 5 views beside the scene;
// config 4 (depth 4; 252 B against 232) +0.8 % while its 24.5 KB of LDS per
// work-group held it at 6 work-groups per CU (profiles/r06u_*), 10.28 ->
// 9.81 ms (-4.6 %) once lean views (20.5 KB) let the seventh in
// (profiles/r06y_ab_lean_views.log); 5 waves +9 %
#define RT_WPE_WIDE 7
#endif
#define RT_WAVES_PER_EU(d, shape) \
    (((d) >= 2 && ((shape) & kShapeWide) != 0) ? RT_WPE_WIDE \
     : (d) == 2 ? RT_WPE2 : ((d) >= 2 ? RT_WPE_DEEP : ((d) == 0 ? RT_WPE0 : 1)))
#endif
#ifndef RT_WPE0_MC
// depth-0 Monte-Carlo kernel (config 5): 6 waves, 80 VGPRs + 16 B scratch:
// 38.9 us per sample frame, against 42.6 at 8 waves (64 VGPRs + 84 B of
// spills reloaded in the sample loop) and 41.2 at 5 (94 VGPRs), r03l
#define RT_WPE0_MC 6
#endif
#define RT_OCCUPANCY \
    __attribute__((amdgpu_waves_per_eu((kAccum && kDepth == 0) ? RT_WPE0_MC : RT_WAVES_PER_EU(kDepth, kShape))))
// Reductions over aligned groups of 8 lanes (DPP: quad butterflies, then the
// half-row mirror); every lane of the group ends with the result.
__device__ __forceinline__ float group8_min(float v) {
    v = fminf(v, dpp<0xB1, 0xF>(v));
    v = fminf(v, dpp<0x4E, 0xF>(v));
    return fminf(v, dpp<0x141, 0xF>(v));
}
__device__ __forceinline__ float group8_max(float v) {
    v = fmaxf(v, dpp<0xB1, 0xF>(v));
    v = fmaxf(v, dpp<0x4E, 0xF>(v));
    return fmaxf(v, dpp<0x141, 0xF>(v));
}

// Per-frame constants of one view, written to LDS: the camera-origin terms of
// every sphere (oc, qc :587-588) and box (local origin :655, strictly-inside
// flag) and every sphere's conservative pixel footprint. Reads the scene from
// the device blob (not from its LDS copy), so it needs no barrier after the
// staging; a sphere's footprint is spread over 8 lanes, one corner of its
// bounding cube each (group-of-8 DPP min / max), to keep the prologue short.
__device__ __forceinline__ void frame_setup(const LaunchParams &p, const FrameView &V, float4 *sph_cam,
                                            int4 *sph_px, float4 *box_cam) {
    const float4 *blob = static_cast<const float4 *>(V.blob ? V.blob : p.scene);
    const v3 origin = mk(V.origin[0], V.origin[1], V.origin[2]);
    const int hw = p.width / 2, hh = p.height / 2;
    const bool cull = V.cull && hw > 0 && hh > 0;
    const float *P = V.proj;
    for (int item = threadIdx.x; item < 8 * p.n_spheres; item += kThreads) {  // whole groups of 8 lanes
        const int s = item >> 3, i = item & 7;
        const float4 c = blob[p.off_spheres + s];
        const float rad = __int_as_float(reinterpret_cast<const int4 *>(blob + p.off_smeta)[s].z);
        // corner i of the (inflated) bounding cube, projected with proj*view
        const float r = rad * 1.001f + 1e-3f;
        const float X = c.x + ((i & 1) ? r : -r), Y = c.y + ((i & 2) ? r : -r), Z = c.z + ((i & 4) ? r : -r);
        const float cw = P[3] * X + P[7] * Y + P[11] * Z + P[15];
        const float cx = P[0] * X + P[4] * Y + P[8] * Z + P[12];
        const float cy = P[1] * X + P[5] * Y + P[9] * Z + P[13];
        const float iw = __builtin_amdgcn_rcpf(cw);  // 2-pixel margin >> its error
        const bool ok_i = cw > 1e-4f && r == r && c.x == c.x && c.y == c.y && c.z == c.z;
        const float x0 = group8_min(cx * iw), x1 = group8_max(cx * iw);
        const float y0 = group8_min(cy * iw), y1 = group8_max(cy * iw);
        const bool ok = group8_min(ok_i ? 1.0f : 0.0f) == 1.0f;  // every corner in front of the camera
        if (i == 0) {
            const v3 oc = sub(origin, mk(c.x, c.y, c.z));
            if (sph_cam) sph_cam[s] = make_float4(oc.x, oc.y, oc.z, dot(oc, oc) - c.w);  // (lean views: none)
            // pixel x <-> NDC (x - hw) / hw (:377); two pixels of margin
            const float fx0 = floorf(x0 * hw + hw) - 2.0f, fx1 = ceilf(x1 * hw + hw) + 2.0f;
            const float fy0 = floorf(y0 * hh + hh) - 2.0f, fy1 = ceilf(y1 * hh + hh) + 2.0f;
            const float lim = 1.0e9f;
            const bool fin = fabsf(fx0) < lim && fabsf(fx1) < lim && fabsf(fy0) < lim && fabsf(fy1) < lim;
            sph_px[s] = cull && ok && fin ? make_int4(static_cast<int>(fx0), static_cast<int>(fx1),
                                                      static_cast<int>(fy0), static_cast<int>(fy1))
                                          : make_int4(INT_MIN / 2, INT_MAX / 2, INT_MIN / 2, INT_MAX / 2);
        }
    }
    const BoxRec *box = reinterpret_cast<const BoxRec *>(blob + p.off_boxes);
    for (int b = threadIdx.x; b < p.n_boxes; b += kThreads) {
        const v3 rs = xform_point(box[b].w2l, origin);
        box_cam[b] = make_float4(rs.x, rs.y, rs.z, strictly_inside(box[b], rs) ? 1.0f : 0.0f);
    }
}

// The pixel of lane `lane` in wave tile (wx, wy): frame column x, local row
// (row of the launch's output) and frame row y (:327-329).
struct Pixel {
    int x, local_row, y;
    bool active;
};
__device__ __forceinline__ Pixel wave_pixel(const LaunchParams &p, int wx, int wy) {
    const int lane = threadIdx.x & 63;
    Pixel px;
    px.x = wx * 8 + (lane & 7);
    px.local_row = p.slice_begin + wy * 8 + (lane >> 3);
    px.active = px.x < p.width && px.local_row < p.slice_begin + p.slice_rows;
    px.y = output_row(p, px.active ? px.local_row : p.slice_begin + wy * 8);
    return px;
}

// Camera ray through pixel (x, y) offset by (jx, jy) (:377-392); jx = jy = 0
// for the reference's one ray per pixel (float(x - hw) + 0.0f is exact).
__device__ __forceinline__ Ray camera_ray(const LaunchParams &p, const FrameView &V, int x, int y, float jx,
                                          float jy) {
    const int hw = p.width / 2, hh = p.height / 2;
    const float *M = V.unproj;  // column-major
    // x - hw + jx is +0 or a multiple of 2^-24 of magnitude <= 2^16: the
    // short division by the (uniform) W/2, H/2 >= 1 is the correctly rounded
    // one (a 1-pixel-wide or -high frame divides by 0: IEEE path)
    const float nx = static_cast<float>(x - hw) + jx, ny = static_cast<float>(y - hh) + jy;
    float vx, vy;
    if (hw > 0 && hh > 0) {
        vx = div_r(nx, rcp_refined(static_cast<float>(hw)));
        vy = div_r(ny, rcp_refined(static_cast<float>(hh)));
    } else {
        vx = nx / static_cast<float>(hw);
        vy = ny / static_cast<float>(hh);
    }
    float ws[4], we[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ws[k] = M[k] * vx + M[4 + k] * vy + M[8 + k] * 0.5f + M[12 + k] * 1.0f;
        we[k] = M[k] * vx + M[4 + k] * vy + M[8 + k] * 1.0f + M[12 + k] * 1.0f;
    }
    // (the same short divisions behind a per-wave range check measured
    // slower, config 2 38.9 -> 40.3 us per frame: the check is now made once
    // per launch on the host and read as a uniform argument)
    v3 s3, e3;
    if (p.cam_short) {
        // the host proved every numerator +0 or in [2^-60, 2^60] and every w
        // in [2^-20, 2^20] for this frame (rt_scene.cpp camera_short_divisions):
        // one refined reciprocal per w and one correction per quotient, the
        // correctly rounded quotients (config 2 -3.2 %, config 5 -5.4 %, r03w)
        const Rcp rs3 = rcp_refined(ws[3]), re3 = rcp_refined(we[3]);
        s3 = mk(div_r(ws[0], rs3), div_r(ws[1], rs3), div_r(ws[2], rs3));
        e3 = mk(div_r(we[0], re3), div_r(we[1], re3), div_r(we[2], re3));
    } else {
        s3 = mk(fdiv(ws[0], ws[3]), fdiv(ws[1], ws[3]), fdiv(ws[2], ws[3]));
        e3 = mk(fdiv(we[0], we[3]), fdiv(we[1], we[3]), fdiv(we[2], we[3]));
    }
    Ray ray;
    ray.start = mk(V.origin[0], V.origin[1], V.origin[2]);
    ray.dir = normalize(sub(e3, s3));
    return ray;
}


// One 8x8 wave tile (wx, wy) of view z: lane l renders pixel (8 wx + l % 8,
// 8 wy + l / 8). `pre`: the lane's camera ray, already computed (the tiled
// path computes it while the scene is staged), or nullptr.
template <int kDepth, bool kAccum, int kShape>
__device__ __forceinline__ void render_wave_tile(const LaunchParams &p, Scene S, const FrameView &V, int wx, int wy,
                                                 int z, const Pixel &px, const Ray &pre, bool have_pre) {
    S.cull = V.cull;
    S.room = 0;
    S.cam_terms = kLeanViews(kShape) ? 0 : 1;
    if (!S.cull) S.cbplane = nullptr;  // (culling off: every box tested)
    // the scene's shape as constants (scene_shape checked it on the host):
    // every feature test on the path folds, and with a room (one box) every
    // loop over the boxes and the shadow queries' box shortcut test
    if constexpr ((kShape & kShapeMaskBytes) != 0) {
        // depth 0: the shadow queries walk LDS direction masks
        static_assert(kDepth == 0, "LDS-mask shapes: depth-0 kernels (no secondary rays, no BVH walk)");
        S.cull = 1;
        S.dmask_bytes = kShape & kShapeMaskBytes;
        S.cone = nullptr;
        S.nbvh = 0;
        S.dmask_n = kShapeMaskTexels;
        // LDS masks exist for 1..kMaskMaxSpheres spheres: one pass of the
        // primary rays' 64-lane footprint test
        __builtin_assume(S.ns > 0 && S.ns <= kMaskMaxSpheres);
    }
    if constexpr ((kShape & kShapeWide) != 0) {
        // depth >= 2: wide masks with their candidate lists, origin-sphere lists
        static_assert(kDepth >= 2, "wide shapes: the recursive kernels");
        S.cull = 1;
        S.dmask = nullptr;
        S.cone = nullptr;
        __builtin_assume(S.gmask != nullptr);
        __builtin_assume(S.glist != nullptr);
        __builtin_assume(S.olist != nullptr);
    }
    if constexpr ((kShape & kShapeRoom) != 0) {
        S.nb = 1;
        S.room = 1;
        S.dmask_box = 0;  // (a room scene's masks carry no box bits: rt_scene.cpp)
        S.cbplane = nullptr;  // (nor separating planes: one box)
    }
    RT_CYC(kCycRaygen);
    if (!wave_any(px.active)) return;
    const int x = px.x, y = px.y, local_row = px.local_row;
    const bool active = px.active;
    const int lr0 = p.slice_begin + wy * 8;
    S.tx0 = wx * 8;
    S.tx1 = S.tx0 + 7;
    if (p.n_shards <= 0 || (p.block_rows % 8 == 0 && lr0 % 8 == 0)) {
        // the wave's 8 local rows lie in one block: 8 consecutive frame rows
        S.ty0 = output_row(p, lr0);
        S.ty1 = S.ty0 + 7;
    } else {
        S.ty0 = INT_MAX;
        S.ty1 = INT_MIN;
        for (int i = 0; i < 8; ++i) {
            const int fy = output_row(p, lr0 + i);
            S.ty0 = fy < S.ty0 ? fy : S.ty0;
            S.ty1 = fy > S.ty1 ? fy : S.ty1;
        }
    }
    float4 *out = p.out + static_cast<size_t>(z) * p.n_rows * p.width;
    const uint32_t idx = static_cast<uint32_t>(local_row) * static_cast<uint32_t>(p.width) + static_cast<uint32_t>(x);

    if constexpr (!kAccum) {
        const Ray ray = have_pre ? pre : camera_ray(p, V, x, y, 0.0f, 0.0f);
#if defined(RT_ABLATE_RAYGEN)
        (void)ray;
        const v3 col = mk(float(x), float(y), 0.0f);
#elif defined(RT_ABLATE_TRACE)
        const v3 col = ray.dir;
#else
        if constexpr (kDepth > 0) {
            // each lane's pixel stored as soon as its tree is finished
            trace_tree<kDepth>(S, ray, active, [&](v3 col) { store_pixel(p, z, idx, col); });
            return;
        }
        const v3 col = trace0(S, ray, active);
#endif
        RT_CYC_AFTER(kCycStore, col.x);
        if (active) store_pixel(p, z, idx, col);
    } else {
        const uint32_t pixel = static_cast<uint32_t>(y) * static_cast<uint32_t>(p.width) + static_cast<uint32_t>(x);
        v3 acc = mk(0.0f, 0.0f, 0.0f);
        for (int smp = 0; smp < p.spp; ++smp) {
            const uint32_t sid = static_cast<uint32_t>(p.sample0 + smp);
            const float jx = p.jitter ? jitter_u(p.seed, sid, pixel, 0u) : 0.0f;
            const float jy = p.jitter ? jitter_u(p.seed, sid, pixel, 1u) : 0.0f;
            v3 col = mk(0.0f, 0.0f, 0.0f);
            if constexpr (kDepth == 0) col = trace0(S, camera_ray(p, V, x, y, jx, jy), active);
            else trace_tree<kDepth>(S, camera_ray(p, V, x, y, jx, jy), active, [&](v3 c) { col = c; });
            acc = add(acc, col);
        }
        if (active) {
            const float4 o = out[idx];
            out[idx] = make_float4(o.x + acc.x, o.y + acc.y, o.z + acc.z, o.w + 0.0f);
        }
    }
}

// Work distribution.
//  * Tiled (p.sched == nullptr: depth 0-1, views of several scenes, or too
//    few wave tiles to fill the chip; launch_kernel decides): one work-group
//    per kTileX x kTileY tile of a view (blockIdx.z), wave w rendering its
//    8x8 quadrant; the scene and the view's per-frame constants are staged
//    into LDS per work-group.
//  * Queued (depth >= 2, more wave tiles than resident waves, p.sched set,
//    one scene): a grid of as many work-groups as are resident at once;
//    each stages the scene and the per-frame constants of every view of the
//    launch once, then every wave renders 8x8 wave tiles on its own until
//    the launch is done — no barrier after the prologue, and the launch ends
//    on wave-tile granularity instead of with a tail of late work-groups.
//    Item t is wave tile t % T of view t / T (T tiles per view: the views
//    in order, and one tail per launch instead of one per frame). The
//    items are dealt to kQueues queues by index (item t in queue
//    t % kQueues, spatially interleaved, so the queues carry equal work);
//    global wave g belongs to queue g % kQueues, starts with tile g and then
//    takes the queue's next tile from its atomic head, fetched one tile
//    ahead. The last wave of a queue to run dry resets the queue's head and
//    done counters for the next launch.
// Queued distribution pays where the cost per wave tile varies most (the
// recursive depths); depth 0 / 1 keep the tiled kernel, whose body the
// compiler schedules with fewer registers (config 2: 70 vs 81 VGPRs).
// (r02: queued from depth 0, 64 VGPRs + 84 B scratch: config 2 single frame
// 52 -> 67 us, 8-frame launches, tiled either way, 41.5 -> 50.6 us per frame)
constexpr bool kQueuedDepth(int depth) { return depth >= 2; }

// kDev: a batch of more than kMaxViews views (depth 0-1): view z and its
// frame constants come from the context's device buffer (p.views_dev,
// p.consts_dev) instead of the kernel arguments; the view is read through
// the constant address space (scalar loads, as the kernel arguments are).
template <int kDepth, bool kAccum, bool kDev = false, int kShape = 0>
__global__ __launch_bounds__(kThreads) RT_OCCUPANCY void render_kernel(LaunchParams p) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    // A wave in its prologue (kernel arguments, the scene into LDS, the
    // barrier) issues ahead of the older waves of its SIMD, which the arbiter
    // otherwise favours by age; back to 0 after the barrier. Depth-0
    // batches -1.4 % (config 2, shipped), one frame per launch -2.1 %, any
    // level above 0 alike (profiles/r06ze_ab_prio.log, r06zf_ab_prio_levels.log).
    __builtin_amdgcn_s_setprio(1);
    const bool queued = kQueuedDepth(kDepth) && !kDev && p.sched != nullptr;
    const int z = queued ? 0 : static_cast<int>(blockIdx.z);
    const int n_staged = queued ? p.n_views : 1;  // views whose constants this work-group stages
    FrameView Vdev;
    if constexpr (kDev) Vdev = cload((const __attribute__((address_space(4))) FrameView *)(p.views_dev) + z);
    const FrameView &V = kDev ? Vdev : p.view[z];
    // wave index through readfirstlane: provably wave-uniform to the compiler,
    // so the tile coordinates and culling rectangles stay in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // ---- prologue: stage the scene blob into LDS and derive the view's
    // per-frame constants (both from the device blob, one barrier); the tiled
    // path computes its camera rays while the staging loads are in flight ----
    RT_PHASE(0);
#ifdef RT_PHASE_TRACE
    {  // where the wave runs: HW_ID (cu / simd / se) and XCC_ID
        const unsigned wg_ = (blockIdx.y * gridDim.x + blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        if ((threadIdx.x & 63) == 0 && wg_ < kPhaseWaves) {
            rt_phase_buf[wg_ * 16 + 8] = hw;
            rt_phase_buf[wg_ * 16 + 9] = xcc;
        }
    }
#endif
    const float4 *blob = static_cast<const float4 *>(V.blob ? V.blob : p.scene);
    const int tid = threadIdx.x;
    float4 first = make_float4(0.0f, 0.0f, 0.0f, 0.0f), fc = first;
    if (tid < p.blob_units) first = blob[tid];
    // this view's per-frame constants computed on the host (when every
    // view's fit in the kernel arguments: host_frame_setup) — else derived
    // below by every work-group
    static_assert(kMaxViewConsts <= kThreads, "one record per thread");
    // lean views (the wide shapes, kLeanViews): the host's records of a view
    // minus their first n_spheres (the camera terms) go to LDS
    constexpr bool kLean = kLeanViews(kShape);
    const int skip = kLean ? p.n_spheres : 0, keep = p.n_frame_consts - skip;
    if (tid < keep) fc = (kDev ? p.consts_dev : p.frame_consts)[z * p.n_frame_consts + skip + tid];
    float4 *const views = lds + p.blob_units;  // view k's records at views + k * view_units
    float4 *sph_cam = kLean ? nullptr : views;
    int4 *sph_px = reinterpret_cast<int4 *>(views + (kLean ? 0 : p.n_spheres));
    float4 *box_cam = reinterpret_cast<float4 *>(sph_px + p.n_spheres);
    const int own_wx = static_cast<int>(blockIdx.x) * kWavesX + wave % kWavesX;
    const int own_wy = static_cast<int>(blockIdx.y) * kWavesY + wave / kWavesX;
    const Pixel own = wave_pixel(p, own_wx, own_wy);
    RT_PHASE_AFTER(14, own.y);
    Ray own_ray{mk(0.0f, 0.0f, 0.0f), mk(0.0f, 0.0f, 0.0f)};
    if (!queued && !kAccum) own_ray = camera_ray(p, V, own.x, own.y, 0.0f, 0.0f);
    RT_PHASE_AFTER(15, own_ray.dir.x + own_ray.dir.y + own_ray.dir.z);
    RT_PHASE(10);
    if (tid < p.blob_units) lds[tid] = first;
    RT_PHASE(11);
    for (int i = tid + kThreads; i < p.blob_units; i += kThreads) lds[i] = blob[i];
    const int view_units = (kLean ? 1 : 2) * p.n_spheres + p.n_boxes;
    if (p.n_frame_consts > 0) {
        if (tid < keep) views[tid] = fc;
        if (kLean) {
            for (int i = tid + keep; i < n_staged * keep; i += kThreads) {
                const int k = i / keep;
                views[i] = p.frame_consts[k * p.n_frame_consts + skip + (i - k * keep)];
            }
        } else {
            for (int i = tid + p.n_frame_consts; i < n_staged * p.n_frame_consts; i += kThreads)
                views[i] = p.frame_consts[i];
        }
    } else {
        frame_setup(p, V, sph_cam, sph_px, box_cam);
        for (int k = 1; k < n_staged; ++k) {
            float4 *c = views + k * view_units;
            int4 *px = reinterpret_cast<int4 *>(c + (kLean ? 0 : p.n_spheres));
            frame_setup(p, p.view[k], kLean ? nullptr : c, px, reinterpret_cast<float4 *>(px + p.n_spheres));
        }
    }
    RT_PHASE(12);
#ifdef RT_STATS
    if (lane < kStats) rt_stats_lds[wave][lane] = 0u;
#endif
#ifdef RT_CYCLES
    if (lane <= kCycPhases) rt_cyc_lds[wave][lane] = lane == kCycPhases ? __builtin_amdgcn_s_memtime() : 0u;
    if (lane == 0) rt_cyc_cur[wave] = kCycPrologue;
#endif
    __syncthreads();
    __builtin_amdgcn_s_setprio(0);
    RT_PHASE(13);
    Scene S;
    S.sph = lds + p.off_spheres;
    S.smeta = reinterpret_cast<const int4 *>(lds + p.off_smeta);
    S.sph_cam = sph_cam;
    S.sph_px = sph_px;
    S.box = reinterpret_cast<const BoxRec *>(lds + p.off_boxes);
    S.box_cam = box_cam;
    S.mat = reinterpret_cast<const MatRec *>(lds + p.off_mats);
    S.light = reinterpret_cast<const LightRec *>(lds + p.off_lights);
    S.lm = reinterpret_cast<const LightMatRec *>(lds + p.off_lightmat);
    S.bvh = lds + p.off_bvh;
    S.blink = reinterpret_cast<const uint32_t *>(lds + p.off_blink);
    S.cone = p.off_cone >= 0 ? reinterpret_cast<const ShadowCone *>(lds + p.off_cone) : nullptr;
    S.dmask = p.off_dmask >= 0 ? reinterpret_cast<const char *>(lds + p.off_dmask) : nullptr;
    S.dmask_n = p.dmask_n;
    S.dmask_bytes = p.dmask_bytes;
    S.dmask_box = p.dmask_box;
    S.cbplane = p.off_bplane >= 0 ? (const __attribute__((address_space(4))) float4 *)(blob + p.off_bplane) : nullptr;
    // (recursive depths only: the depth-0/1 kernels keep their register
    // budget and use the per-wave cone for such scenes)
    S.gmask = kDepth >= 2 && p.off_gmask >= 0 ? reinterpret_cast<const uint64_t *>(blob + p.off_gmask) : nullptr;
    S.gwords = p.gmask_words;
    S.glist = S.gmask && p.off_glist >= 0 ? reinterpret_cast<const uint4 *>(blob + p.off_glist) : nullptr;
    S.olist = kDepth >= 2 && p.off_olist >= 0 ? reinterpret_cast<const uint4 *>(blob + p.off_olist) : nullptr;
    S.cbox = (const __attribute__((address_space(4))) BoxRec *)(blob + p.off_boxes);
    S.clight = (const __attribute__((address_space(4))) LightRec *)(blob + p.off_lights);
#ifdef RT_UNIFORM_MAT
    S.cmat = (const __attribute__((address_space(4))) MatRec *)(blob + p.off_mats);
    S.clm = (const __attribute__((address_space(4))) LightMatRec *)(blob + p.off_lightmat);
#endif
    S.nbvh = p.n_bvh;
    S.ns = p.n_spheres;
    S.nb = p.n_boxes;
    S.nl = p.n_lights;
    S.nm = p.n_mats;
    const int wtx = (p.width + 7) / 8;
    const int view_tiles = wtx * ((p.slice_rows + 7) / 8);
    const int total = queued ? view_tiles * p.n_views : 1;
    const int g = static_cast<int>(blockIdx.x) * (kThreads / 64) + wave;  // global wave
    const int n_waves = static_cast<int>(gridDim.x) * (kThreads / 64);
    const int q = g % kQueues;
    const int q_waves = (n_waves - q + kQueues - 1) / kQueues;  // waves of queue q
    int *head = p.sched + q * kQueueStride;
    int *done = p.sched + (kQueues + q) * kQueueStride;
    // tiled: the wave's quadrant of the block's tile; queued: item g / kQueues
    // of queue q (its first q_waves items are dealt statically), then the
    // queue's head (one render call site for both: the kernel body is inlined once)
    int t = queued ? g : 0;
    RT_PHASE(1);
    while (t < total) {
        int nxt = 0;
        if (queued && lane == 0) nxt = atomicAdd(head, 1);  // fetched one tile ahead
        // (queued: the item's view and tile; t is wave-uniform)
        const int zt = queued && p.n_views > 1 ? t / view_tiles : z, r = t - zt * view_tiles;
        const int wx = queued ? r % wtx : own_wx, wy = queued ? r / wtx : own_wy;
        Scene St = S;
        if (queued && zt != 0) {
            const float4 *c = views + zt * view_units;
            St.sph_cam = kLean ? nullptr : c;
            St.sph_px = reinterpret_cast<const int4 *>(c + (kLean ? 0 : p.n_spheres));
            St.box_cam = reinterpret_cast<const float4 *>(St.sph_px + p.n_spheres);
        }
        render_wave_tile<kDepth, kAccum, kShape>(p, St, queued ? p.view[zt] : V, wx, wy, zt,
                                              queued ? wave_pixel(p, wx, wy) : own, own_ray, !(queued || kAccum));
        t = queued ? (q_waves + __builtin_amdgcn_readfirstlane(nxt)) * kQueues + q : total;
    }
    RT_PHASE(7);
#ifdef RT_STATS
    if (lane < kStats) atomicAdd(&rt_stats[lane], static_cast<unsigned long long>(rt_stats_lds[wave][lane]));
#endif
#ifdef RT_CYCLES
    RT_CYC(kCycStore);
    if (lane < kCycPhases) atomicAdd(&rt_cycles[lane], rt_cyc_lds[wave][lane]);
#endif
    if (!queued) return;
    if (lane == 0 && atomicAdd(done, 1) == q_waves - 1) {
        atomicExch(head, 0);  // every wave of the queue has made its last fetch
        atomicExch(done, 0);
    }
}

// Resident work-groups per CU of a kernel at a dynamic LDS size (cached: the
// occupancy query is host work).
int groups_per_cu(const void *fn, size_t lds) {
    struct Entry {
        const void *fn;
        size_t lds;
        int n;
    };
    thread_local Entry cache[8] = {};
    thread_local int next = 0;
    for (const Entry &e : cache)
        if (e.fn == fn && e.lds == lds && e.n > 0) return e.n;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, lds) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 1;
    }
    cache[next] = {fn, lds, n};
    next = (next + 1) % 8;
    return n;
}

// LDS of a queued launch of n views: the scene and every view's per-frame
// constants.
size_t queued_lds_bytes(const LaunchParams &p, int n) {
    return lds_bytes(p) + static_cast<size_t>(n - 1) * view_units(p) * sizeof(float4);
}

// Views of one scene a queued launch holds at the one-view launch's resident
// work-groups per CU (their constants beside the scene in LDS), at most
// kMaxViews (cached per kernel and scene shape: occupancy queries are host
// work).
int queued_views_for(const void *fn, const LaunchParams &p) {
    struct Entry {
        const void *fn;
        size_t lds;
        int units, n;
    };
    thread_local Entry cache[8] = {};
    thread_local int next = 0;
    const size_t lds = lds_bytes(p);
    const int units = view_units(p);
    for (const Entry &e : cache)
        if (e.fn == fn && e.lds == lds && e.units == units && e.n > 0) return e.n;
    const int g1 = groups_per_cu(fn, lds);
    int n = 1;
    while (n < kMaxViews && queued_lds_bytes(p, n + 1) <= kMaxLds &&
           groups_per_cu(fn, queued_lds_bytes(p, n + 1)) >= g1)
        ++n;
    cache[next] = {fn, lds, units, n};
    next = (next + 1) % 8;
    return n;
}

template <int kDepth, bool kAccum, bool kDev = false, int kShape = 0>
hipError_t launch_kernel(LaunchParams &p, hipStream_t stream) {
    p.lean_views = kLeanViews(kShape) ? 1 : 0;
    size_t lds = lds_bytes(p);
    const void *fn = reinterpret_cast<const void *>(&render_kernel<kDepth, kAccum, kDev, kShape>);
    dim3 grid((p.width + kTileX - 1) / kTileX, (p.slice_rows + kTileY - 1) / kTileY, p.n_views);
    const int wave_tiles = ((p.width + 7) / 8) * ((p.slice_rows + 7) / 8) * p.n_views;
    const int resident = p.n_cu > 0 ? groups_per_cu(fn, lds) * p.n_cu : 0;
    // queued: more wave tiles than resident waves, every queue has a wave (a
    // queue without one would leave its tiles unrendered), and for several
    // views: one scene (staged once) and every view's constants in LDS at the
    // same resident work-groups (queued_views)
    bool one_scene = p.n_views <= kMaxViews;
    for (int k = 0; k < p.n_views && one_scene; ++k) one_scene = p.view[k].blob == nullptr;
    if (kQueuedDepth(kDepth) && p.sched && wave_tiles > resident * (kThreads / 64) &&
        resident * (kThreads / 64) >= kQueues &&
        (p.n_views == 1 || (one_scene && queued_views_for(fn, p) >= p.n_views))) {
        grid = dim3(resident, 1, 1);
        lds = queued_lds_bytes(p, p.n_views);
    } else {
        p.sched = nullptr;
    }
    hipLaunchKernelGGL((render_kernel<kDepth, kAccum, kDev, kShape>), grid, dim3(kThreads), lds, stream, p);
    return hipGetLastError();
}

// The depth-0 kernels in the scene's shape (scene_shape): 2-, 4- or 8-byte
// LDS masks, one box or several; anything else runs the general kernel.
template <bool kAccum, bool kDev>
hipError_t launch_depth0(LaunchParams &p, hipStream_t stream) {
    switch (scene_shape(p, 0)) {
        case 2: return launch_kernel<0, kAccum, kDev, 2>(p, stream);
        case 4: return launch_kernel<0, kAccum, kDev, 4>(p, stream);
        case 8: return launch_kernel<0, kAccum, kDev, 8>(p, stream);
        case 2 | kShapeRoom: return launch_kernel<0, kAccum, kDev, 2 | kShapeRoom>(p, stream);
        case 4 | kShapeRoom: return launch_kernel<0, kAccum, kDev, 4 | kShapeRoom>(p, stream);
        case 8 | kShapeRoom: return launch_kernel<0, kAccum, kDev, 8 | kShapeRoom>(p, stream);
        default: return launch_kernel<0, kAccum, kDev, 0>(p, stream);
    }
}

// The recursive kernels in the wide-mask shape (scene_shape), else general.
template <int kDepth>
hipError_t launch_deep(LaunchParams &p, hipStream_t stream) {
    switch (scene_shape(p, kDepth)) {
        case kShapeWide: return launch_kernel<kDepth, false, false, kShapeWide>(p, stream);
        case kShapeWide | kShapeRoom: return launch_kernel<kDepth, false, false, kShapeWide | kShapeRoom>(p, stream);
        default: return launch_kernel<kDepth, false, false, 0>(p, stream);
    }
}

template <int kDepth>
hipError_t launch_depth(LaunchParams &p, hipStream_t stream) {
    if (p.views_dev) {  // a device-side view batch (render_batch_impl: depth 0-1, no accumulation)
        if constexpr (kDepth == 0) {
            if (p.spp == 0) return launch_depth0<false, true>(p, stream);
        } else if constexpr (kDepth == 1) {
            if (p.spp == 0) return launch_kernel<kDepth, false, true>(p, stream);
        }
        return hipErrorInvalidValue;
    }
    if constexpr (kDepth == 0) return p.spp > 0 ? launch_depth0<true, false>(p, stream) : launch_depth0<false, false>(p, stream);
    if constexpr (kDepth >= 2) {
        if (p.spp == 0) return launch_deep<kDepth>(p, stream);
    }
    return p.spp > 0 ? launch_kernel<kDepth, true>(p, stream) : launch_kernel<kDepth, false>(p, stream);
}

}  // namespace

int scene_shape(const LaunchParams &p, int max_depth) {
    if (!p.shape_cull) return 0;  // culling off for a view (or RT_OPT_SCENE_SHAPES 0)
    const int box = p.n_boxes == 1 && p.scene_room ? kShapeRoom : 0;
    if (max_depth == 0) {  // every shadow query walks the LDS masks
        if (p.off_dmask < 0 || (p.dmask_bytes != 2 && p.dmask_bytes != 4 && p.dmask_bytes != 8) ||
            p.dmask_n != kShapeMaskTexels)
            return 0;
        return p.dmask_bytes | box;
    }
    if (max_depth >= 2) {  // the wide masks' lists and the origin-sphere lists take the rays
        if (p.off_gmask < 0 || p.off_glist < 0 || p.off_olist < 0) return 0;
        return kShapeWide | box;
    }
    return 0;
}

size_t lds_bytes(const LaunchParams &p) {
    // blob + one view's records: per-sphere camera terms (16 B; not with
    // lean views) and footprint (16 B) + per-box camera terms
    return (static_cast<size_t>(p.blob_units) + view_units(p)) * sizeof(float4);
}

int queued_views(const LaunchParams &p, int max_depth) {
    const void *fn = nullptr;
    switch (max_depth) {  // (the view-batch kernels: no accumulation)
        case 2: fn = reinterpret_cast<const void *>(&render_kernel<2, false>); break;
        case 3: fn = reinterpret_cast<const void *>(&render_kernel<3, false>); break;
        case 4: fn = reinterpret_cast<const void *>(&render_kernel<4, false>); break;
        case 5: fn = reinterpret_cast<const void *>(&render_kernel<5, false>); break;
        case 6: fn = reinterpret_cast<const void *>(&render_kernel<6, false>); break;
        case 7: fn = reinterpret_cast<const void *>(&render_kernel<7, false>); break;
        case 8: fn = reinterpret_cast<const void *>(&render_kernel<8, false>); break;
        case 9: fn = reinterpret_cast<const void *>(&render_kernel<9, false>); break;
        default: return 1;
    }
    static_assert(!kQueuedDepth(1) && kQueuedDepth(2), "queued from depth 2");
    return queued_views_for(fn, p);
}

hipError_t launch_render(LaunchParams &p, int max_depth, hipStream_t stream) {
    if (p.slice_rows <= 0) {  // the whole launch as one slice
        p.slice_begin = 0;
        p.slice_rows = p.n_rows;
    }
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

// Kernel-argument self-test (rt_create): the launch parameter block is larger
// than HIP's documented 4 KiB argument limit; a runtime that truncated it
// would silently corrupt renders. One lane copies the block's last words.
__global__ void kernarg_probe(LaunchParams p, float4 *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = p.frame_consts[kMaxFrameConsts - 1];
        out[1] = make_float4(__int_as_float(p.n_frame_consts), __int_as_float(p.out_format), 0.0f, 0.0f);
    }
}

int check_kernarg_block(hipStream_t stream) {
    LaunchParams p{};
    p.frame_consts[kMaxFrameConsts - 1] = make_float4(1.5f, -2.25f, 3.125f, 4096.0f);
    p.n_frame_consts = 0x5a5a;
    p.out_format = 0x3c3c;
    float4 *d = nullptr, h[2] = {};
    hipError_t e = hipMalloc(&d, sizeof h);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(kernarg_probe, dim3(1), dim3(64), 0, stream, p, d);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        (void)hipFree(d);
    }
    if (e != hipSuccess) {
        set_error(std::string("rt_create: kernel argument probe: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    if (h[0].x != 1.5f || h[0].y != -2.25f || h[0].z != 3.125f || h[0].w != 4096.0f ||
        __builtin_bit_cast(uint32_t, h[1].x) != 0x5a5au || __builtin_bit_cast(uint32_t, h[1].y) != 0x3c3cu) {
        set_error("rt_create: this HIP runtime does not pass a " + std::to_string(sizeof(LaunchParams)) +
                  "-byte kernel argument block intact");
        return RT_ERR_UNSUPPORTED;
    }
    return RT_OK;
}

// Allow dynamic LDS above the 64 KiB default for every depth instantiation
// (gfx950 has 160 KiB per CU). Best effort: a failure only lowers the largest
// scene that fits, which rt_scene_create checks.
hipError_t allow_large_lds(size_t bytes) {
#define RT_KFN(d) reinterpret_cast<const void *>(&render_kernel<d, false>), \
                  reinterpret_cast<const void *>(&render_kernel<d, true>)
#define RT_SHAPES(k) reinterpret_cast<const void *>(&render_kernel<0, false, false, k>), \
                     reinterpret_cast<const void *>(&render_kernel<0, true, false, k>),  \
                     reinterpret_cast<const void *>(&render_kernel<0, false, true, k>)
#define RT_WIDE(d) reinterpret_cast<const void *>(&render_kernel<d, false, false, kShapeWide>), \
                   reinterpret_cast<const void *>(&render_kernel<d, false, false, kShapeWide | kShapeRoom>)
    const void *fns[] = {RT_KFN(0), RT_KFN(1), RT_KFN(2), RT_KFN(3), RT_KFN(4),
                         RT_KFN(5), RT_KFN(6), RT_KFN(7), RT_KFN(8), RT_KFN(9),
                         reinterpret_cast<const void *>(&render_kernel<0, false, true>),
                         reinterpret_cast<const void *>(&render_kernel<1, false, true>),
                         RT_SHAPES(2), RT_SHAPES(4), RT_SHAPES(8),
                         RT_SHAPES(2 | kShapeRoom), RT_SHAPES(4 | kShapeRoom), RT_SHAPES(8 | kShapeRoom),
                         RT_WIDE(2), RT_WIDE(3), RT_WIDE(4), RT_WIDE(5), RT_WIDE(6), RT_WIDE(7), RT_WIDE(8), RT_WIDE(9)};
#undef RT_KFN
#undef RT_SHAPES
#undef RT_WIDE
    for (const void *f : fns)
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
    (void)hipGetLastError();  // do not leak a sticky error into the next launch check
    return hipSuccess;
}

}  // namespace rtamd

#ifdef RT_STATS
extern "C" int rt_debug_stats(unsigned long long *dst, int clear) {
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(rtamd::rt_stats), sizeof(rtamd::rt_stats), 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
        return -1;
    if (clear) {
        void *ptr = nullptr;
        if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(rtamd::rt_stats)) != hipSuccess) return -1;
        return hipMemset(ptr, 0, sizeof(rtamd::rt_stats)) == hipSuccess ? 0 : -1;
    }
    return 0;
}
#endif
#ifdef RT_CYCLES
extern "C" int rt_debug_cycles(unsigned long long *dst, int clear) {
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(rtamd::rt_cycles), sizeof(rtamd::rt_cycles), 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
        return -1;
    if (clear) {
        void *ptr = nullptr;
        if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(rtamd::rt_cycles)) != hipSuccess) return -1;
        return hipMemset(ptr, 0, sizeof(rtamd::rt_cycles)) == hipSuccess ? 0 : -1;
    }
    return 0;
}
#endif
#ifdef RT_PHASE_TRACE
extern "C" int rt_debug_phase_read(void *dst, size_t bytes) {
    const size_t n = bytes < sizeof(rtamd::rt_phase_buf) ? bytes : sizeof(rtamd::rt_phase_buf);
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(rtamd::rt_phase_buf), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int rt_debug_occupancy(size_t lds) {
    int n = -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&rtamd::render_kernel<0, false>),
                                                     rtamd::kThreads, lds) != hipSuccess)
        return -1;
    return n;
}
extern "C" int rt_debug_phase_clear(void) {
    void *ptr = nullptr;
    if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(rtamd::rt_phase_buf)) != hipSuccess) return -1;
    return hipMemset(ptr, 0, sizeof(rtamd::rt_phase_buf)) == hipSuccess ? 0 : -1;
}
#endif
