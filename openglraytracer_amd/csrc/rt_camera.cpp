// rt_camera.cpp — the reference's orbiting camera (raytrace_compute.glsl:
// 334-392, :411-545) evaluated the way the reference's own GL evaluates it.
//
// The reference computes its camera in float32 per invocation; its golden
// renders (tests/golden) come from Mesa llvmpipe. Reproducing that frame
// constant bit for bit needs three things measured on llvmpipe (probe
// shaders built from the reference's own camera functions,
// tests/golden/make_camera_golden.py):
//  * run-time sin / cos are gallivm's polynomials (Cephes range reduction by
//    4/pi, three-part pi/4 subtraction, the two minimax polynomials, every
//    multiply-add fused) — gl_sin / gl_cos below;
//  * everything that depends only on constants is folded at compile time in
//    float (tan(45 deg) -> 1, cos(DEG_TO_RAD * 90), the projection terms, the
//    identity pitch / roll rotations);
//  * the compiler's inexact-float rewrites: products and sums with a
//    constant 0 or 1 vanish, a product by a constant times another constant
//    becomes one product by the folded constant ((10 cos s) * c -> cos s *
//    (10 c)), and mod()'s `(x - 360 floor(x/360)) + 90` becomes
//    `(x + 90) - 360 floor(x/360)`; no multiply-add is fused.
// Gf below carries that bookkeeping: a value, whether it is a compile-time
// constant, and whether it is a run-time value times a constant. With it the
// float32 chain — GLSL matrix products (column sums left to right), Mesa's
// inverse(mat4) (2x2 sub-factors, adjugate, determinant, true division) —
// matches llvmpipe's inverse(proj * view) and view matrix exactly
// (tests/test_host.py: 1200 probed times and every golden fixture).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "rt_internal.h"

namespace rtamd {

namespace {

constexpr float kPi = 3.14159265358f;       // raytrace_compute.glsl:13
constexpr float kDegToRad = kPi / 180.0f;    // :17, folded in float

float bits_to_float(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
uint32_t float_to_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// gallivm's lp_build_sin / lp_build_cos (Mesa llvmpipe, the GL the
// reference's golden renders come from), in float32 with fused multiply-adds.
float gallivm_sincos(float a, bool want_cos) {
    const float x_abs = std::fabs(a);
    const float scale_y = x_abs * 1.27323954473516f;  // 4 / pi
    const int emm2_i = static_cast<int>(scale_y);     // truncation
    const int emm2_add = emm2_i + 1;
    const int emm2_and = emm2_add & ~1;  // j = (j + 1) & ~1
    const float y_2 = static_cast<float>(emm2_and);
    uint32_t sign_bit;
    bool poly_mask;
    if (want_cos) {
        const int emm2_2 = emm2_and - 2;
        sign_bit = static_cast<uint32_t>((~emm2_2) & 4) << 29;
        poly_mask = (emm2_2 & 2) == 0;
    } else {
        sign_bit = (static_cast<uint32_t>(emm2_add & 4) << 29) ^ (float_to_bits(a) & 0x80000000u);
        poly_mask = (emm2_and & 2) == 0;
    }
    // extended-precision modular arithmetic: x - j * pi/4 in three parts
    float x = std::fmaf(y_2, -0.78515625f, x_abs);
    x = std::fmaf(y_2, -2.4187564849853515625e-4f, x);
    x = std::fmaf(y_2, -3.77489497744594108e-8f, x);
    const float z = x * x;
    // cosine polynomial
    float yc = std::fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    yc = std::fmaf(yc, z, 4.166664568298827e-2f);
    yc = yc * z;
    yc = yc * z;
    yc = std::fmaf(z, -0.5f, yc);
    yc = yc + 1.0f;
    // sine polynomial
    float ys = std::fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ys = std::fmaf(ys, z, -1.6666654611e-1f);
    ys = ys * z;
    ys = std::fmaf(ys, x, x);
    const float r = poly_mask ? ys : yc;
    return bits_to_float(float_to_bits(r) ^ sign_bit);
}

// A float32 value of the camera chain with the compiler's constant
// bookkeeping (see the file comment): `konst` — known at compile time;
// `scaled` — a run-time value `base` times the constant `k` (v = base * k).
struct Gf {
    float v;
    bool konst = false;
    bool scaled = false;
    float base = 0.0f, k = 0.0f;
};
Gf cst(float v) {
    Gf r;
    r.v = v;
    r.konst = true;
    return r;
}
Gf run(float v) {
    Gf r;
    r.v = v;
    return r;
}
Gf neg(const Gf &a) {
    Gf r = a;
    r.v = -a.v;
    r.k = -a.k;  // -(b k) == b (-k) exactly
    return r;
}
Gf mul(const Gf &a, const Gf &b) {
    if (a.konst && b.konst) return cst(a.v * b.v);
    const Gf *c = a.konst ? &a : (b.konst ? &b : nullptr);
    if (!c) return run(a.v * b.v);
    const Gf &x = a.konst ? b : a;
    if (c->v == 0.0f) return cst(0.0f);    // x * 0 -> 0
    if (c->v == 1.0f) return x;            // x * 1 -> x
    if (c->v == -1.0f) return neg(x);      // x * -1 -> -x
    Gf r;
    r.scaled = true;
    if (x.scaled) {  // (base * k) * c -> base * (k c)
        r.base = x.base;
        r.k = x.k * c->v;
    } else {
        r.base = x.v;
        r.k = c->v;
    }
    r.v = r.base * r.k;
    return r;
}
Gf add(const Gf &a, const Gf &b) {
    if (a.konst && b.konst) return cst(a.v + b.v);
    if (a.konst && a.v == 0.0f) return b;  // 0 + x -> x
    if (b.konst && b.v == 0.0f) return a;
    return run(a.v + b.v);
}
Gf sub(const Gf &a, const Gf &b) { return add(a, neg(b)); }
Gf div(const Gf &a, const Gf &b) {
    if (a.konst && b.konst) return cst(a.v / b.v);
    if (a.konst && a.v == 0.0f) return cst(0.0f);
    return run(a.v / b.v);
}

struct Gm {
    Gf m[4][4];  // column-major, m[col][row]
};
Gm ident() {
    Gm r;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) r.m[c][w] = cst(c == w ? 1.0f : 0.0f);
    return r;
}
// mat4 * mat4 as GLSL lowers it: column c = A[0] b.x + A[1] b.y + A[2] b.z + A[3] b.w
Gm mul(const Gm &a, const Gm &b) {
    Gm r;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) {
            Gf acc = mul(a.m[0][w], b.m[c][0]);
            for (int k = 1; k < 4; ++k) acc = add(acc, mul(a.m[k][w], b.m[c][k]));
            r.m[c][w] = acc;
        }
    return r;
}
// rotation_matrix_{x,y,z} (:444-486) from their cosine and sine
Gm rot(int axis, const Gf &c, const Gf &s) {
    Gm r = ident();
    if (axis == 0) { r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = neg(s); r.m[2][2] = c; }
    if (axis == 1) { r.m[0][0] = c; r.m[0][2] = neg(s); r.m[2][0] = s; r.m[2][2] = c; }
    if (axis == 2) { r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = neg(s); r.m[1][1] = c; }
    return r;
}
// GLSL inverse(mat4) as Mesa's builtin lowers it: 2x2 sub-factors, the
// adjugate, det = m0.x a0 + (m0.y a1 + (m0.z a2 + m0.w a3)), adj / det.
Gm inverse(const Gm &M) {
    const Gf(*m)[4] = M.m;
    auto d = [](const Gf &a, const Gf &b, const Gf &c, const Gf &e) { return sub(mul(a, b), mul(c, e)); };
    auto t3 = [](const Gf &a, const Gf &x, const Gf &b, const Gf &y, const Gf &c, const Gf &z) {
        return add(sub(mul(a, x), mul(b, y)), mul(c, z));
    };
    const Gf S00 = d(m[2][2], m[3][3], m[3][2], m[2][3]), S01 = d(m[2][1], m[3][3], m[3][1], m[2][3]);
    const Gf S02 = d(m[2][1], m[3][2], m[3][1], m[2][2]), S03 = d(m[2][0], m[3][3], m[3][0], m[2][3]);
    const Gf S04 = d(m[2][0], m[3][2], m[3][0], m[2][2]), S05 = d(m[2][0], m[3][1], m[3][0], m[2][1]);
    const Gf S06 = d(m[1][2], m[3][3], m[3][2], m[1][3]), S07 = d(m[1][1], m[3][3], m[3][1], m[1][3]);
    const Gf S08 = d(m[1][1], m[3][2], m[3][1], m[1][2]), S09 = d(m[1][0], m[3][3], m[3][0], m[1][3]);
    const Gf S10 = d(m[1][0], m[3][2], m[3][0], m[1][2]), S11 = d(m[1][1], m[3][3], m[3][1], m[1][3]);
    const Gf S12 = d(m[1][0], m[3][1], m[3][0], m[1][1]), S13 = d(m[1][2], m[2][3], m[2][2], m[1][3]);
    const Gf S14 = d(m[1][1], m[2][3], m[2][1], m[1][3]), S15 = d(m[1][1], m[2][2], m[2][1], m[1][2]);
    const Gf S16 = d(m[1][0], m[2][3], m[2][0], m[1][3]), S17 = d(m[1][0], m[2][2], m[2][0], m[1][2]);
    const Gf S18 = d(m[1][0], m[2][1], m[2][0], m[1][1]);
    Gm adj;
    adj.m[0][0] = t3(m[1][1], S00, m[1][2], S01, m[1][3], S02);
    adj.m[1][0] = neg(t3(m[1][0], S00, m[1][2], S03, m[1][3], S04));
    adj.m[2][0] = t3(m[1][0], S01, m[1][1], S03, m[1][3], S05);
    adj.m[3][0] = neg(t3(m[1][0], S02, m[1][1], S04, m[1][2], S05));
    adj.m[0][1] = neg(t3(m[0][1], S00, m[0][2], S01, m[0][3], S02));
    adj.m[1][1] = t3(m[0][0], S00, m[0][2], S03, m[0][3], S04);
    adj.m[2][1] = neg(t3(m[0][0], S01, m[0][1], S03, m[0][3], S05));
    adj.m[3][1] = t3(m[0][0], S02, m[0][1], S04, m[0][2], S05);
    adj.m[0][2] = t3(m[0][1], S06, m[0][2], S07, m[0][3], S08);
    adj.m[1][2] = neg(t3(m[0][0], S06, m[0][2], S09, m[0][3], S10));
    adj.m[2][2] = t3(m[0][0], S11, m[0][1], S09, m[0][3], S12);
    adj.m[3][2] = neg(t3(m[0][0], S08, m[0][1], S10, m[0][2], S12));
    adj.m[0][3] = neg(t3(m[0][1], S13, m[0][2], S14, m[0][3], S15));
    adj.m[1][3] = t3(m[0][0], S13, m[0][2], S16, m[0][3], S17);
    adj.m[2][3] = neg(t3(m[0][0], S14, m[0][1], S16, m[0][3], S18));
    adj.m[3][3] = t3(m[0][0], S15, m[0][1], S17, m[0][2], S18);
    const Gf det = add(mul(m[0][0], adj.m[0][0]),
                       add(mul(m[0][1], adj.m[1][0]), add(mul(m[0][2], adj.m[2][0]), mul(m[0][3], adj.m[3][0]))));
    Gm r;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) r.m[c][w] = div(adj.m[c][w], det);
    return r;
}

// transpose(inverse(mat3(m))) as Mesa's builtin lowers inverse(mat3): the
// three cofactors of the first column, det = (m00 c0 - m01 c1) + m02 c2, the
// adjugate over det; returned column-major (r[col][row]).
void normal_matrix(const Gm &M, Gf r[3][3]) {
    const Gf(*m)[4] = M.m;
    auto d = [](const Gf &a, const Gf &b, const Gf &c, const Gf &e) { return sub(mul(a, b), mul(c, e)); };
    const Gf f0 = d(m[1][1], m[2][2], m[2][1], m[1][2]);
    const Gf f1 = d(m[1][0], m[2][2], m[2][0], m[1][2]);
    const Gf f2 = d(m[1][0], m[2][1], m[2][0], m[1][1]);
    const Gf det = add(sub(mul(m[0][0], f0), mul(m[0][1], f1)), mul(m[0][2], f2));
    Gf inv[3][3];  // inv[col][row]
    inv[0][0] = div(f0, det);
    inv[1][0] = div(neg(f1), det);
    inv[2][0] = div(f2, det);
    inv[0][1] = div(neg(d(m[0][1], m[2][2], m[2][1], m[0][2])), det);
    inv[1][1] = div(d(m[0][0], m[2][2], m[2][0], m[0][2]), det);
    inv[2][1] = div(neg(d(m[0][0], m[2][1], m[2][0], m[0][1])), det);
    inv[0][2] = div(d(m[0][1], m[1][2], m[1][1], m[0][2]), det);
    inv[1][2] = div(neg(d(m[0][0], m[1][2], m[1][0], m[0][2])), det);
    inv[2][2] = div(d(m[0][0], m[1][1], m[1][0], m[0][1]), det);
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) r[c][w] = inv[w][c];  // transpose
}

// rotation_matrix_{x,y,z} (:444-486) of a run-time angle in degrees
Gm rot_deg(int axis, float deg) {
    const float a = mul(cst(kDegToRad), run(deg)).v;
    return rot(axis, run(gl_cos(a)), run(gl_sin(a)));
}

}  // namespace

float gl_sin(float a) { return gallivm_sincos(a, false); }
float gl_cos(float a) { return gallivm_sincos(a, true); }

// main() :334-364: speed, the orbit position and the yaw angle.
void reference_orbit(float time, float *speed_out, float pos[3], float *yaw_out) {
    const float speed = time * 0.4f + 0.5f;  // :343 (time_scale 0.4, :236)
    pos[0] = 10.0f * gl_cos(speed);
    pos[1] = 10.0f * gl_sin(speed);
    pos[2] = 0.0f;
    // :353 yaw = mod(speed * (180 / 3.1416), 360) + 90, as compiled:
    // (x + 90) - 360 floor(x / 360)
    const float x = speed * (180.0f / 3.1416f);
    const float yaw = (x + 90.0f) - 360.0f * std::floor(x / 360.0f);
    if (speed_out) *speed_out = speed;
    if (yaw_out) *yaw_out = yaw;
}

// inverse(proj_mat * view_mat) (:383) and view_mat (:368) of the reference
// orbit camera at `time`, column-major, as llvmpipe computes them.
void reference_view_gl(float time, float unproj[16], float view[16]) {
    float speed, pos[3], yaw;
    reference_orbit(time, &speed, pos, &yaw);
    const float a = kDegToRad * yaw;
    const Gm Rz = rot(2, run(gl_cos(a)), run(gl_sin(a)));
    // pitch = roll = 0 are constants: cos 0 = 1, sin 0 = 0 folded
    const Gm R = mul(mul(mul(ident(), Rz), rot(0, cst(1.0f), cst(0.0f))), rot(1, cst(1.0f), cst(0.0f)));
    Gm T = ident();
    T.m[3][0] = mul(cst(10.0f), run(gl_cos(speed)));
    T.m[3][1] = mul(cst(10.0f), run(gl_sin(speed)));
    T.m[3][2] = cst(0.0f);
    // flip_y_and_z = rotation_matrix_x(90) (:542), folded at compile time:
    // cos(DEG_TO_RAD * 90) = -4.371139e-8 (0xb33bbd2e), sin = 1
    const Gm flip = rot(0, cst(bits_to_float(0xb33bbd2eu)), cst(1.0f));
    const Gm V = inverse(mul(mul(T, R), flip));
    // calc_projection_matrix (:411-426) folded: q = 1 / tan(45 deg) = 1
    Gm P;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) P.m[c][w] = cst(0.0f);
    P.m[0][0] = cst(1.0f / (16.0f / 9.0f));
    P.m[1][1] = cst(1.0f);
    P.m[2][2] = cst((0.1f + 1000.0f) / (0.1f - 1000.0f));
    P.m[2][3] = cst(-1.0f);
    P.m[3][2] = cst((2.0f * 0.1f * 1000.0f) / (0.1f - 1000.0f));
    const Gm U = inverse(mul(P, V));
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) {
            if (unproj) unproj[c * 4 + w] = U.m[c][w].v;
            if (view) view[c * 4 + w] = V.m[c][w].v;
        }
}

// intersect_box_object's transforms (:650-652, :718) as llvmpipe evaluates
// them: local_to_world = calc_transform_matrix(position, angles) (:529-532:
// translation_matrix * (mat4(1) * Rz(yaw) * Rx(pitch) * Ry(roll))), its
// Mesa inverse, and transpose(inverse(mat3(local_to_world))). The object's
// fields are run-time values (objects[] is indexed by the loop counter), so
// only the functions' own constants fold. Column-major outputs (m[col][row]
// at col * 4 + row; the normal matrix at col * 3 + row). Probed bit-exact
// against llvmpipe on the shipped scene (tests/golden/make_box_golden.py).
void reference_box_transforms(const float pos[3], const float ang[3], float l2w[16], float w2l[16],
                              float nrm[9]) {
    Gm T = ident();
    for (int k = 0; k < 3; ++k) T.m[3][k] = run(pos[k]);
    const Gm R = mul(mul(mul(ident(), rot_deg(2, ang[1])), rot_deg(0, ang[0])), rot_deg(1, ang[2]));
    const Gm L = mul(T, R);
    const Gm W = inverse(L);
    Gf N[3][3];
    normal_matrix(L, N);
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) {
            l2w[c * 4 + w] = L.m[c][w].v;
            w2l[c * 4 + w] = W.m[c][w].v;
        }
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) nrm[c * 3 + w] = N[c][w].v;
}

}  // namespace rtamd
