/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 * A scalar float32 restatement of /root/reference/OpenGLRaytracer/
 * raytrace_compute.glsl. Every function cites the GLSL lines it follows and
 * keeps the GLSL operation order. Matrices are GLSL column-major: m[col][row].
 * Built with -ffp-contract=off (no FMA contraction) and without fast-math.
 *
 * Floating-point notes (pinned against llvmpipe fixtures):
 *  - normalize(v) = v * inversesqrt(dot(v, v)) (GLSL builtin lowering).
 *  - mix(x, y, a) = x + a * (y - x); dot(vec3) = x + (y + z);
 *  - inverse(mat4) = GLM/Mesa cofactor scheme with a true division.
 *  - pow(x, y) = llvmpipe's exp2(log2(x) * y) polynomials (glsl_pow).
 *  - reflect/refract follow the GLSL spec formulas.
 */
#include "rt_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { float m[4][4]; } m4; /* m[col][row] */
typedef struct { float m[3][3]; } m3;

/* raytrace_compute.glsl:13-18 (float constants, folded in float) */
static const float PI_F = 3.14159265358f;
#define DEG_TO_RAD (PI_F / 180.0f)

static v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 mul3s(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* dot(vec3): x + (y + z) — the association llvmpipe evaluates (probed). */
static float dot3(v3 a, v3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static v3 normalize3(v3 a) { return mul3s(a, 1.0f / sqrtf(dot3(a, a))); }
static v4 add4(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static v4 mul4(v4 a, v4 b) { return V4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static v4 mul4s(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
static v4 ld4(const float *p) { return V4(p[0], p[1], p[2], p[3]); }
static v3 ld3(const float *p) { return V3(p[0], p[1], p[2]); }
static float maxf(float a, float b) { return a > b ? a : b; } /* GLSL max on ordered values */
static float minf(float a, float b) { return a < b ? a : b; }
static float comp3(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
/* GLSL mix(x, y, a), evaluated as x + a * (y - x) (the lerp form llvmpipe uses, probed). */
static v3 mix3(v3 x, v3 y, float a) { return add3(x, mul3s(sub3(y, x), a)); }
/* GLSL reflect(I, N) = I - 2 * dot(N, I) * N */
static v3 reflect3(v3 i, v3 n) { return sub3(i, mul3s(n, 2.0f * dot3(n, i))); }
/* GLSL refract(I, N, eta); k = 1 - eta * (eta * (1 - d*d)) is the
 * association Mesa's builtin uses (probed against llvmpipe). */
static v3 refract3(v3 i, v3 n, float eta) {
    float d = dot3(n, i);
    float k = 1.0f - eta * (eta * (1.0f - d * d));
    if (k < 0.0f) return V3(0.0f, 0.0f, 0.0f);
    return sub3(mul3s(i, eta), mul3s(n, eta * d + sqrtf(k)));
}

/* GLSL pow(x, y) as llvmpipe evaluates it for a run-time exponent:
 * exp2(log2(x) * y) with gallivm's polynomial log2/exp2 (even/odd-split
 * polynomials, every multiply-add fused). Probed bit-exact against llvmpipe
 * for x in (0, 1], y in {3, 4, 10} (DESIGN.md "Parity"). */
static float poly_eo(float x, const float *c, int n) {
    float x2 = x * x, even = 0.0f, odd = 0.0f;
    int have_even = 0, have_odd = 0;
    for (int i = n - 1; i >= 0; i--) {
        if (i % 2 == 0) { even = have_even ? fmaf(x2, even, c[i]) : c[i]; have_even = 1; }
        else { odd = have_odd ? fmaf(x2, odd, c[i]) : c[i]; have_odd = 1; }
    }
    return fmaf(odd, x, even);
}
static float glsl_log2(float x) {
    static const float C[5] = {2.88539009343309178325f, 0.961791550404184197881f, 0.577440339438736392009f,
                               0.403343858251329912514f, 0.406718052498846252698f};
    if (x == 0.0f) return -INFINITY;
    if (x < 0.0f || x != x) return NAN;
    if (isinf(x)) return INFINITY;
    uint32_t i;
    memcpy(&i, &x, 4);
    float e = (float)((int)((i >> 23) & 0xffu) - 127);
    uint32_t mi = (i & 0x007fffffu) | 0x3f800000u;
    float mant;
    memcpy(&mant, &mi, 4);
    float y = (mant - 1.0f) / (mant + 1.0f);
    float z = y * y;
    return fmaf(y, poly_eo(z, C, 5), e);
}
static float glsl_exp2(float x) {
    static const float C[6] = {1.0f, 0.693153073200168932794f, 0.240153617044375388211f,
                               0.0558263180532956664775f, 0.00898934009049466391101f,
                               0.00187757667519147912699f};
    x = x < 129.0f ? x : 129.0f;
    x = x > -126.99999f ? x : -126.99999f;
    float ip = floorf(x);
    float fp = x - ip;
    uint32_t ei = (uint32_t)((int)ip + 127) << 23;
    float ex;
    memcpy(&ex, &ei, 4);
    return ex * poly_eo(fp, C, 6);
}
static float glsl_pow(float x, float y) { return glsl_exp2(glsl_log2(x) * y); }

static m4 ident4(void) {
    m4 r;
    memset(&r, 0, sizeof r);
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f;
    return r;
}
static m4 mul44(m4 a, m4 b) {
    m4 r;
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++)
            r.m[c][row] = a.m[0][row] * b.m[c][0] + a.m[1][row] * b.m[c][1] + a.m[2][row] * b.m[c][2] +
                          a.m[3][row] * b.m[c][3];
    return r;
}
static v4 mul4v(m4 a, v4 v) {
    return V4(a.m[0][0] * v.x + a.m[1][0] * v.y + a.m[2][0] * v.z + a.m[3][0] * v.w,
              a.m[0][1] * v.x + a.m[1][1] * v.y + a.m[2][1] * v.z + a.m[3][1] * v.w,
              a.m[0][2] * v.x + a.m[1][2] * v.y + a.m[2][2] * v.z + a.m[3][2] * v.w,
              a.m[0][3] * v.x + a.m[1][3] * v.y + a.m[2][3] * v.z + a.m[3][3] * v.w);
}
static v3 mul3v(m3 a, v3 v) {
    return V3(a.m[0][0] * v.x + a.m[1][0] * v.y + a.m[2][0] * v.z,
              a.m[0][1] * v.x + a.m[1][1] * v.y + a.m[2][1] * v.z,
              a.m[0][2] * v.x + a.m[1][2] * v.y + a.m[2][2] * v.z);
}

/* GLSL inverse(mat4), as Mesa's builtin lowers it (the GLM cofactor scheme:
 * 2x2 sub-factors, adjugate, determinant from column 0, then adj / det with a
 * true division) — probed bit-exact against llvmpipe, DESIGN.md "Parity". */
static float t3(float a, float x, float b, float y, float c, float z) { return a * x - b * y + c * z; }
static m4 inverse4(m4 a) {
    const float(*m)[4] = a.m;
    float S00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float S01 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float S02 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float S03 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float S04 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float S05 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float S06 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float S07 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S08 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float S09 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float S10 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float S11 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S12 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float S13 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float S14 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float S15 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float S16 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float S17 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float S18 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    m4 adj;
    adj.m[0][0] = t3(m[1][1], S00, m[1][2], S01, m[1][3], S02);
    adj.m[1][0] = -t3(m[1][0], S00, m[1][2], S03, m[1][3], S04);
    adj.m[2][0] = t3(m[1][0], S01, m[1][1], S03, m[1][3], S05);
    adj.m[3][0] = -t3(m[1][0], S02, m[1][1], S04, m[1][2], S05);
    adj.m[0][1] = -t3(m[0][1], S00, m[0][2], S01, m[0][3], S02);
    adj.m[1][1] = t3(m[0][0], S00, m[0][2], S03, m[0][3], S04);
    adj.m[2][1] = -t3(m[0][0], S01, m[0][1], S03, m[0][3], S05);
    adj.m[3][1] = t3(m[0][0], S02, m[0][1], S04, m[0][2], S05);
    adj.m[0][2] = t3(m[0][1], S06, m[0][2], S07, m[0][3], S08);
    adj.m[1][2] = -t3(m[0][0], S06, m[0][2], S09, m[0][3], S10);
    adj.m[2][2] = t3(m[0][0], S11, m[0][1], S09, m[0][3], S12);
    adj.m[3][2] = -t3(m[0][0], S08, m[0][1], S10, m[0][2], S12);
    adj.m[0][3] = -t3(m[0][1], S13, m[0][2], S14, m[0][3], S15);
    adj.m[1][3] = t3(m[0][0], S13, m[0][2], S16, m[0][3], S17);
    adj.m[2][3] = -t3(m[0][0], S14, m[0][1], S16, m[0][3], S18);
    adj.m[3][3] = t3(m[0][0], S15, m[0][1], S17, m[0][2], S18);
    float det = m[0][0] * adj.m[0][0] + m[0][1] * adj.m[1][0] + m[0][2] * adj.m[2][0] + m[0][3] * adj.m[3][0];
    m4 r;
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++) r.m[c][row] = adj.m[c][row] / det;
    return r;
}

/* :432-437 */
static m4 translation_matrix(v3 t) {
    m4 r = ident4();
    r.m[3][0] = t.x; r.m[3][1] = t.y; r.m[3][2] = t.z; r.m[3][3] = 1.0f;
    return r;
}
/* :444-454 */
static m4 rotation_matrix_x(float deg) {
    float c = cosf(DEG_TO_RAD * deg), s = sinf(DEG_TO_RAD * deg);
    m4 r = ident4();
    r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = -s; r.m[2][2] = c;
    return r;
}
/* :460-470 */
static m4 rotation_matrix_y(float deg) {
    float c = cosf(DEG_TO_RAD * deg), s = sinf(DEG_TO_RAD * deg);
    m4 r = ident4();
    r.m[0][0] = c; r.m[0][2] = -s; r.m[2][0] = s; r.m[2][2] = c;
    return r;
}
/* :476-486 */
static m4 rotation_matrix_z(float deg) {
    float c = cosf(DEG_TO_RAD * deg), s = sinf(DEG_TO_RAD * deg);
    m4 r = ident4();
    r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = -s; r.m[1][1] = c;
    return r;
}
/* :492-503 (yaw about z, then pitch about x, then roll about y) */
static m4 rotation_matrix(v3 r) {
    m4 res = ident4();
    res = mul44(res, rotation_matrix_z(r.y));
    res = mul44(res, rotation_matrix_x(r.x));
    res = mul44(res, rotation_matrix_y(r.z));
    return res;
}
/* :529-532 */
static m4 calc_transform_matrix(v3 pos, v3 angles) { return mul44(translation_matrix(pos), rotation_matrix(angles)); }

/* :411-426 */
static m4 calc_projection_matrix(const rt_camera *c) {
    float q = 1.0f / tanf(DEG_TO_RAD * 0.5f * c->v_fov);
    float A = q / c->aspect;
    float B = (c->near_plane + c->far_plane) / (c->near_plane - c->far_plane);
    float C = (2.0f * c->near_plane * c->far_plane) / (c->near_plane - c->far_plane);
    m4 r;
    memset(&r, 0, sizeof r);
    r.m[0][0] = A; r.m[1][1] = q; r.m[2][2] = B; r.m[2][3] = -1.0f; r.m[3][2] = C;
    return r;
}
/* :538-545 */
static m4 calc_view_matrix(const rt_camera *c) {
    m4 flip = rotation_matrix_x(90.0f);
    return inverse4(mul44(calc_transform_matrix(ld3(c->position), ld3(c->angles)), flip));
}

/* ---- frame constants in float64 --------------------------------------
 * The camera unprojection inverse(proj*view) (:383) is ill-conditioned
 * (near/far = 1e-4): llvmpipe's float result carries optimiser-dependent
 * rounding (its compiler re-associates inexact float ops), which no float
 * restatement reproduces. The oracle therefore evaluates the frame constants
 * (camera matrices, per-object transforms of :650-652,:718) in float64 and
 * rounds each entry once to float32 — measured closer to llvmpipe than any
 * float32 order tried (DESIGN.md "Parity"). Per-pixel work stays float32. */
static int g_f64_frame = 1;
void oracle_set_f64_frame_constants(int on) { g_f64_frame = on; }

typedef struct { double m[4][4]; } dm4;
static dm4 d_ident(void) {
    dm4 r;
    memset(&r, 0, sizeof r);
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0;
    return r;
}
static dm4 d_mul(dm4 a, dm4 b) {
    dm4 r;
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++) {
            double acc = 0.0;
            for (int k = 0; k < 4; k++) acc += a.m[k][row] * b.m[c][k];
            r.m[c][row] = acc;
        }
    return r;
}
/* Gauss-Jordan with partial pivoting (float64). */
static dm4 d_inverse(dm4 a) {
    double M[4][8];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            M[r][c] = a.m[c][r];
            M[r][4 + c] = (r == c) ? 1.0 : 0.0;
        }
    for (int c = 0; c < 4; c++) {
        int p = c;
        for (int r = c + 1; r < 4; r++)
            if (fabs(M[r][c]) > fabs(M[p][c])) p = r;
        if (p != c)
            for (int k = 0; k < 8; k++) { double t = M[c][k]; M[c][k] = M[p][k]; M[p][k] = t; }
        double iv = 1.0 / M[c][c];
        for (int k = 0; k < 8; k++) M[c][k] *= iv;
        for (int r = 0; r < 4; r++)
            if (r != c) {
                double f = M[r][c];
                for (int k = 0; k < 8; k++) M[r][k] -= f * M[c][k];
            }
    }
    dm4 r;
    for (int row = 0; row < 4; row++)
        for (int c = 0; c < 4; c++) r.m[c][row] = M[row][4 + c];
    return r;
}
static dm4 d_rot(int axis, float deg) {
    double rad = (double)(DEG_TO_RAD * deg); /* the float argument GLSL forms */
    double c = cos(rad), s = sin(rad);
    dm4 r = d_ident();
    if (axis == 0) { r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = -s; r.m[2][2] = c; }
    if (axis == 1) { r.m[0][0] = c; r.m[0][2] = -s; r.m[2][0] = s; r.m[2][2] = c; }
    if (axis == 2) { r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = -s; r.m[1][1] = c; }
    return r;
}
static dm4 d_transform(v3 pos, v3 ang) {
    dm4 t = d_ident();
    t.m[3][0] = pos.x; t.m[3][1] = pos.y; t.m[3][2] = pos.z;
    dm4 r = d_mul(d_mul(d_rot(2, ang.y), d_rot(0, ang.x)), d_rot(1, ang.z));
    return d_mul(t, r);
}
static m4 d_round(dm4 a) {
    m4 r;
    for (int c = 0; c < 4; c++)
        for (int row = 0; row < 4; row++) r.m[c][row] = (float)a.m[c][row];
    return r;
}
/* Test knob: pin the unprojection matrix (column-major 16 floats, e.g. the
 * value llvmpipe computed for a fixture) instead of computing it. */
static int g_pinned_unproj = 0;
static m4 g_unproj;
void oracle_pin_unprojection(const float *m16) {
    g_pinned_unproj = m16 != NULL;
    if (m16) memcpy(g_unproj.m, m16, 64);
}
static m4 camera_unprojection(const rt_camera *c) {
    if (g_pinned_unproj) return g_unproj;
    if (!g_f64_frame) return inverse4(mul44(calc_projection_matrix(c), calc_view_matrix(c)));
    double q = 1.0 / tan((double)(DEG_TO_RAD * 0.5f * c->v_fov));
    double n = c->near_plane, f = c->far_plane;
    dm4 P;
    memset(&P, 0, sizeof P);
    P.m[0][0] = q / c->aspect; P.m[1][1] = q; P.m[2][2] = (n + f) / (n - f); P.m[2][3] = -1.0;
    P.m[3][2] = (2.0 * n * f) / (n - f);
    dm4 V = d_inverse(d_mul(d_transform(ld3(c->position), ld3(c->angles)), d_rot(0, 90.0f)));
    return d_round(d_inverse(d_mul(P, V)));
}
/* the frame's unprojection: pinned, or the reference orbit camera as
 * llvmpipe computes it (cam == NULL), or an explicit camera in float64 */
static void gl_reference_matrices(float time, m4 *inv, m4 *view, m4 *proj);
static m4 frame_unprojection(const rt_camera *cam, float time) {
    if (g_pinned_unproj || cam) {
        rt_camera c;
        if (!cam) {
            oracle_reference_camera(time, &c);
            cam = &c;
        }
        return camera_unprojection(cam);
    }
    m4 inv;
    gl_reference_matrices(time, &inv, NULL, NULL);
    return inv;
}
/* per-object transforms of intersect_box_object (:650-652, :718): as
 * llvmpipe evaluates them (gl_object_transforms below) */
static void gl_object_transforms(v3 pos, v3 ang, m4 *l2w, m4 *w2l, m3 *nrm);
static void object_transforms(v3 pos, v3 ang, m4 *l2w, m4 *w2l, m3 *nrm) { gl_object_transforms(pos, ang, l2w, w2l, nrm); }

/* ---- reference scene ------------------------------------------------- */
static void set_mat(rt_material *m, v4 amb, v4 dif, v4 spe, float shin, v4 emi, float refl, float transp,
                    float ior) {
    memcpy(m->ambient, &amb, 16); memcpy(m->diffuse, &dif, 16); memcpy(m->specular, &spe, 16);
    m->shininess = shin; memcpy(m->emissive, &emi, 16);
    m->reflectivity = refl; m->transparency = transp; m->refraction_index = ior;
}
static v4 S4(float s) { return V4(s, s, s, s); }

/* :74-157 */
void oracle_reference_materials(rt_material out[7]) {
    set_mat(&out[0], S4(1), V4(0.5f, 0, 0, 1), S4(1), 4.0f, S4(0), 1.0f, 0.0f, 1.5f); /* material1 */
    set_mat(&out[1], S4(1), V4(0.3f, 0.6f, 0.3f, 1), S4(1), 4.0f, S4(0), 1.0f, 0.0f, 1.5f); /* material2 */
    set_mat(&out[2], S4(1), V4(1, 0, 0, 1), S4(1), 10.0f, S4(0), 0.8f, 0.4f, 1.5f); /* red_glass */
    set_mat(&out[3], S4(1), V4(0, 1, 0, 1), S4(1), 10.0f, S4(0), 0.4f, 0.6f, 1.5f); /* green_glass */
    set_mat(&out[4], S4(1), V4(0, 0, 1, 1), S4(1), 10.0f, S4(0), 0.4f, 0.6f, 1.5f); /* blue_glass */
    set_mat(&out[5], S4(1), V4(0.6f, 0.6f, 0.6f, 1), S4(1), 4.0f, S4(0), 1.0f, 0.0f, 1.0f); /* mirror */
    set_mat(&out[6], S4(0.5f), S4(0.4f), S4(0.3f), 3.0f, S4(0), 0.3f, 0.0f, 1.0f); /* wall */
}

/* :199-224 */
void oracle_reference_lights(rt_light out[3]) {
    const float pos[3][3] = {{0.1f, 0.1f, 0.1f}, {7, 7, 2}, {3, -3, 4}};
    const v4 amb[3] = {S4(0.3f), S4(0.05f), S4(0.05f)};
    const v4 dif[3] = {S4(0.0f), S4(1.0f), V4(1, 0, 0, 1)};
    const v4 spe[3] = {S4(0.0f), S4(1.0f), V4(1, 0, 0, 1)};
    for (int i = 0; i < 3; i++) {
        memcpy(out[i].position, pos[i], 12);
        memcpy(out[i].ambient, &amb[i], 16);
        memcpy(out[i].diffuse, &dif[i], 16);
        memcpy(out[i].specular, &spe[i], 16);
    }
}

static void set_obj(rt_object *o, v3 mins, v3 maxs, float radius, v3 pos, v3 ang, int mat) {
    memcpy(o->box_mins, &mins, 12); memcpy(o->box_maxs, &maxs, 12);
    o->radius = radius; memcpy(o->position, &pos, 12); memcpy(o->angles, &ang, 12);
    o->material = mat;
}

/* ---- the reference orbit camera as llvmpipe compiles it ----------------
 * (DESIGN.md "Parity"; pinned by tests/golden/camera_llvmpipe.npz, made by
 * tests/golden/make_camera_golden.py from the reference's own camera
 * functions.) Run-time sin/cos are gallivm's polynomials with fused
 * multiply-adds; constant-only terms are folded in float; x*0, x*1, x+0
 * vanish; (x * #a) * #b becomes x * #(a b); mod()+90 becomes (x + 90) -
 * 360 floor(x/360); nothing else is fused or reordered. */
static float gv_sincos(float a, int want_cos) {
    float xa = fabsf(a);
    int j = (int)(xa * 1.27323954473516f);
    int jp = j + 1, je = jp & ~1;
    float yj = (float)je;
    uint32_t sign;
    int poly;
    if (want_cos) {
        sign = (uint32_t)((~(je - 2)) & 4) << 29;
        poly = ((je - 2) & 2) == 0;
    } else {
        uint32_t ab;
        memcpy(&ab, &a, 4);
        sign = ((uint32_t)(jp & 4) << 29) ^ (ab & 0x80000000u);
        poly = (je & 2) == 0;
    }
    float x = fmaf(yj, -0.78515625f, xa);
    x = fmaf(yj, -2.4187564849853515625e-4f, x);
    x = fmaf(yj, -3.77489497744594108e-8f, x);
    float z = x * x;
    float c = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    c = fmaf(c, z, 4.166664568298827e-2f);
    c = c * z;
    c = c * z;
    c = fmaf(z, -0.5f, c);
    c = c + 1.0f;
    float sn = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    sn = fmaf(sn, z, -1.6666654611e-1f);
    sn = sn * z;
    sn = fmaf(sn, x, x);
    float r = poly ? sn : c;
    uint32_t rb;
    memcpy(&rb, &r, 4);
    rb ^= sign;
    memcpy(&r, &rb, 4);
    return r;
}
float oracle_gl_sin(float a) { return gv_sincos(a, 0); }
float oracle_gl_cos(float a) { return gv_sincos(a, 1); }

/* a value of the compiled camera chain: kind 0 run-time, 1 compile-time
 * constant, 2 run-time `b` times the constant `k` */
typedef struct { float v; int kind; float b, k; } gv;
static gv gv_c(float v) { gv r = {v, 1, 0, 0}; return r; }
static gv gv_r(float v) { gv r = {v, 0, 0, 0}; return r; }
static gv gv_neg(gv a) { a.v = -a.v; a.k = -a.k; return a; }
static gv gv_mul(gv a, gv b) {
    if (a.kind == 1 && b.kind == 1) return gv_c(a.v * b.v);
    if (a.kind != 1 && b.kind != 1) return gv_r(a.v * b.v);
    gv c = a.kind == 1 ? a : b, x = a.kind == 1 ? b : a;
    if (c.v == 0.0f) return gv_c(0.0f);
    if (c.v == 1.0f) return x;
    if (c.v == -1.0f) return gv_neg(x);
    gv r;
    r.kind = 2;
    r.b = x.kind == 2 ? x.b : x.v;
    r.k = x.kind == 2 ? x.k * c.v : c.v;
    r.v = r.b * r.k;
    return r;
}
static gv gv_add(gv a, gv b) {
    if (a.kind == 1 && b.kind == 1) return gv_c(a.v + b.v);
    if (a.kind == 1 && a.v == 0.0f) return b;
    if (b.kind == 1 && b.v == 0.0f) return a;
    return gv_r(a.v + b.v);
}
static gv gv_sub(gv a, gv b) { return gv_add(a, gv_neg(b)); }
typedef struct { gv m[4][4]; } gm; /* m[col][row] */
static gm gm_ident(void) {
    gm r;
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) r.m[c][w] = gv_c(c == w ? 1.0f : 0.0f);
    return r;
}
static gm gm_mul(gm a, gm b) { /* column c = a0 b.x + a1 b.y + a2 b.z + a3 b.w */
    gm r;
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) {
            gv acc = gv_mul(a.m[0][w], b.m[c][0]);
            for (int k = 1; k < 4; k++) acc = gv_add(acc, gv_mul(a.m[k][w], b.m[c][k]));
            r.m[c][w] = acc;
        }
    return r;
}
static gv gv_d(gv a, gv b, gv c, gv e) { return gv_sub(gv_mul(a, b), gv_mul(c, e)); }
static gv gv_t3(gv a, gv x, gv b, gv y, gv c, gv z) { return gv_add(gv_sub(gv_mul(a, x), gv_mul(b, y)), gv_mul(c, z)); }
static gm gm_inverse(gm A) { /* Mesa's inverse(mat4), as inverse4 above */
    gv(*m)[4] = A.m;
    gv S00 = gv_d(m[2][2], m[3][3], m[3][2], m[2][3]), S01 = gv_d(m[2][1], m[3][3], m[3][1], m[2][3]);
    gv S02 = gv_d(m[2][1], m[3][2], m[3][1], m[2][2]), S03 = gv_d(m[2][0], m[3][3], m[3][0], m[2][3]);
    gv S04 = gv_d(m[2][0], m[3][2], m[3][0], m[2][2]), S05 = gv_d(m[2][0], m[3][1], m[3][0], m[2][1]);
    gv S06 = gv_d(m[1][2], m[3][3], m[3][2], m[1][3]), S07 = gv_d(m[1][1], m[3][3], m[3][1], m[1][3]);
    gv S08 = gv_d(m[1][1], m[3][2], m[3][1], m[1][2]), S09 = gv_d(m[1][0], m[3][3], m[3][0], m[1][3]);
    gv S10 = gv_d(m[1][0], m[3][2], m[3][0], m[1][2]), S11 = gv_d(m[1][1], m[3][3], m[3][1], m[1][3]);
    gv S12 = gv_d(m[1][0], m[3][1], m[3][0], m[1][1]), S13 = gv_d(m[1][2], m[2][3], m[2][2], m[1][3]);
    gv S14 = gv_d(m[1][1], m[2][3], m[2][1], m[1][3]), S15 = gv_d(m[1][1], m[2][2], m[2][1], m[1][2]);
    gv S16 = gv_d(m[1][0], m[2][3], m[2][0], m[1][3]), S17 = gv_d(m[1][0], m[2][2], m[2][0], m[1][2]);
    gv S18 = gv_d(m[1][0], m[2][1], m[2][0], m[1][1]);
    gm a;
    a.m[0][0] = gv_t3(m[1][1], S00, m[1][2], S01, m[1][3], S02);
    a.m[1][0] = gv_neg(gv_t3(m[1][0], S00, m[1][2], S03, m[1][3], S04));
    a.m[2][0] = gv_t3(m[1][0], S01, m[1][1], S03, m[1][3], S05);
    a.m[3][0] = gv_neg(gv_t3(m[1][0], S02, m[1][1], S04, m[1][2], S05));
    a.m[0][1] = gv_neg(gv_t3(m[0][1], S00, m[0][2], S01, m[0][3], S02));
    a.m[1][1] = gv_t3(m[0][0], S00, m[0][2], S03, m[0][3], S04);
    a.m[2][1] = gv_neg(gv_t3(m[0][0], S01, m[0][1], S03, m[0][3], S05));
    a.m[3][1] = gv_t3(m[0][0], S02, m[0][1], S04, m[0][2], S05);
    a.m[0][2] = gv_t3(m[0][1], S06, m[0][2], S07, m[0][3], S08);
    a.m[1][2] = gv_neg(gv_t3(m[0][0], S06, m[0][2], S09, m[0][3], S10));
    a.m[2][2] = gv_t3(m[0][0], S11, m[0][1], S09, m[0][3], S12);
    a.m[3][2] = gv_neg(gv_t3(m[0][0], S08, m[0][1], S10, m[0][2], S12));
    a.m[0][3] = gv_neg(gv_t3(m[0][1], S13, m[0][2], S14, m[0][3], S15));
    a.m[1][3] = gv_t3(m[0][0], S13, m[0][2], S16, m[0][3], S17);
    a.m[2][3] = gv_neg(gv_t3(m[0][0], S14, m[0][1], S16, m[0][3], S18));
    a.m[3][3] = gv_t3(m[0][0], S15, m[0][1], S17, m[0][2], S18);
    gv det = gv_add(gv_mul(m[0][0], a.m[0][0]),
                    gv_add(gv_mul(m[0][1], a.m[1][0]), gv_add(gv_mul(m[0][2], a.m[2][0]), gv_mul(m[0][3], a.m[3][0]))));
    gm r;
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) {
            gv x = a.m[c][w];
            r.m[c][w] = (x.kind == 1 && det.kind == 1) ? gv_c(x.v / det.v)
                        : (x.kind == 1 && x.v == 0.0f) ? gv_c(0.0f) : gv_r(x.v / det.v);
        }
    return r;
}
static gm gm_rot(int axis, gv c, gv s) { /* :444-486 */
    gm r = gm_ident();
    if (axis == 0) { r.m[1][1] = c; r.m[1][2] = s; r.m[2][1] = gv_neg(s); r.m[2][2] = c; }
    if (axis == 1) { r.m[0][0] = c; r.m[0][2] = gv_neg(s); r.m[2][0] = s; r.m[2][2] = c; }
    if (axis == 2) { r.m[0][0] = c; r.m[0][1] = s; r.m[1][0] = gv_neg(s); r.m[1][1] = c; }
    return r;
}
/* inverse(proj_mat * view_mat) (:383), view_mat (:368) and proj_mat of the
 * orbit camera at `time` as llvmpipe computes them */
static void gl_reference_matrices(float time, m4 *inv, m4 *view, m4 *proj) {
    float speed = time * 0.4f + 0.5f;                                    /* :343 */
    float x = speed * (180.0f / 3.1416f);
    float yaw = (x + 90.0f) - 360.0f * floorf(x / 360.0f);              /* :353 as compiled */
    float a = DEG_TO_RAD * yaw;
    gm Rz = gm_rot(2, gv_r(gv_sincos(a, 1)), gv_r(gv_sincos(a, 0)));
    gm R = gm_mul(gm_mul(gm_mul(gm_ident(), Rz), gm_rot(0, gv_c(1.0f), gv_c(0.0f))), gm_rot(1, gv_c(1.0f), gv_c(0.0f)));
    gm T = gm_ident();
    T.m[3][0] = gv_mul(gv_c(10.0f), gv_r(gv_sincos(speed, 1)));
    T.m[3][1] = gv_mul(gv_c(10.0f), gv_r(gv_sincos(speed, 0)));
    T.m[3][2] = gv_c(0.0f);
    float c90 = cosf(DEG_TO_RAD * 90.0f); /* folded at compile time (host libm) */
    gm V = gm_inverse(gm_mul(gm_mul(T, R), gm_rot(0, gv_c(c90), gv_c(1.0f))));
    gm P;
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) P.m[c][w] = gv_c(0.0f);
    float q = 1.0f / (sinf(DEG_TO_RAD * 0.5f * 90.0f) / cosf(DEG_TO_RAD * 0.5f * 90.0f)); /* tan = sin/cos, folded */
    P.m[0][0] = gv_c(q / (16.0f / 9.0f));
    P.m[1][1] = gv_c(q);
    P.m[2][2] = gv_c((0.1f + 1000.0f) / (0.1f - 1000.0f));
    P.m[2][3] = gv_c(-1.0f);
    P.m[3][2] = gv_c((2.0f * 0.1f * 1000.0f) / (0.1f - 1000.0f));
    gm U = gm_inverse(gm_mul(P, V));
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) {
            if (inv) inv->m[c][w] = U.m[c][w].v;
            if (view) view->m[c][w] = V.m[c][w].v;
            if (proj) proj->m[c][w] = P.m[c][w].v;
        }
}

/* The box transforms of intersect_box_object as llvmpipe evaluates them:
 * the object's fields are run-time values (objects[] is indexed by the loop
 * counter), the functions' own constants fold (gv rules); the normal matrix
 * transpose(inverse(mat3(L))) with Mesa's mat3 inverse (normal_matrix). */
static gv gv_div(gv a, gv det) {
    if (a.kind == 1 && det.kind == 1) return gv_c(a.v / det.v);
    if (a.kind == 1 && a.v == 0.0f) return gv_c(0.0f);
    return gv_r(a.v / det.v);
}
static gm gm_rot_deg(int axis, float deg) { /* rotation_matrix_{x,y,z} of a run-time angle */
    float a = gv_mul(gv_c(DEG_TO_RAD), gv_r(deg)).v;
    return gm_rot(axis, gv_r(gv_sincos(a, 1)), gv_r(gv_sincos(a, 0)));
}
static void gl_object_transforms(v3 pos, v3 ang, m4 *l2w, m4 *w2l, m3 *nrm) {
    gm T = gm_ident();
    T.m[3][0] = gv_r(pos.x); T.m[3][1] = gv_r(pos.y); T.m[3][2] = gv_r(pos.z);
    gm R = gm_mul(gm_mul(gm_mul(gm_ident(), gm_rot_deg(2, ang.y)), gm_rot_deg(0, ang.x)), gm_rot_deg(1, ang.z));
    gm L = gm_mul(T, R), W = gm_inverse(L);
    gv(*m)[4] = L.m;
    gv f0 = gv_d(m[1][1], m[2][2], m[2][1], m[1][2]);
    gv f1 = gv_d(m[1][0], m[2][2], m[2][0], m[1][2]);
    gv f2 = gv_d(m[1][0], m[2][1], m[2][0], m[1][1]);
    gv det = gv_add(gv_sub(gv_mul(m[0][0], f0), gv_mul(m[0][1], f1)), gv_mul(m[0][2], f2));
    gv inv[3][3]; /* [col][row] */
    inv[0][0] = gv_div(f0, det);
    inv[1][0] = gv_div(gv_neg(f1), det);
    inv[2][0] = gv_div(f2, det);
    inv[0][1] = gv_div(gv_neg(gv_d(m[0][1], m[2][2], m[2][1], m[0][2])), det);
    inv[1][1] = gv_div(gv_d(m[0][0], m[2][2], m[2][0], m[0][2]), det);
    inv[2][1] = gv_div(gv_neg(gv_d(m[0][0], m[2][1], m[2][0], m[0][1])), det);
    inv[0][2] = gv_div(gv_d(m[0][1], m[1][2], m[1][1], m[0][2]), det);
    inv[1][2] = gv_div(gv_neg(gv_d(m[0][0], m[1][2], m[1][0], m[0][2])), det);
    inv[2][2] = gv_div(gv_d(m[0][0], m[1][1], m[1][0], m[0][1]), det);
    for (int c = 0; c < 4; c++)
        for (int w = 0; w < 4; w++) {
            l2w->m[c][w] = L.m[c][w].v;
            w2l->m[c][w] = W.m[c][w].v;
        }
    for (int c = 0; c < 3; c++)
        for (int w = 0; w < 3; w++) nrm->m[c][w] = inv[w][c].v; /* transpose */
}

/* Test export: gl_object_transforms of an object, column-major:
 * out[0..16) local_to_world, out[16..32) world_to_local, out[32..41) normal. */
void oracle_object_transforms(const rt_object *o, float out[41]) {
    m4 l, w;
    m3 n;
    gl_object_transforms(ld3(o->position), ld3(o->angles), &l, &w, &n);
    memcpy(out, l.m, 64);
    memcpy(out + 16, w.m, 64);
    memcpy(out + 32, n.m, 36);
}

/* :236-237, :261-321. scaled_time * k = (time * time_scale) * k is compiled
 * as time * (time_scale * k) (constant products fold; probed on llvmpipe). */
static float st_k(float time, float k) { return time * (0.4f * k); }
void oracle_reference_objects(float time, rt_object out[5]) {
    v3 z = V3(0, 0, 0);
    set_obj(&out[0], V3(-11, -11, -11), V3(11, 11, 11), -1.0f, z, z, 6);
    float s = 0.5f * gv_sincos(st_k(time, 0.5f), 0) + 1.5f; /* run-time sin: gallivm */
    set_obj(&out[1], mul3s(V3(-1, -1, -1), s), mul3s(V3(1, 1, 1), s), -1.0f, V3(0, 0, gv_sincos(st_k(time, 3.0f), 0)),
            V3(0, st_k(time, 90.0f), 0), 5);
    set_obj(&out[2], V3(-10, -10, -1), V3(10, 10, 1), -1.0f, V3(0, 0, -3),
            V3(gv_sincos(st_k(time, 5.0f), 0) * 10.0f, 45, 0), 3);
    set_obj(&out[3], V3(-1, -1, -2), V3(1, 1, 2), -1.0f, V3(3, 4, 1),
            V3(45.0f + st_k(time, 45.0f), 0, 45.0f + st_k(time, 180.0f)), 4);
    set_obj(&out[4], z, z, 2.0f, V3(-3, 4, 1), z, 2);
}

/* :334-364 */
void oracle_reference_camera(float time, rt_camera *c) {
    float radius = 10.0f;
    float speed = time * 0.4f + 0.5f;
    c->position[0] = radius * gv_sincos(speed, 1); /* run-time cos / sin: gallivm */
    c->position[1] = radius * gv_sincos(speed, 0);
    c->position[2] = 0.0f;
    float x = 1.0f * speed * (180.0f / 3.1416f);
    float yaw = (x + 90.0f) - 360.0f * floorf(x / 360.0f); /* GLSL mod + 90, as compiled */
    c->angles[0] = 0.0f; c->angles[1] = yaw; c->angles[2] = 0.0f;
    c->near_plane = 0.1f; c->far_plane = 1000.0f; c->aspect = 16.0f / 9.0f; c->v_fov = 90.0f;
}

/* Camera matrices of main() (:366-367, :383), column-major, for probing:
 * out[0..16) inverse(proj*view), out[16..32) view, out[32..48) proj. */
void oracle_camera_matrices(const rt_camera *cam_in, float time, float out[48]) {
    rt_camera cam;
    if (cam_in) cam = *cam_in;
    else oracle_reference_camera(time, &cam);
    m4 proj, view, inv;
    if (cam_in) {
        proj = calc_projection_matrix(&cam);
        view = calc_view_matrix(&cam);
        inv = inverse4(mul44(proj, view));
    } else {
        gl_reference_matrices(time, &inv, &view, &proj);
    }
    memcpy(out, inv.m, 64);
    memcpy(out + 16, view.m, 64);
    memcpy(out + 32, proj.m, 64);
}

/* ---- per-frame precompute (values identical to the per-ray GLSL ones) - */
typedef struct {
    int kind; /* 0 skip, 1 box, 2 sphere (:749-771) */
    v3 mins, maxs, pos;
    float radius;
    m4 l2w, w2l; /* :650-652 */
    m3 nrm;      /* :718 */
    const rt_material *mat;
} obj_t;

typedef struct {
    const obj_t *o;
    int n;
    const rt_light *lights;
    int nl;
} scene_t;

typedef struct { v3 start, dir; } ray_t;                          /* :25-31 */
typedef struct { float t; v3 p, n; int inside, object_index; } coll_t; /* :561-573 */

/* :583-640 */
static coll_t intersect_sphere_object(ray_t r, const obj_t *o) {
    coll_t c;
    memset(&c, 0, sizeof c);
    float radius = o->radius;
    float qa = dot3(r.dir, r.dir);
    float qb = dot3(mul3s(r.dir, 2.0f), sub3(r.start, o->pos));
    v3 oc = sub3(r.start, o->pos);
    float qc = dot3(oc, oc) - radius * radius;
    float qd = qb * qb - 4.0f * qa * qc;
    c.inside = 0;
    if (qd < 0.0f) { c.t = -1.0f; return c; }
    float sqrt_qd = sqrtf(qd);
    float t1 = (-qb + sqrt_qd) / (2.0f * qa);
    float t2 = (-qb - sqrt_qd) / (2.0f * qa);
    float t_near = minf(t1, t2);
    float t_far = maxf(t1, t2);
    c.t = t_near;
    if (t_far < 0.0f) { c.t = -1.0f; return c; }
    if (t_near < 0.0f) { c.t = t_far; c.inside = 1; }
    c.p = add3(r.start, mul3s(r.dir, c.t));
    c.n = normalize3(sub3(c.p, o->pos));
    if (c.inside) c.n = mul3s(c.n, -1.0f);
    return c;
}

/* :647-724 */
static coll_t intersect_box_object(ray_t r, const obj_t *o) {
    coll_t c;
    memset(&c, 0, sizeof c);
    v4 s4 = mul4v(o->w2l, V4(r.start.x, r.start.y, r.start.z, 1.0f));
    v4 d4 = mul4v(o->w2l, V4(r.dir.x, r.dir.y, r.dir.z, 0.0f));
    v3 rs = V3(s4.x, s4.y, s4.z), rd = V3(d4.x, d4.y, d4.z);
    v3 tmn = V3((o->mins.x - rs.x) / rd.x, (o->mins.y - rs.y) / rd.y, (o->mins.z - rs.z) / rd.z);
    v3 tmx = V3((o->maxs.x - rs.x) / rd.x, (o->maxs.y - rs.y) / rd.y, (o->maxs.z - rs.z) / rd.z);
    v3 t1 = V3(minf(tmn.x, tmx.x), minf(tmn.y, tmx.y), minf(tmn.z, tmx.z));
    v3 t2 = V3(maxf(tmn.x, tmx.x), maxf(tmn.y, tmx.y), maxf(tmn.z, tmx.z));
    float t_near = maxf(maxf(t1.x, t1.y), t1.z);
    float t_far = minf(minf(t2.x, t2.y), t2.z);
    c.t = t_near;
    c.inside = 0;
    if (t_near >= t_far || t_far <= 0.0f) { c.t = -1.0f; return c; }
    float intersection = t_near;
    v3 boundary = t1;
    if (t_near < 0.0f) { c.t = t_far; intersection = t_far; boundary = t2; c.inside = 1; }
    int face = 0;
    if (intersection == boundary.y) face = 1;
    else if (intersection == boundary.z) face = 2;
    float nn[3] = {0, 0, 0};
    nn[face] = 1.0f;
    v3 n = V3(nn[0], nn[1], nn[2]);
    if (comp3(rd, face) > 0.0f) n = mul3s(n, -1.0f);
    c.n = mul3v(o->nrm, n);
    v3 lp = add3(rs, mul3s(rd, c.t));
    v4 p4 = mul4v(o->l2w, V4(lp.x, lp.y, lp.z, 1.0f));
    c.p = V3(p4.x, p4.y, p4.z);
    return c;
}

/* :738-782 */
static coll_t get_closest_collision(const scene_t *S, ray_t r) {
    float closest = 10000.0f;
    coll_t cc;
    memset(&cc, 0, sizeof cc);
    cc.object_index = -1;
    for (int i = 0; i < S->n; i++) {
        coll_t c;
        if (S->o[i].kind == 1) {
            c = intersect_box_object(r, &S->o[i]);
            if (c.t <= 0.0f) continue;
        } else if (S->o[i].kind == 2) {
            c = intersect_sphere_object(r, &S->o[i]);
            if (c.t <= 0.0f) continue;
        } else {
            continue;
        }
        if (c.t < closest) {
            closest = c.t;
            cc = c;
            cc.object_index = i;
        }
    }
    return cc;
}

static int in_shadow(const scene_t *S, coll_t c, const rt_light *L) {
    ray_t lr;
    lr.start = add3(c.p, mul3s(c.n, 0.01f));
    lr.dir = sub3(ld3(L->position), c.p);
    coll_t cs = get_closest_collision(S, lr);
    return cs.object_index != -1 && cs.t < 1.0f;
}

/* :789-840 */
static v3 ads_phong_lighting(const scene_t *S, ray_t r, coll_t c) {
    const rt_material *mat = S->o[c.object_index].mat;
    v4 ambient = S4(0), diffuse = S4(0), specular = S4(0);
    for (int j = 0; j < S->nl; j++) {
        const rt_light *L = &S->lights[j];
        ambient = add4(ambient, mul4(ld4(L->ambient), ld4(mat->ambient)));
        v3 light_dir = normalize3(sub3(ld3(L->position), c.p));
        if (!in_shadow(S, c, L)) {
            v3 light_ref = normalize3(reflect3(neg3(light_dir), c.n));
            float cos_theta = dot3(light_dir, c.n);
            float cos_phi = dot3(normalize3(neg3(r.dir)), light_ref);
            diffuse = add4(diffuse, mul4s(mul4(ld4(L->diffuse), ld4(mat->diffuse)), maxf(cos_theta, 0.0f)));
            specular = add4(specular, mul4s(mul4(ld4(L->specular), ld4(mat->specular)),
                                            glsl_pow(maxf(cos_phi, 0.0f), mat->shininess)));
        }
    }
    v4 ph = add4(add4(add4(ambient, diffuse), specular), ld4(mat->emissive));
    return mul3s(V3(ph.x, ph.y, ph.z), ph.w);
}

/* ---- the stack machine, :848-1105 ------------------------------------ */
enum { RAY_TYPE_REFLECTION = 1, RAY_TYPE_REFRACTION = 2, STACK_SIZE = 100 };
typedef struct {
    int type, depth, counter;
    v3 phong_color, reflected_color, refracted_color;
    int reflected, refracted;
    v3 final_color;
    ray_t ray;
    coll_t collision;
    int is_null;
} elem_t;

typedef struct {
    elem_t stack[STACK_SIZE];
    int sp;
    elem_t popped;
} machine_t;

static elem_t null_elem(void) {
    elem_t e;
    memset(&e, 0, sizeof e);
    e.depth = -1; e.counter = -1; e.collision.t = -1.0f; e.collision.object_index = -1;
    e.is_null = 1;
    return e;
}

/* :886-909 */
static void push_elem(machine_t *M, ray_t r, int depth, int type) {
    if (M->sp >= STACK_SIZE) return;
    elem_t e = null_elem();
    e.is_null = 0;
    e.type = type; e.depth = depth; e.counter = 0;
    e.ray = r;
    M->stack[M->sp++] = e;
}
/* :914-922 */
static void pop_elem(machine_t *M) {
    M->sp--;
    M->popped = M->stack[M->sp];
    M->stack[M->sp] = null_elem();
}

/* :930-1065 — one phase per call */
static void process_elem(const scene_t *S, machine_t *M, int idx) {
    elem_t *e = &M->stack[idx];
    if (!M->popped.is_null) {
        if (M->popped.type == RAY_TYPE_REFLECTION) e->reflected_color = M->popped.final_color;
        else if (M->popped.type == RAY_TYPE_REFRACTION) e->refracted_color = M->popped.final_color;
        M->popped = null_elem();
    }
    ray_t r = e->ray;
    coll_t c = e->collision;
    if (e->counter < 5) {
        if (e->counter == 0) {
            c = get_closest_collision(S, r);
            if (c.object_index == -1) { pop_elem(M); return; }
            e->collision = c;
        }
        if (e->counter == 1) e->phong_color = ads_phong_lighting(S, r, c);
        if (e->counter == 2 && e->depth > 0 && S->o[c.object_index].mat->reflectivity > 0.0f) {
            ray_t rr;
            rr.start = add3(c.p, mul3s(c.n, 0.001f));
            rr.dir = reflect3(r.dir, c.n);
            int d = e->depth - 1;
            e->reflected = 1;
            push_elem(M, rr, d, RAY_TYPE_REFLECTION);
        }
        if (e->counter == 3 && e->depth > 0 && S->o[c.object_index].mat->transparency > 0.0f) {
            ray_t tr;
            tr.start = sub3(c.p, mul3s(c.n, 0.001f));
            float ratio = 1.0f / S->o[c.object_index].mat->refraction_index;
            if (c.inside) ratio = 1.0f / ratio;
            tr.dir = refract3(r.dir, c.n, ratio);
            int d = e->depth - 1;
            e->refracted = 1;
            push_elem(M, tr, d, RAY_TYPE_REFRACTION);
        }
        if (e->counter == 4) {
            const rt_material *mat = S->o[c.object_index].mat;
            v3 fc = e->phong_color;
            if (e->reflected) fc = mix3(fc, e->reflected_color, mat->reflectivity);
            if (e->refracted) fc = mix3(fc, e->refracted_color, mat->transparency);
            e->final_color = fc;
        }
        e->counter++;
        return;
    }
    pop_elem(M);
}

/* :1071-1105 */
static v3 recursive_raytrace(const scene_t *S, machine_t *M, ray_t r, int max_depth) {
    M->sp = 0;
    M->popped = null_elem();
    M->popped.is_null = 0; /* the global starts zeroed (type 0), not null */
    M->popped.type = 0;
    push_elem(M, r, max_depth, RAY_TYPE_REFLECTION);
    int break_counter = 0;
    const int break_at = 10000;
    while (M->sp > 0) {
        if (break_counter++ > break_at) break;
        process_elem(S, M, M->sp - 1);
    }
    if (break_counter > break_at) return V3(1.0f, 0.0f, 0.0f);
    return M->popped.final_color;
}

/* Monte-Carlo extension: the same counter-based jitter hash as the kernel. */
static uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
    return h;
}
static float jitter_u(uint32_t seed, uint32_t sample, uint32_t pixel, uint32_t axis) {
    uint32_t h = mix32(seed * 0x9E3779B1u + 0x7F4A7C15u);
    h = mix32(h ^ (sample * 0x85EBCA77u));
    h = mix32(h ^ (pixel * 0xC2B2AE3Du + axis));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

/* :377-392 with optional sub-pixel offsets (0 = the reference's ray). */
static ray_t camera_ray(m4 inv, const rt_camera *cam, int x, int y, int hw, int hh, float jx, float jy) {
    float vx = ((float)(x - hw) + jx) / (float)hw;
    float vy = ((float)(y - hh) + jy) / (float)hh;
    v4 ws = mul4v(inv, V4(vx, vy, 0.5f, 1.0f));
    ws = V4(ws.x / ws.w, ws.y / ws.w, ws.z / ws.w, ws.w / ws.w);
    v4 we = mul4v(inv, V4(vx, vy, 1.0f, 1.0f));
    we = V4(we.x / we.w, we.y / we.w, we.z / we.w, we.w / we.w);
    ray_t r;
    r.start = ld3(cam->position);
    r.dir = normalize3(V3(we.x - ws.x, we.y - ws.y, we.z - ws.z));
    return r;
}

static obj_t *prepare_objects(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats) {
    obj_t *o = (obj_t *)calloc((size_t)(n_objs > 0 ? n_objs : 1), sizeof(obj_t));
    for (int i = 0; i < n_objs; i++) {
        const rt_object *s = &objs[i];
        int is_box = !(s->box_mins[0] == 0.0f && s->box_mins[1] == 0.0f && s->box_mins[2] == 0.0f &&
                       s->box_maxs[0] == 0.0f && s->box_maxs[1] == 0.0f && s->box_maxs[2] == 0.0f);
        o[i].kind = is_box ? 1 : (s->radius != -1.0f ? 2 : 0);
        if (s->material < 0 || s->material >= n_mats) { free(o); return NULL; }
        o[i].mat = &mats[s->material];
        o[i].mins = ld3(s->box_mins); o[i].maxs = ld3(s->box_maxs);
        o[i].pos = ld3(s->position); o[i].radius = s->radius;
        object_transforms(o[i].pos, ld3(s->angles), &o[i].l2w, &o[i].w2l, &o[i].nrm);
    }
    return o;
}

/* Monte-Carlo accumulation (see rt_render_accumulate in include/rt.h):
 * accum[(y-row0)*W + x] += sum over samples s in order of the colour. */
int oracle_render_accumulate(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats,
                             const rt_light *lights, int n_lights, const rt_camera *cam_in, float time, int width,
                             int height, int max_depth, int spp, int sample0, uint32_t seed, int jitter, int row0,
                             int row1, int n_threads, float *accum) {
    if (!objs || n_objs < 0 || !mats || n_mats <= 0 || (n_lights > 0 && !lights) || n_lights < 0 || width <= 0 ||
        height <= 0 || row0 < 0 || row1 > height || row0 > row1 || max_depth < 0 || spp <= 0 || !accum)
        return -1;
    obj_t *o = prepare_objects(objs, n_objs, mats, n_mats);
    if (!o) return -1;
    scene_t S = {o, n_objs, lights, n_lights};
    rt_camera cam;
    if (cam_in) cam = *cam_in;
    else oracle_reference_camera(time, &cam);
    m4 inv = frame_unprojection(cam_in ? &cam : NULL, time);
    int hw = width / 2, hh = height / 2;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : omp_get_max_threads())
    for (int yy = 0; yy < row1 - row0; yy++) {
        machine_t *M = (machine_t *)malloc(sizeof(machine_t));
        int y = row0 + yy;
        for (int x = 0; x < width; x++) {
            uint32_t pixel = (uint32_t)y * (uint32_t)width + (uint32_t)x;
            v3 acc = V3(0, 0, 0);
            for (int s = 0; s < spp; s++) {
                uint32_t sid = (uint32_t)(sample0 + s);
                float jx = jitter ? jitter_u(seed, sid, pixel, 0u) : 0.0f;
                float jy = jitter ? jitter_u(seed, sid, pixel, 1u) : 0.0f;
                acc = add3(acc, recursive_raytrace(&S, M, camera_ray(inv, &cam, x, y, hw, hh, jx, jy), max_depth));
            }
            float *px = accum + ((size_t)yy * width + x) * 4;
            px[0] = px[0] + acc.x; px[1] = px[1] + acc.y; px[2] = px[2] + acc.z; px[3] = px[3] + 0.0f;
        }
        free(M);
    }
    free(o);
    return 0;
}

/* :325-405 */
int oracle_render(const rt_object *objs, int n_objs, const rt_material *mats, int n_mats,
                  const rt_light *lights, int n_lights, const rt_camera *cam_in, float time, int width,
                  int height, int max_depth, int row0, int row1, int probe, int n_threads, float *out) {
    if (!objs || n_objs < 0 || !mats || n_mats <= 0 || (n_lights > 0 && !lights) || n_lights < 0 || width <= 0 ||
        height <= 0 || row0 < 0 || row1 > height || row0 > row1 || max_depth < 0 || !out)
        return -1;
    obj_t *o = prepare_objects(objs, n_objs, mats, n_mats);
    if (!o) return -1;
    scene_t S = {o, n_objs, lights, n_lights};
    rt_camera cam;
    if (cam_in) cam = *cam_in;
    else oracle_reference_camera(time, &cam);
    m4 inv = frame_unprojection(cam_in ? &cam : NULL, time); /* :366-367, :383 */
    int hw = width / 2, hh = height / 2;  /* integer halves, :377-378 */
    int nrows = row1 - row0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : omp_get_max_threads())
    for (int yy = 0; yy < nrows; yy++) {
        machine_t *M = (machine_t *)malloc(sizeof(machine_t));
        int y = row0 + yy;
        for (int x = 0; x < width; x++) {
            ray_t r = camera_ray(inv, &cam, x, y, hw, hh, 0.0f, 0.0f);
            v3 col;
            if (probe == 0) {
                col = recursive_raytrace(&S, M, r, max_depth);
            } else if (probe == 1) {
                col = r.dir;
            } else {
                coll_t c = get_closest_collision(&S, r);
                if (probe == 2) {
                    float mask = 0.0f;
                    if (c.object_index != -1)
                        for (int j = 0; j < n_lights; j++)
                            if (in_shadow(&S, c, &lights[j])) mask += (float)(1 << j);
                    col = V3((float)c.object_index, c.t, mask);
                } else if (c.object_index == -1) {
                    col = V3(0, 0, 0);
                } else {
                    col = probe == 3 ? c.n : c.p;
                }
            }
            float *px = out + ((size_t)yy * width + x) * 4;
            px[0] = col.x; px[1] = col.y; px[2] = col.z; px[3] = 0.0f;
        }
        free(M);
    }
    free(o);
    return 0;
}
