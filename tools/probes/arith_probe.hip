// Exhaustive / randomised checks of short arithmetic forms against the
// correctly rounded IEEE operations on gfx950 (development probe, not product
// code). Prints mismatch counts; every kernel is a bounded grid-stride loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_refined(float b) {
    float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div_r2(float a, float b, float r) {  // current form: two corrections
    float q = a * r;
    float t = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(t, r, q);
    t = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(t, r, q);
}
__device__ __forceinline__ float div_r1(float a, float b, float r) {  // Markstein: one correction
    const float q = a * r;
    const float t = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(t, r, q);
}
__device__ __forceinline__ float sqrt_short(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u), up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
    return __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
}
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16; return h;
}
// counters: 0 raw sqrt, 1 sqrt_short, 2 raw rcp, 3 rcp_refined, 4 inv_sqrt short (rcp_refined of sqrt_short),
// 5 div one-correction, 6 div two-corrections, 7 samples
__global__ void exhaustive(uint32_t lo, uint32_t n, unsigned long long *cnt) {
    unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(lo + i);
        const float s = sqrtf(x), r = 1.0f / x;
        c0 += __builtin_amdgcn_sqrtf(x) != s;
        c1 += sqrt_short(x) != s;
        c2 += __builtin_amdgcn_rcpf(x) != r;
        c3 += rcp_refined(x) != r;
        c4 += rcp_refined(sqrt_short(x)) != 1.0f / s;
    }
    atomicAdd(cnt + 0, (unsigned long long)c0);
    atomicAdd(cnt + 1, (unsigned long long)c1);
    atomicAdd(cnt + 2, (unsigned long long)c2);
    atomicAdd(cnt + 3, (unsigned long long)c3);
    atomicAdd(cnt + 4, (unsigned long long)c4);
}
// direction of v_sqrt's error: counters 8 (correct = raw + 1 ulp), 9 (correct = raw - 1 ulp), 10 (other)
__global__ void sqrt_dir(uint32_t lo, uint32_t n, unsigned long long *cnt) {
    unsigned up = 0, dn = 0, other = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(lo + i);
        const uint32_t s = __float_as_uint(sqrtf(x)), r = __float_as_uint(__builtin_amdgcn_sqrtf(x));
        up += s == r + 1u;
        dn += s == r - 1u;
        other += s != r && s != r + 1u && s != r - 1u;
    }
    atomicAdd(cnt + 8, (unsigned long long)up);
    atomicAdd(cnt + 9, (unsigned long long)dn);
    atomicAdd(cnt + 10, (unsigned long long)other);
}
// random pairs a, b with exponents in [2^-emax, 2^emax]
__global__ void division(uint32_t seed, uint32_t per_thread, int emax, unsigned long long *cnt) {
    unsigned c5 = 0, c6 = 0;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t k = 0; k < per_thread; ++k) {
        const uint32_t h1 = mix32(seed ^ mix32(tid * 0x9E3779B1u + k)), h2 = mix32(h1 + 0x85EBCA77u), h3 = mix32(h2);
        const int ea = static_cast<int>(h3 % (2 * emax + 1)) - emax, eb = static_cast<int>((h3 >> 12) % (2 * emax + 1)) - emax;
        const float a = __uint_as_float(((127 + ea) << 23) | (h1 & 0x7fffffu) | (h3 & 0x80000000u));
        const float b = __uint_as_float(((127 + eb) << 23) | (h2 & 0x7fffffu) | ((h3 << 1) & 0x80000000u));
        const float want = a / b, r = rcp_refined(b);
        c5 += div_r1(a, b, r) != want;
        c6 += div_r2(a, b, r) != want;
    }
    atomicAdd(cnt + 5, (unsigned long long)c5);
    atomicAdd(cnt + 6, (unsigned long long)c6);
    atomicAdd(cnt + 7, (unsigned long long)per_thread);
}

// usage: arith_probe [quick]   (quick: one binade pair, fewer division pairs;
// tests/test_gpu_arith.py runs it)
int main(int argc, char **argv) {
    const bool quick = argc > 1 && argv[1][0] == 'q';
    unsigned long long *d = nullptr, h[12];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    struct R { const char *name; uint32_t lo, n; } ranges[] = {
        {"[1,4)", 0x3f800000u, 1u << 24},
        {"[2^-60,2^-58)", (67u << 23), 1u << 24},
        {"[2^40,2^42)", (167u << 23), 1u << 24},
        {"[2^-96,2^-94)", (31u << 23), 1u << 24},
    };
    for (const R &rg : ranges) {
        if (quick && rg.lo != 0x3f800000u) continue;
        hipMemset(d, 0, sizeof h);
        hipLaunchKernelGGL(exhaustive, dim3(4096), dim3(256), 0, 0, rg.lo, rg.n, d);
        if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        printf("%-14s n=%u  raw_sqrt=%llu sqrt_short=%llu raw_rcp=%llu rcp_refined=%llu invsqrt_short=%llu\n", rg.name,
               rg.n, h[0], h[1], h[2], h[3], h[4]);
        hipMemset(d, 0, sizeof h);
        hipLaunchKernelGGL(sqrt_dir, dim3(4096), dim3(256), 0, 0, rg.lo, rg.n, d);
        if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 4;
        printf("%-14s v_sqrt low by 1 ulp=%llu high by 1 ulp=%llu other=%llu\n", rg.name, h[8], h[9], h[10]);
    }
    for (int emax : {4, 30, 60}) {
        if (quick && emax != 30) continue;
        hipMemset(d, 0, sizeof h);
        hipLaunchKernelGGL(division, dim3(4096), dim3(256), 0, 0, 12345u + emax, quick ? 64u : 1024u, emax, d);
        if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
        printf("division emax=%d samples=%llu one_correction_bad=%llu two_corrections_bad=%llu\n", emax, h[7], h[5], h[6]);
    }
    hipFree(d);
    return 0;
}
