// Issue-rate probe (development, run on the MI355X): does scalar-ALU work
// share an issue budget with vector-ALU work on gfx950?
//
// The depth-0 render kernel issues about 420 SALU instructions per wave
// beside its 870 VALU (profiles/pmc_config2_latest.json: SQ_INSTS_SALU /
// SQ_INSTS_VALU = 0.49) and reaches 68 % of the VALU issue peak. A CU has one
// scalar unit for its four SIMDs; if it issues one SALU instruction per cycle,
// a CU's 32 waves can feed it 1 SALU per 2 VALU before it — not the SIMDs —
// sets the pace. This kernel times a loop body of N independent v_fma_f32 and
// M scalar adds (4 independent SGPR chains, or 64-bit ands) per wave at 8
// waves per SIMD, for several M, and prints cycles per loop iteration per
// SIMD against the VALU-only floor (2 cycles per wave64 VALU per SIMD).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/issue_probe tools/probes/issue_probe.hip
//   tools/probes/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

constexpr int kIters = 4096;
constexpr int kValu = 16;  // v_fma_f32 per iteration (4 independent accumulators)

template <int M, bool k64>
__global__ __launch_bounds__(256) void probe(float *out, int *sout, float b, float c) {
    float a0 = threadIdx.x, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
    unsigned s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    unsigned long long m0 = blockIdx.x, m1 = m0 + 7, m2 = m0 * 3, m3 = ~m0;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < kValu / 4; ++k) {
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a0) : "v"(b), "v"(c));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a1) : "v"(b), "v"(c));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a2) : "v"(b), "v"(c));
            asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a3) : "v"(b), "v"(c));
            if constexpr (M > 0) {
#pragma unroll
                for (int j = 0; j < M / (kValu / 4); ++j) {
                    if constexpr (k64) {
                        switch (j & 3) {
                            case 0: asm volatile("s_and_b64 %0, %0, %1" : "+s"(m0) : "s"(m1) : "scc"); break;
                            case 1: asm volatile("s_or_b64 %0, %0, %1" : "+s"(m1) : "s"(m2) : "scc"); break;
                            case 2: asm volatile("s_xor_b64 %0, %0, %1" : "+s"(m2) : "s"(m3) : "scc"); break;
                            default: asm volatile("s_andn2_b64 %0, %0, %1" : "+s"(m3) : "s"(m0) : "scc"); break;
                        }
                    } else {
                        switch (j & 3) {
                            case 0: asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1) : "scc"); break;
                            case 1: asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(s2) : "scc"); break;
                            case 2: asm volatile("s_add_u32 %0, %0, %1" : "+s"(s2) : "s"(s3) : "scc"); break;
                            default: asm volatile("s_add_u32 %0, %0, %1" : "+s"(s3) : "s"(s0) : "scc"); break;
                        }
                    }
                }
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0)  // (a vector store of the scalar results)
        sout[blockIdx.x] = static_cast<int>(s0 ^ s1 ^ s2 ^ s3 ^ static_cast<unsigned>(m0 ^ m1 ^ m2 ^ m3));
}

template <int M, bool k64>
int run(int n_cu, float *out, int *sout, double clock_ghz) {
    const int groups = n_cu * 8;  // 8 x 256 threads = 32 waves per CU = 8 per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<M, k64>), dim3(groups), dim3(256), 0, 0, out, sout, 1.0f, 0.0f);
    CHECK(hipGetLastError());
    std::vector<float> ms;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((probe<M, k64>), dim3(groups), dim3(256), 0, 0, out, sout, 1.0f, 0.0f);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float t = 0;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    float best = ms[0];
    for (float t : ms) best = t < best ? t : best;
    // per SIMD: 8 waves x kIters iterations
    const double cyc_per_iter_simd = best * 1e-3 * clock_ghz * 1e9 / kIters;
    const double valu_floor = 8.0 * kValu * 2.0;  // 8 waves x kValu VALU x 2 cycles
    std::printf("{\"salu_per_iter\": %d, \"salu_kind\": \"%s\", \"valu_per_iter\": %d, \"ms\": %.4f, "
                "\"cycles_per_iter_per_simd\": %.1f, \"valu_floor_cycles\": %.1f, \"ratio\": %.3f, "
                "\"salu_per_cu_cycle\": %.3f}\n",
                M, k64 ? "s_*_b64" : "s_add_u32", kValu, best, cyc_per_iter_simd, valu_floor,
                cyc_per_iter_simd / valu_floor, 32.0 * M / (cyc_per_iter_simd));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

int main(int argc, char **argv) {
    double clock_ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
    int n_cu = 0;
    CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
    float *out = nullptr;
    int *sout = nullptr;
    CHECK(hipMalloc(&out, sizeof(float) * n_cu * 8 * 256));
    CHECK(hipMalloc(&sout, sizeof(int) * n_cu * 8));
    std::printf("# %d CUs, clock assumed %.2f GHz (pass the measured one as argv[1])\n", n_cu, clock_ghz);
    int rc = 0;
    rc |= run<0, false>(n_cu, out, sout, clock_ghz);
    rc |= run<4, false>(n_cu, out, sout, clock_ghz);
    rc |= run<8, false>(n_cu, out, sout, clock_ghz);
    rc |= run<12, false>(n_cu, out, sout, clock_ghz);
    rc |= run<16, false>(n_cu, out, sout, clock_ghz);
    rc |= run<24, false>(n_cu, out, sout, clock_ghz);
    rc |= run<32, false>(n_cu, out, sout, clock_ghz);
    rc |= run<8, true>(n_cu, out, sout, clock_ghz);
    rc |= run<16, true>(n_cu, out, sout, clock_ghz);
    rc |= run<32, true>(n_cu, out, sout, clock_ghz);
    (void)hipFree(out);
    (void)hipFree(sout);
    return rc;
}
