// VALU issue rate of the integer instructions the root-FC kernels use, on
// gfx950: 16 independent register chains per wave, 8 waves per SIMD, every
// CU busy.  Prints, per instruction, the shader cycles one SIMD spends per
// wave-instruction (= 64 lanes) -- the roofline's denominator for k_root_fc
// (v_cmp_lt_u32 + v_cndmask_b32 + v_add3_u32) and k_root_fc16
// (v_pk_sub_u16 clamp + v_pk_min_u16 + v_dot2_u32_u16).  v_fma_f32 and
// v_add_u32 as references.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kIters = 16384;

#define CH16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

#define KERNEL(NAME, BODY)                                                                     \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, unsigned seed, unsigned long long *clk) { \
        unsigned r0 = seed ^ threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,   \
                 r6 = r0 + 6, r7 = r0 + 7, r8 = r0 + 8, r9 = r0 + 9, r10 = r0 + 10, r11 = r0 + 11,           \
                 r12 = r0 + 12, r13 = r0 + 13, r14 = r0 + 14, r15 = r0 + 15;                                 \
        unsigned y = seed * 3u + 0x00010001u, z = 0x00010001u;                                               \
        asm volatile("" : "+v"(y), "+v"(z));                                                                 \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                          \
        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();                                      \
        for (int it = 0; it < kIters; it++) {                                                                \
            CH16(BODY)                                                                                       \
        }                                                                                                    \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                          \
        const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();                                      \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                                                           \
            clk[0] = t1 - t0;                                                                                \
            clk[1] = w1 - w0;                                                                                \
        }                                                                                                    \
        out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ r8 ^ r9 ^ r10 ^ r11 ^ \
                                              r12 ^ r13 ^ r14 ^ r15;                                         \
    }

#define B_ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r##i) : "v"(y));
#define B_PKSUB(i) asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(r##i) : "v"(y));
#define B_PKMIN(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(r##i) : "v"(y));
#define B_DOT2(i) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(r##i) : "v"(y), "v"(z));
#define B_ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r##i) : "v"(y), "v"(z));
#define B_CNDMASK(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r##i) : "v"(y));
#define B_FMA(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r##i) : "v"(y), "v"(z));

KERNEL(k_add, B_ADD)
KERNEL(k_pksub, B_PKSUB)
KERNEL(k_pkmin, B_PKMIN)
KERNEL(k_dot2, B_DOT2)
KERNEL(k_add3, B_ADD3)
KERNEL(k_cndmask, B_CNDMASK)
KERNEL(k_fma, B_FMA)

typedef void (*Kern)(unsigned *, unsigned, unsigned long long *);

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int waves_per_simd = 8, blocks = cus * waves_per_simd;   // 256 threads = 1 wave per SIMD per block
    unsigned *out;
    unsigned long long *clk, hclk[2];
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct {
        const char *name;
        Kern k;
    } ks[] = {{"v_add_u32", k_add},       {"v_pk_sub_u16_clamp", k_pksub}, {"v_pk_min_u16", k_pkmin},
              {"v_dot2_u32_u16", k_dot2}, {"v_add3_u32", k_add3},       {"v_cndmask_b32", k_cndmask},
              {"v_fma_f32", k_fma}};
    printf("{\"cus\": %d, \"waves_per_simd\": %d, \"results\": [", cus, waves_per_simd);
    for (int q = 0; q < (int)(sizeof ks / sizeof ks[0]); q++) {
        for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(ks[q].k, dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[q].k, dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
        const double mhz = (double)hclk[0] / (double)hclk[1] * 100.0;
        // wave-instructions per SIMD = waves_per_simd x iters x 16
        const double per_simd = (double)waves_per_simd * kIters * 16;
        const double cyc = ms * 1e-3 * mhz * 1e6 / per_simd;
        printf("%s{\"insn\": \"%s\", \"ms\": %.4f, \"mhz\": %.0f, \"cycles_per_wave_insn\": %.3f}", q ? ", " : "",
               ks[q].name, ms, mhz, cyc);
    }
    printf("]}\n");
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
