// Microbenchmark: issue rate of the bitwise VALU ops the FEC kernels use (not product code).
//
// v_bitop3_b32 (3-input XOR) on wave64, W waves per SIMD (W workgroups of 4 waves per CU,
// one wave per SIMD each), independent chains: the achieved wave-instructions per cycle per
// SIMD says how many waves a SIMD needs before the VALU, not the per-wave issue, is the
// limit.  Also: the same with one SALU instruction per VALU instruction interleaved (does a
// wave's scalar work take its own VALU issue slots?), and the wall time from HIP events,
// which gives the clock s_memtime counts at.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 16;   // independent chains per lane

// OP 0: bitop3 only; 1: bitop3 + one s_add per VALU op (dependent SALU chain); 2: bitop3 +
// one scalar branch per 4 VALU ops
template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(uint32_t* out, uint64_t* cycles,
                                                  uint32_t seed) {
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) a[i] = seed * (threadIdx.x + 1) + i;
    const uint32_t b = seed ^ threadIdx.x, c = seed + blockIdx.x;
    int s = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            a[i] = __builtin_amdgcn_bitop3_b32(a[i], b, c, 0x96);
            if (OP == 1) asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));
            if (OP == 2 && (i & 3) == 3) {
                asm volatile(
                    "s_cmp_eq_u32 %0, 12345\n\t"
                    "s_cbranch_scc1 1f\n\t"
                    "s_add_u32 %0, %0, 3\n\t"
                    "1:"
                    : "+s"(s));
            }
        }
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                     "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
                     "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = (uint32_t)s;
#pragma unroll
    for (int i = 0; i < CH; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* out;
    uint64_t* cyc;
    CK(hipMalloc(&out, (size_t)cus * 16 * 256 * 4));
    CK(hipMalloc(&cyc, (size_t)cus * 16 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"bitop3", "bitop3+salu", "bitop3+br/4"};
    for (int op = 0; op < 3; ++op) {
        for (int wps : {1, 2, 3, 4, 5, 6, 8}) {   // waves per SIMD = workgroups per CU
            const int nb = cus * wps;
            for (int rep = 0; rep < 2; ++rep) {   // first launch warms up
                CK(hipEventRecord(e0, 0));
                if (op == 0) valu_kernel<0><<<nb, 256>>>(out, cyc, 7);
                else if (op == 1) valu_kernel<1><<<nb, 256>>>(out, cyc, 7);
                else valu_kernel<2><<<nb, 256>>>(out, cyc, 7);
                CK(hipEventRecord(e1, 0));
                CK(hipDeviceSynchronize());
            }
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            uint64_t* h = (uint64_t*)malloc(nb * 8);
            CK(hipMemcpy(h, cyc, nb * 8, hipMemcpyDeviceToHost));
            double mean = 0;
            for (int i = 0; i < nb; ++i) mean += (double)h[i];
            mean /= nb;
            free(h);
            const double instr_per_simd = (double)ITERS * CH * wps;
            const double wall_instr_rate = (double)ITERS * CH * wps * cus * 4 / (ms * 1e-3);
            printf("%-12s waves/SIMD=%d  memtime/(wave-instr per SIMD) = %.3f  wall %.3f ms  "
                   "chip wave-instr/s = %.3e  memtime ticks/ns = %.3f\n",
                   names[op], wps, mean / instr_per_simd, ms, wall_instr_rate,
                   mean / (ms * 1e6));
        }
    }
    return 0;
}
