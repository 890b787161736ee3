// Microbenchmark: issue rate of the bitwise VALU ops the FEC kernels use (not product code).
//
// v_bitop3_b32 (3-input XOR) and v_xor_b32 on wave64, W waves per SIMD, independent chains:
// the achieved wave-instructions per cycle per SIMD says whether these ops issue every 2
// cycles (32-lane SIMD, two waves interleaved) or every 4.  Clock from s_memtime inside
// the kernel (shader cycles), so DVFS does not enter.
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

template <int OP>
__global__ void valu_kernel(uint32_t* out, uint64_t* cycles, uint32_t seed) {
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) a[i] = seed * (threadIdx.x + 1) + i;
    const uint32_t b = seed ^ threadIdx.x, c = seed + blockIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if (OP == 0) a[i] = __builtin_amdgcn_bitop3_b32(a[i], b, c, 0x96);
            else a[i] ^= b;
        }
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                     "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
                     "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
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
    CK(hipMalloc(&out, (size_t)cus * 1024 * 4 * 8));
    CK(hipMalloc(&cyc, (size_t)cus * 8 * 8));
    for (int op = 0; op < 2; ++op) {
        for (int wps : {1, 2, 3, 4, 8}) {   // waves per SIMD: one workgroup of 4*wps waves per CU
            const int threads = 64 * 4 * wps;
            if (threads > 1024) continue;
            if (op == 0) valu_kernel<0><<<cus, threads>>>(out, cyc, 7);
            else valu_kernel<1><<<cus, threads>>>(out, cyc, 7);
            CK(hipDeviceSynchronize());
            uint64_t* h = (uint64_t*)malloc(cus * 8);
            CK(hipMemcpy(h, cyc, cus * 8, hipMemcpyDeviceToHost));
            double mean = 0;
            for (int i = 0; i < cus; ++i) mean += (double)h[i];
            mean /= cus;
            free(h);
            const double instr_per_simd = (double)ITERS * CH * wps;
            printf("%-12s waves/SIMD=%d  cycles/(wave-instr per SIMD) = %.2f\n",
                   op == 0 ? "v_bitop3" : "v_xor", wps, mean / instr_per_simd);
        }
    }
    return 0;
}
