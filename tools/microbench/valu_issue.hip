// Microbenchmark (not product code): VALU issue cost per instruction FORM on gfx950, against
// the waves per SIMD.  Each mode issues 16 independent instructions per iteration (inline
// asm, so the compiler cannot change the form), 20,000 iterations, and reports shader cycles
// (s_memtime) per instruction per SIMD: one wave's cycles / (its instructions x waves per
// SIMD).
//   bitop3   v_bitop3_b32 (VOP3, 8 bytes): acc ^= a ^ b, the D kernels' XOR3
//   xor      v_xor_b32_e32 (VOP2, 4 bytes): acc ^= a
//   fma      v_fma_f32 (VOP3): the guide's reference instruction
//   bitop3s  v_bitop3_b32 with one SGPR operand
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 valu_issue.hip -o valu_issue
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

struct Stamp {
    uint64_t cyc, real;
};

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

template <int OP, int WPS>
__global__ __launch_bounds__(256, WPS) void issue_kernel(uint32_t* out, Stamp* st, uint32_t seed,
                                                         int iters) {
    uint32_t a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = seed * (threadIdx.x + 1) + i;
    uint32_t b = seed ^ threadIdx.x, c = seed + threadIdx.x * 3;
    const uint32_t s = __builtin_amdgcn_readfirstlane(seed * 5 + blockIdx.x);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#define QB(i)                                                                                  \
    if constexpr (OP == 0)                                                                     \
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c)); \
    else if constexpr (OP == 1)                                                                \
        asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[i]) : "v"(b));                            \
    else if constexpr (OP == 2)                                                                \
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                \
    else                                                                                       \
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "s"(s));
        R16(QB)
#undef QB
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x % 64 == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        st[w].cyc = c1 - c0;
        st[w].real = r1 - r0;
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <class K>
void run(K kernel, const char* name, int wps, int cus, uint32_t* out, Stamp* st, int iters) {
    const int nb = cus * wps;
    auto launch = [&]() {
        hipLaunchKernelGGL(kernel, dim3(nb), dim3(256), 0, 0, out, st, 7u, iters);
        CK(hipGetLastError());
    };
    static bool warmed = false;
    if (!warmed) {
        for (int i = 0; i < 40; ++i) launch();
        CK(hipDeviceSynchronize());
        warmed = true;
    }
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    const int nw = nb * 4;
    Stamp* h = (Stamp*)malloc(nw * sizeof(Stamp));
    CK(hipMemcpy(h, st, nw * sizeof(Stamp), hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < nw; ++i) cyc += (double)h[i].cyc, real += (double)h[i].real;
    free(h);
    cyc /= nw;
    real /= nw;
    printf("%-8s waves/SIMD=%d  cyc/instr(SIMD) %.3f  cyc/instr(wave) %.2f  clock %.3f GHz\n", name,
           wps, cyc / ((double)iters * 16 * wps), cyc / ((double)iters * 16), cyc / real * 0.1);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* out;
    Stamp* st;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    CK(hipMalloc(&st, (size_t)cus * 8 * 4 * sizeof(Stamp)));
    const int IT = 20000;
#define PTS(OP, NAME)                                            \
    run(issue_kernel<OP, 1>, NAME, 1, cus, out, st, IT);         \
    run(issue_kernel<OP, 2>, NAME, 2, cus, out, st, IT);         \
    run(issue_kernel<OP, 3>, NAME, 3, cus, out, st, IT);         \
    run(issue_kernel<OP, 4>, NAME, 4, cus, out, st, IT);         \
    run(issue_kernel<OP, 8>, NAME, 8, cus, out, st, IT);
    PTS(0, "bitop3")
    PTS(1, "xor")
    PTS(2, "fma")
    PTS(3, "bitop3s")
    return 0;
}
