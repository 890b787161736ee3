// Microbenchmark (not product code): VALU issue rate, and the cost of one run-time GF(256)
// coefficient applied to a bit-sliced block, against the waves per SIMD.
//
// Every point runs >= 10 ms of back-to-back launches (so the clock has settled and launch
// overhead is noise) and reports, per SIMD:
//   cyc/VALU   shader cycles (s_memtime) per wave-instruction issued on one SIMD
//   cyc/apply  shader cycles per (coefficient, block) application on one SIMD
//   clock      in-kernel clock: delta s_memtime / delta s_memrealtime x 100 MHz
//              (MI355X_MICROARCH.md, DVFS give-back item 6)
// Nothing the timed loop computes can be dropped: every iteration folds a value that depends
// on the loop counter (a scalar register read by a VALU op) into the accumulators, and the
// accumulators are written to memory at the end.
//
// Modes:
//   xor3      16 independent v_bitop3 chains (the VALU rate itself)
//   xor3+salu the same with one dependent s_add per v_bitop3, its result fed back through a
//             VGPR every iteration (does scalar work take VALU issue slots?)
//   xor3+br   the same with one uniform s_cbranch per 4 v_bitop3
//   nibble    run-time coefficient, W/Z expansion + scalar nibble dispatch (gf_bitslice.h
//             apply_nibble, the current preset decode): 2 dispatches of 8 VALU per apply
//   mask      run-time coefficient, no branches: acc[r] ^= W[b + r] & mask_b for the 8 bits b
//             (v_bitop3 0x78 with the mask in an SGPR): 64 VALU per apply
//   window    compile-time coefficient chosen by a 16-way uniform switch, windowed form
//             (win_apply, 8 VALU per apply on a window built once per block)
//   gpridx    run-time coefficient in the windowed form: acc[r] ^= lo[a_r] ^ hi[b_r] with the
//             per-row nibbles (a_r, b_r) of c * alpha^r from a table and the window read by
//             uniform register indexing (s_set_gpr_idx_on + v_mov): no branches
//   jump      run-time coefficient in the windowed form through one indirect jump into a
//             table of 256 leaves (gf_winjump.h win_mul_rt), product into a temporary then
//             XORed into the output: 16 VALU + 6 scalar instructions per apply
//   nibjump   the W/Z nibble form with each nibble's dispatch an indirect jump into a table
//             of 16 leaves (gf_winjump.h wz_mul_acc_rt), compile-time target: 16 VALU + 12
//             scalar instructions per apply
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../quic_amd/csrc -I../../build/gen
//         valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "gf_bitslice.h"
#include "gf_winjump.h"

using namespace qfec;

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

constexpr int CH = 16;   // independent chains per lane (rate modes)
constexpr int NOUT = 4;  // outputs per block (apply modes): 4 coefficients per block

struct Stamp {
    uint64_t cyc, real;
};

__device__ __forceinline__ void stamp_out(Stamp* st, uint64_t c0, uint64_t r0) {
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x % 64 == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        st[w].cyc = c1 - c0;
        st[w].real = r1 - r0;
    }
}

// OP 0 xor3, 1 xor3+salu, 2 xor3+br
template <int OP, int WPS>
__global__ __launch_bounds__(256, WPS) void rate_kernel(uint32_t* out, Stamp* st, uint32_t seed,
                                                        int iters) {
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) a[i] = seed * (threadIdx.x + 1) + i;
    uint32_t b = seed ^ threadIdx.x;
    const uint32_t c = seed + blockIdx.x;
    int s = __builtin_amdgcn_readfirstlane((int)seed);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            a[i] = __builtin_amdgcn_bitop3_b32(a[i], b, c, 0x96);
            if (OP == 1) asm volatile("s_add_u32 %0, %0, %1" : "+s"(s) : "s"(it));
            if (OP == 2 && (i & 3) == 3) {
                asm volatile(
                    "s_cmp_eq_u32 %0, 12345\n\t"
                    "s_cbranch_scc1 1f\n\t"
                    "s_add_u32 %0, %0, 3\n\t"
                    "1:"
                    : "+s"(s));
            }
        }
        // the scalar chain feeds a VGPR every iteration: nothing can be dropped
        b ^= (uint32_t)s + (uint32_t)it;
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                     "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]),
                     "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]), "+v"(b));
    }
    stamp_out(st, c0, r0);
    uint32_t x = (uint32_t)s ^ b;
#pragma unroll
    for (int i = 0; i < CH; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// The coefficient tables live in a buffer read through s_load (wave-uniform): NOUT bytes per
// iteration, random.
__device__ __forceinline__ uint32_t coef_word(const uint32_t* __restrict__ tab, int it) {
    return tab[it & 4095];
}

// OP 0 nibble, 1 mask, 2 window(switch), 3 gpridx, 4 jump, 5 nibjump
template <int OP, int WPS>
__global__ __launch_bounds__(256, WPS) void apply_kernel(const uint32_t* __restrict__ tab,
                                                         uint32_t* out, Stamp* st, uint32_t seed,
                                                         int iters) {
    uint32_t in[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) in[t] = seed * (threadIdx.x + 3 * t + 1);
    uint32_t acc[NOUT][8];
#pragma unroll
    for (int j = 0; j < NOUT; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[j][r] = 0;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        const uint32_t cw = coef_word(tab, it);
        // a fresh block every iteration (8 VALU, as the realignment of a streamed block)
#pragma unroll
        for (int t = 0; t < 8; ++t) in[t] ^= (uint32_t)it + t;
        if constexpr (OP == 0) {
            WZ v;
#pragma unroll
            for (int t = 0; t < 8; ++t) v.W[t] = in[t];
            expand_wz(v);
#pragma unroll
            for (int j = 0; j < NOUT; ++j) {
                const uint32_t cf = (cw >> (8 * j)) & 0xFFu;
                apply_nibble<0>(acc[j], cf & 15u, v);
                apply_nibble<4>(acc[j], cf >> 4, v);
            }
        } else if constexpr (OP == 1) {
            uint32_t W[15];
#pragma unroll
            for (int t = 0; t < 8; ++t) W[t] = in[t];
#pragma unroll
            for (int n = 8; n < 15; ++n) W[n] = xor3(W[n - 1], W[n - 6], W[n - 7] ^ W[n - 8]);
#pragma unroll
            for (int j = 0; j < NOUT; ++j) {
                const uint32_t cf = (cw >> (8 * j)) & 0xFFu;
#pragma unroll
                for (int bt = 0; bt < 8; ++bt) {
                    const uint32_t mk = (uint32_t)__builtin_amdgcn_readfirstlane(
                        (int)(0u - ((cf >> bt) & 1u)));
#pragma unroll
                    for (int r = 0; r < 8; ++r)
                        acc[j][r] = __builtin_amdgcn_bitop3_b32(acc[j][r], W[bt + r], mk, 0x78);
                }
            }
        } else if constexpr (OP == 3) {
            // two plain local arrays (a struct would be left in scratch memory; plain arrays
            // are promoted to registers and indexed with s_set_gpr_idx)
            uint32_t lo[16], hi[16];
            win_group(in, lo);
            win_group(in + 4, hi);
#pragma unroll
            for (int j = 0; j < NOUT; ++j) {
                // 8 bytes per coefficient: (a_r | b_r << 4) for r = 0..7
                const uint32_t n0 = tab[(it * 8 + 2 * j) & 4095], n1 = tab[(it * 8 + 2 * j + 1) & 4095];
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint32_t nb = ((r < 4 ? n0 : n1) >> (8 * (r & 3))) & 0xFFu;
                    acc[j][r] = xor3(acc[j][r], lo[nb & 15u], hi[nb >> 4]);
                }
            }
        } else if constexpr (OP == 4) {
            Win w;
            win_build(in, w);
#pragma unroll 1
            for (int j = 0; j < NOUT; ++j) {
                const uint32_t cf = (uint32_t)__builtin_amdgcn_readfirstlane((int)((cw >> (8 * j)) & 0xFFu));
                uint32_t t[8];
                win_mul_rt(t, w, cf);
                // j is run-time (one call site): scatter through a 4-way uniform switch
                switch (j) {
#define QM_J(J) \
    case J: _Pragma("unroll") for (int r = 0; r < 8; ++r) acc[J][r] ^= t[r]; break;
                    QM_J(0) QM_J(1) QM_J(2) default: QM_J(3)
#undef QM_J
                }
            }
        } else if constexpr (OP == 5) {
            WZ v;
#pragma unroll
            for (int t = 0; t < 8; ++t) v.W[t] = in[t];
            expand_wz(v);
            static_for<NOUT>([&](auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value;
                const uint32_t cf = (uint32_t)__builtin_amdgcn_readfirstlane((int)((cw >> (8 * j)) & 0xFFu));
                wz_mul_acc_rt(acc[j], v, cf);
            });
        } else {
            Win w;
            win_build(in, w);
#pragma unroll
            for (int j = 0; j < NOUT; ++j) {
                const uint32_t sel = (cw >> (8 * j)) & 15u;
                switch (sel) {
#define QM_C(N, C) \
    case N: win_apply<C>(acc[j], w); break;
                    QM_C(0, 0x8e) QM_C(1, 0x13) QM_C(2, 0xd4) QM_C(3, 0x61) QM_C(4, 0x2b)
                    QM_C(5, 0xf7) QM_C(6, 0x3c) QM_C(7, 0x95) QM_C(8, 0x48) QM_C(9, 0xba)
                    QM_C(10, 0x06) QM_C(11, 0xe3) QM_C(12, 0x7f) QM_C(13, 0x51) QM_C(14, 0xc9)
                    default: win_apply<0x24>(acc[j], w); break;
#undef QM_C
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NOUT; ++j)
#pragma unroll
            for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[j][r]));
    }
    stamp_out(st, c0, r0);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < NOUT; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) x ^= acc[j][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

struct Res {
    double cyc_per_wave, ms, clock_ghz;
};

template <class K>
Res run(K kernel, int wps, int cus, const uint32_t* tab, uint32_t* out, Stamp* st, int iters,
        bool apply) {
    const int nb = cus * wps;   // 256-thread workgroups: one wave per SIMD each
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&]() {
        if (apply)
            hipLaunchKernelGGL((void (*)(const uint32_t*, uint32_t*, Stamp*, uint32_t, int))kernel,
                               dim3(nb), dim3(256), 0, 0, tab, out, st, 7u, iters);
        else
            hipLaunchKernelGGL((void (*)(uint32_t*, Stamp*, uint32_t, int))kernel, dim3(nb),
                               dim3(256), 0, 0, out, st, 7u, iters);
        CK(hipGetLastError());
    };
    // warm up >= 2 s of back-to-back launches on the first point only (clock settles)
    static bool warmed = false;
    if (!warmed) {
        for (int i = 0; i < 40; ++i) launch();
        CK(hipDeviceSynchronize());
        warmed = true;
    }
    // one timed launch sizes the repeat count: >= 10 ms per point
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms1 = 0;
    CK(hipEventElapsedTime(&ms1, e0, e1));
    const int reps = ms1 >= 10.f ? 1 : (int)(10.f / (ms1 > 0.01f ? ms1 : 0.01f)) + 1;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const int nw = nb * 4;
    Stamp* h = (Stamp*)malloc(nw * sizeof(Stamp));
    CK(hipMemcpy(h, st, nw * sizeof(Stamp), hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < nw; ++i) {
        cyc += (double)h[i].cyc;
        real += (double)h[i].real;
    }
    free(h);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return {cyc / nw, ms / reps, (cyc / real) * 0.1};   // memrealtime: 100 MHz
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *out, *tab;
    Stamp* st;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    CK(hipMalloc(&st, (size_t)cus * 8 * 4 * sizeof(Stamp)));
    CK(hipMalloc(&tab, 4096 * 4));
    {
        uint32_t h[4096];
        uint64_t x = 0x9e3779b97f4a7c15ull;
        for (int i = 0; i < 4096; ++i) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            h[i] = (uint32_t)x;
        }
        CK(hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice));
    }
    printf("CUs %d; per point: mean over waves of s_memtime cycles; clock = memtime/memrealtime\n",
           cus);
    // VALU per iteration per wave: rate modes 16 (+ the b update), measured directly
    const int RITERS = 40000;
#define RATE(OP, W, NAME)                                                                      \
    {                                                                                          \
        Res r = run(rate_kernel<OP, W>, W, cus, tab, out, st, RITERS, false);                 \
        const double per_simd = r.cyc_per_wave / ((double)RITERS * CH * W);                   \
        printf("%-10s waves/SIMD=%d  cyc/VALU(SIMD) %.3f  kernel %.2f ms  clock %.3f GHz\n", \
               NAME, W, per_simd, r.ms, r.clock_ghz);                                          \
    }
#define RATES(OP, NAME) RATE(OP, 1, NAME) RATE(OP, 2, NAME) RATE(OP, 4, NAME) RATE(OP, 8, NAME)
    RATES(0, "xor3")
    RATES(1, "xor3+salu")
    RATES(2, "xor3+br")
    const int AITERS = 8000;
#define APPLY(OP, W, NAME)                                                                     \
    {                                                                                          \
        Res r = run(apply_kernel<OP, W>, W, cus, tab, out, st, AITERS, true);                 \
        const double per_simd = r.cyc_per_wave / ((double)AITERS * NOUT * W);                 \
        printf("%-10s waves/SIMD=%d  cyc/apply(SIMD) %.2f  kernel %.2f ms  clock %.3f GHz\n", \
               NAME, W, per_simd, r.ms, r.clock_ghz);                                          \
    }
#define APPLIES(OP, NAME) APPLY(OP, 1, NAME) APPLY(OP, 2, NAME) APPLY(OP, 4, NAME) APPLY(OP, 5, NAME)
    APPLIES(0, "nibble")
    APPLIES(1, "mask")
    APPLIES(2, "window")
    APPLIES(3, "gpridx")
    APPLIES(4, "jump")
    APPLIES(5, "nibjump")
    return 0;
}
