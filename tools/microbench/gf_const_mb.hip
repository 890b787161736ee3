// Microbenchmark: bit-sliced GF apply with compile-time coefficients (every nibble
// dispatch folds away) vs the runtime-coefficient branchy dispatch, on the B (32, 4, 1352)
// and D (128, 16, 9008) encode layouts.  Timing only (random coefficients).  Not product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -structurizecfg-skip-uniform-regions=true \
//         gf_const_mb.hip -o gf_const_mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include "../../quic_amd/csrc/gf_bitslice.h"

using namespace qfec;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef uint32_t u32ua __attribute__((aligned(1)));

struct CoefTab {
    uint8_t c[16][128];
};
constexpr CoefTab make_tab() {
    CoefTab t{};
    uint32_t s = 12345;
    for (int j = 0; j < 16; ++j)
        for (int x = 0; x < 128; ++x) {
            s = s * 1103515245u + 12345u;
            t.c[j][x] = (uint8_t)(s >> 16) | 1;
        }
    return t;
}
constexpr CoefTab kTab = make_tab();

__global__ void fill(uint8_t* p, size_t n, uint64_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (size_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
}

// One wave = (group, chunk of RC outputs starting at J0, 64-word tile).  CONST: coefficients
// from kTab at compile time (full unroll over x); else read at run time from `coef`.
template <int K, int RC, int J0, int PD, bool CONST, bool P0>
__global__ __launch_bounds__(256) void gfc_kernel(const uint8_t* __restrict__ in, uint8_t* out,
                                                  const uint8_t* __restrict__ coef, int bb,
                                                  int ntiles, int m, long long units) {
    const int lane = threadIdx.x & 63;
    const long long unit = (long long)blockIdx.x * 4 + wave_id();
    if (unit >= units) return;
    const int tile = (int)(unit % ntiles);
    const long long g = unit / ntiles;
    const int s = bb >> 3;
    const int nw = (s + 3) >> 2;
    const int c = tile * 64 + lane;
    const int cc = c < nw ? c : nw - 1;
    const int off = 4 * cc;
    const int lo = min(off, s - 4);
    const int shift = 8 * (off - lo);
    const uint8_t* gin = in + g * K * bb + lo;
    uint32_t acc[RC][8];
#pragma unroll
    for (int j = 0; j < RC; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[j][r] = 0;
    uint32_t raw[PD][8];
#pragma unroll
    for (int u = 0; u < PD; ++u)
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[u][t] = *(const u32ua*)(gin + (long long)u * bb + t * s);
#pragma unroll
    for (int x = 0; x < K; ++x) {
        WZ v;
#pragma unroll
        for (int t = 0; t < 8; ++t) v.W[t] = raw[x % PD][t] >> shift;
        if (x + PD < K) {
#pragma unroll
            for (int t = 0; t < 8; ++t) raw[x % PD][t] = *(const u32ua*)(gin + (long long)(x + PD) * bb + t * s);
        }
        expand_wz(v);
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            if (P0 && j == 0) {
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                continue;
            }
            uint32_t cf;
            if (CONST) cf = kTab.c[J0 + j][x];
            else cf = coef[(J0 + j) * 128 + x];
            apply_nibble<0>(acc[j], cf & 15u, v);
            apply_nibble<4>(acc[j], cf >> 4, v);
        }
    }
    const int nwf = s >> 2;
#pragma unroll
    for (int j = 0; j < RC; ++j) {
        uint8_t* dst = out + (g * m + J0 + j) * (long long)bb;
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (c < nwf) *(u32ua*)(dst + r * s + 4 * c) = acc[j][r];
    }
}

template <int K, int RC, int J0, int PD, bool CONST, bool P0>
void run(const char* name, const uint8_t* in, uint8_t* out, const uint8_t* coef, int bb, int m,
         long long G, int reps, int nchunks) {
    const int s = bb / 8, nw = (s + 3) / 4, ntiles = (nw + 63) / 64;
    const long long units = G * ntiles;
    auto kern = gfc_kernel<K, RC, J0, PD, CONST, P0>;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned nb = (unsigned)((units + 3) / 4);
    hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, in, out, coef, bb, ntiles, m, units);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, in, out, coef, bb, ntiles, m, units);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    // bytes of a whole encode (all chunks) if each chunk costs the same
    const double bytes = (double)G * (K + m) * bb;
    printf("%-4s K=%3d RC=%2d J0=%d PD=%d CONST=%d P0=%d : %8.3f ms per chunk -> x%d = %8.3f ms  %6.0f GB/s\n",
           name, K, RC, J0, PD, (int)CONST, (int)P0, ms, nchunks, ms * nchunks, bytes / (ms * nchunks) / 1e6);
}

int main() {
    const int reps = 10;
    const long long GB_ = 65536, GD = 8192;
    const size_t inB = (size_t)GB_ * 32 * 1352, inD = (size_t)GD * 128 * 9008;
    const size_t inmax = std::max(inB, inD);
    uint8_t *in, *out, *coef;
    CK(hipMalloc(&in, inmax + 4096)); CK(hipMalloc(&out, inmax / 4)); CK(hipMalloc(&coef, 4096));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, inmax, 1ull);
    CK(hipMemcpy(coef, &kTab, sizeof(kTab), hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    run<32, 4, 0, 2, false, false>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<32, 4, 0, 2, false, true>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<32, 4, 0, 2, true, true>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<32, 4, 0, 3, true, true>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<32, 4, 0, 4, true, true>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<32, 2, 0, 2, true, true>("B", in, out, coef, 1352, 4, GB_, reps, 1);
    run<128, 8, 0, 2, false, true>("D", in, out, coef, 9008, 16, GD, reps, 2);
    run<128, 8, 0, 2, true, true>("D", in, out, coef, 9008, 16, GD, reps, 2);
    run<128, 8, 8, 2, true, false>("D", in, out, coef, 9008, 16, GD, reps, 2);
    run<128, 16, 0, 2, true, true>("D", in, out, coef, 9008, 16, GD, reps, 1);
    run<128, 4, 4, 2, true, false>("D", in, out, coef, 9008, 16, GD, reps, 4);
    return 0;
}
