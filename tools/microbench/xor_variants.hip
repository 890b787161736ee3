// Microbenchmark: HBM ceilings and m = 1 XOR-encode kernel variants on gfx950.
// Not part of the product; used to choose the shipped kernel shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 xor_variants.hip -o xor_variants
//   ./xor_variants [groups=65536] [k=10] [bb=1352] [reps=30]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
typedef uint32_t u32ua __attribute__((aligned(1)));

// ---- ceilings
__global__ void read_only(const u32x4* __restrict__ a, size_t n, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= a[i];
    if ((acc.x & 0xfffffff) == 0x1234567) sink[0] = acc;
}
__global__ void read_only_nt(const u32x4* __restrict__ a, size_t n, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(&a[i]);
    if ((acc.x & 0xfffffff) == 0x1234567) sink[0] = acc;
}
__global__ void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}
// read 10 lines, write 1: the XOR pattern on an aligned layout (bb = 1408 = 88*16)
__global__ void xor_aligned(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, int nu, unsigned total) {
    unsigned u = blockIdx.x * 256u + threadIdx.x;
    if (u >= total) return;
    unsigned g = u / nu, q = u - g * nu;
    const uint8_t* s = d + (size_t)g * k * bb + q * 16;
    u32x4 acc = *(const u32x4*)s;
#pragma unroll
    for (int x = 1; x < 10; ++x) acc ^= *(const u32x4*)(s + (size_t)x * bb);
    *(u32x4*)(p + (size_t)g * bb + q * 16) = acc;
}

// ---- variants on the real layout (bb = 1352)
// V1: flat 16B units (8-aligned), shifted tail
template <bool NT>
__global__ __launch_bounds__(256) void v_flat16(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, int nu, unsigned total) {
    unsigned u = blockIdx.x * 256u + threadIdx.x;
    if (u >= total) return;
    unsigned g = u / nu; int q = u - g * nu;
    int off = min(q * 16, bb - 16);
    const uint8_t* s = d + (size_t)g * k * bb + off;
    u32x4 acc;
    if (NT) acc = __builtin_nontemporal_load((const u32x4a8*)s); else acc = *(const u32x4a8*)s;
#pragma unroll
    for (int x = 1; x < 10; ++x) {
        if (NT) acc ^= __builtin_nontemporal_load((const u32x4a8*)(s + (size_t)x * bb));
        else acc ^= *(const u32x4a8*)(s + (size_t)x * bb);
    }
    uint8_t* o = p + (size_t)g * bb;
    if (q * 16 + 16 <= bb) *(u32x4a8*)(o + off) = acc;
    else *(uint64_t*)(o + q * 16) = ((uint64_t)acc.w << 32) | acc.z;
}
// V2: flat 8B units
__global__ __launch_bounds__(256) void v_flat8(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, int nu, unsigned total) {
    unsigned u = blockIdx.x * 256u + threadIdx.x;
    if (u >= total) return;
    unsigned g = u / nu; int q = u - g * nu;
    const uint8_t* s = d + (size_t)g * k * bb + q * 8;
    uint64_t acc = *(const uint64_t*)s;
#pragma unroll
    for (int x = 1; x < 10; ++x) acc ^= *(const uint64_t*)(s + (size_t)x * bb);
    *(uint64_t*)(p + (size_t)g * bb + q * 8) = acc;
}
// V3: one wave per group, 16B, loop over chunks (the v0 shipped kernel)
__global__ __launch_bounds__(256) void v_wave16(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, long long groups) {
    const int lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const int nq = bb / 16;
    const uint8_t* s = d + g * (long long)k * bb;
    uint8_t* o = p + g * (long long)bb;
    for (int q = lane; q < nq; q += 64) {
        u32x4 acc = *(const u32x4a8*)(s + q * 16);
#pragma unroll
        for (int x = 1; x < 10; ++x) acc ^= *(const u32x4a8*)(s + q * 16 + (size_t)x * bb);
        *(u32x4a8*)(o + q * 16) = acc;
    }
    for (int i = nq * 16 + lane; i < bb; i += 64) {
        uint8_t a = s[i];
        for (int x = 1; x < 10; ++x) a ^= s[(size_t)x * bb + i];
        o[i] = a;
    }
}
// V4: flat, 2 units per thread (32B in flight per block per lane)
__global__ __launch_bounds__(256) void v_flat16x2(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, int nu, unsigned total) {
    unsigned t = blockIdx.x * 256u + threadIdx.x;
    unsigned u0 = (t / 64) * 128 + (t % 64);
    u32x4 acc[2];
    int off[2]; unsigned gg[2]; bool ok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        unsigned u = u0 + 64 * j;
        ok[j] = u < total;
        if (!ok[j]) u = total - 1;
        gg[j] = u / nu; int q = u - gg[j] * nu;
        off[j] = min(q * 16, bb - 16);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = *(const u32x4a8*)(d + (size_t)gg[j] * k * bb + off[j]);
#pragma unroll
    for (int x = 1; x < 10; ++x)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] ^= *(const u32x4a8*)(d + (size_t)gg[j] * k * bb + off[j] + (size_t)x * bb);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!ok[j]) continue;
        unsigned u = u0 + 64 * j; int q = u - gg[j] * nu;
        uint8_t* o = p + (size_t)gg[j] * bb;
        if (q * 16 + 16 <= bb) *(u32x4a8*)(o + off[j]) = acc[j];
        else *(uint64_t*)(o + q * 16) = ((uint64_t)acc[j].w << 32) | acc[j].z;
    }
}
// V5: group-per-wave, but the wave covers the whole block with 2 loads per lane
//     (16B at lane*16 and 16B at 1024 + lane*16, clamped), all 20 loads issued together
__global__ __launch_bounds__(256) void v_wave2(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int k, int bb, long long groups) {
    const int lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= groups) return;
    const uint8_t* s = d + g * (long long)k * bb;
    uint8_t* o = p + g * (long long)bb;
    const int nu = (bb + 15) / 16;   // 85
    int q1 = 64 + lane; bool has1 = q1 < nu;
    int off0 = lane * 16, off1 = min(q1 * 16, bb - 16);
    u32x4 a0 = *(const u32x4a8*)(s + off0), a1 = *(const u32x4a8*)(s + off1);
#pragma unroll
    for (int x = 1; x < 10; ++x) {
        a0 ^= *(const u32x4a8*)(s + off0 + (size_t)x * bb);
        a1 ^= *(const u32x4a8*)(s + off1 + (size_t)x * bb);
    }
    *(u32x4a8*)(o + off0) = a0;
    if (has1) {
        if (q1 * 16 + 16 <= bb) *(u32x4a8*)(o + off1) = a1;
        else *(uint64_t*)(o + q1 * 16) = ((uint64_t)a1.w << 32) | a1.z;
    }
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); f();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
    long long G = argc > 1 ? atoll(argv[1]) : 65536;
    int k = argc > 2 ? atoi(argv[2]) : 10;
    int bb = argc > 3 ? atoi(argv[3]) : 1352;
    int reps = argc > 4 ? atoi(argv[4]) : 30;
    size_t dbytes = (size_t)G * k * bb, pbytes = (size_t)G * bb;
    size_t big = 4ull << 30;
    uint8_t *d, *p, *x, *y;
    CK(hipMalloc(&d, dbytes + 4096)); CK(hipMalloc(&p, pbytes + 4096));
    CK(hipMalloc(&x, big)); CK(hipMalloc(&y, big));
    CK(hipMemset(d, 0x5a, dbytes)); CK(hipMemset(x, 0x33, big));
    u32x4* sink; CK(hipMalloc(&sink, 64));
    size_t n16 = big / 16;
    const int NB = 256 * 8 * 4;
    double bytes_xor = (double)(dbytes + pbytes);
    auto rep = [&](const char* name, float ms, double bytes) {
        printf("%-34s %9.1f us  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", name, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
    };
    rep("read_only 4GiB", timeit([&] { read_only<<<NB, 256>>>((u32x4*)x, n16, sink); }, reps), (double)big);
    rep("read_only_nt 4GiB", timeit([&] { read_only_nt<<<NB, 256>>>((u32x4*)x, n16, sink); }, reps), (double)big);
    rep("copy 4GiB", timeit([&] { copy_k<<<NB, 256>>>((u32x4*)x, (u32x4*)y, n16); }, reps), 2.0 * big);
    {
        int bba = 1408, nua = bba / 16; unsigned tot = (unsigned)(G * nua);
        uint8_t* da; uint8_t* pa;
        CK(hipMalloc(&da, (size_t)G * k * bba)); CK(hipMalloc(&pa, (size_t)G * bba));
        rep("xor_aligned bb=1408", timeit([&] { xor_aligned<<<(tot + 255) / 256, 256>>>(da, pa, k, bba, nua, tot); }, reps), (double)G * (k + 1) * bba);
        CK(hipFree(da)); CK(hipFree(pa));
    }
    int nu16 = (bb + 15) / 16; unsigned t16 = (unsigned)(G * nu16);
    int nu8 = bb / 8; unsigned t8 = (unsigned)(G * nu8);
    rep("v_flat16", timeit([&] { v_flat16<false><<<(t16 + 255) / 256, 256>>>(d, p, k, bb, nu16, t16); }, reps), bytes_xor);
    rep("v_flat16_nt", timeit([&] { v_flat16<true><<<(t16 + 255) / 256, 256>>>(d, p, k, bb, nu16, t16); }, reps), bytes_xor);
    rep("v_flat8", timeit([&] { v_flat8<<<(t8 + 255) / 256, 256>>>(d, p, k, bb, nu8, t8); }, reps), bytes_xor);
    rep("v_wave16 (v0 shipped)", timeit([&] { v_wave16<<<(unsigned)((G + 3) / 4), 256>>>(d, p, k, bb, G); }, reps), bytes_xor);
    unsigned th2 = (unsigned)(((t16 + 127) / 128) * 64);
    rep("v_flat16x2", timeit([&] { v_flat16x2<<<(th2 + 255) / 256, 256>>>(d, p, k, bb, nu16, t16); }, reps), bytes_xor);
    rep("v_wave2", timeit([&] { v_wave2<<<(unsigned)((G + 3) / 4), 256>>>(d, p, k, bb, G); }, reps), bytes_xor);
    // repeat the first ones to see drift
    rep("v_flat16 (again)", timeit([&] { v_flat16<false><<<(t16 + 255) / 256, 256>>>(d, p, k, bb, nu16, t16); }, reps), bytes_xor);
    rep("v_wave16 (again)", timeit([&] { v_wave16<<<(unsigned)((G + 3) / 4), 256>>>(d, p, k, bb, G); }, reps), bytes_xor);
    // bigger batch (L3 cannot hold anything)
    return 0;
}
