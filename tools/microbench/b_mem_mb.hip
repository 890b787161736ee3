// Microbenchmark: memory paths for the bit-sliced B layout (65,536 groups x 32 blocks x
// 1352 B, sub-rows of 169 B).  Each variant reads every input byte once and XORs the 8
// sub-row words of every block into a per-lane accumulator (so nothing is optimised
// away), then writes one 1352-B block per group.  Timing only.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 b_mem_mb.hip -o b_mem_mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))
typedef uint32_t u32ua __attribute__((aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2a4 __attribute__((aligned(4)));

constexpr int K = 32, BB = 1352, S = 169, NW = 43;

__device__ __forceinline__ int wid() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
template <int N> __device__ __forceinline__ void vmw() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void store_out(uint8_t* out, long long g, int lane, const uint32_t (&acc)[8]) {
    if (lane < 42) {
#pragma unroll
        for (int r = 0; r < 8; ++r) *(u32ua*)(out + g * BB + r * S + 4 * lane) = acc[r];
    }
}

// (a) unaligned dword loads straight to registers, PD blocks ahead
template <int PD>
__global__ __launch_bounds__(256) void reg_unaligned(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    const long long g = (long long)blockIdx.x * 4 + wid();
    if (g >= G) return;
    const int lane = threadIdx.x & 63;
    const int c = lane < NW ? lane : NW - 1;
    const int off = min(4 * c, S - 4);
    const uint8_t* p = in + g * K * BB + off;
    uint32_t acc[8] = {0}, raw[PD][8];
#pragma unroll
    for (int u = 0; u < PD; ++u)
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[u][t] = *(const u32ua*)(p + u * BB + t * S);
#pragma unroll
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] ^= raw[x % PD][t];
        if (x + PD < K)
#pragma unroll
            for (int t = 0; t < 8; ++t) raw[x % PD][t] = *(const u32ua*)(p + (x + PD) * BB + t * S);
    }
    store_out(out, g, lane, acc);
}

// (b) aligned dword pairs + alignbyte
template <int PD>
__global__ __launch_bounds__(256) void reg_aligned(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    const long long g = (long long)blockIdx.x * 4 + wid();
    if (g >= G) return;
    const int lane = threadIdx.x & 63;
    const int c = lane < NW ? lane : NW - 1;
    const uint8_t* base = in + g * K * BB;
    uint32_t acc[8] = {0};
    u32x2 raw[PD][8];
    auto ld = [&](int x, int t) -> u32x2 {
        const uintptr_t a = (uintptr_t)(base + x * BB + t * S + 4 * c);
        return *(const u32x2a4*)(a & ~(uintptr_t)3);
    };
#pragma unroll
    for (int u = 0; u < PD; ++u)
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[u][t] = ld(u, t);
#pragma unroll
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const unsigned sh = (unsigned)((uintptr_t)(base + x * BB + t * S) & 3);
            acc[t] ^= __builtin_amdgcn_alignbyte(raw[x % PD][t].y, raw[x % PD][t].x, sh);
        }
        if (x + PD < K)
#pragma unroll
            for (int t = 0; t < 8; ++t) raw[x % PD][t] = ld(x + PD, t);
    }
    store_out(out, g, lane, acc);
}

// (c) per-wave LDS ring of NS block windows via LDS-DMA, one group per wave
template <int NS, bool CLAMP = false, int WPB = 4>
__global__ __launch_bounds__(256) void lds_ring(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    constexpr int SLOT = CLAMP ? 2048 : 1376;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const long long g = (long long)blockIdx.x * WPB + wid();
    if (g >= G) return;
    const int lane = threadIdx.x & 63;
    const int w = wid();
    uint8_t* ring = smem + w * NS * SLOT;
    const int c = lane < NW ? lane : NW - 1;
    const uint8_t* gbase = in + g * K * BB;
    auto issue = [&](int x) {
        const uintptr_t b = (uintptr_t)(gbase + x * BB);
        const uintptr_t b0 = b & ~(uintptr_t)15;
        const int U = (int)(((b + BB + 15) & ~(uintptr_t)15) - b0) >> 4;
        uint8_t* sl = ring + (x % NS) * SLOT;
        __builtin_amdgcn_global_load_lds(GPTR(b0 + lane * 16), LPTR(sl), 16, 0, 2);
        if (CLAMP) {
            // all lanes active: lanes past the window re-load its last 16 B into the
            // slot's padding (slot = 2 KiB)
            const int u = min(64 + lane, U - 1);
            __builtin_amdgcn_global_load_lds(GPTR(b0 + u * 16), LPTR(sl + 1024), 16, 0, 2);
        } else if (64 + lane < U) {
            __builtin_amdgcn_global_load_lds(GPTR(b0 + 1024 + lane * 16), LPTR(sl + 1024), 16, 0, 2);
        }
    };
    uint32_t acc[8] = {0};
#pragma unroll
    for (int x = 0; x < NS - 1; ++x) issue(x);
#pragma unroll
    for (int x = 0; x < K; ++x) {
        if (x + NS - 1 < K) { issue(x + NS - 1); vmw<2 * (NS - 1)>(); }
        else vmw<0>();
        const uint32_t blk = (uint32_t)(ring - smem) + (x % NS) * SLOT + (uint32_t)((uintptr_t)(gbase + x * BB) & 15) + 4 * c;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t o = blk + t * S;
            const uint32_t* q = (const uint32_t*)(smem + (o & ~3u));
            acc[t] ^= __builtin_amdgcn_alignbyte(q[1], q[0], o & 3u);
        }
    }
    store_out(out, g, lane, acc);
}

// (d) whole-group LDS-DMA (43,264 B per group, 43 x 1 KiB pieces), 1 group per wave,
// NWV waves per workgroup
__global__ __launch_bounds__(256) void lds_group(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const long long g = (long long)blockIdx.x * (blockDim.x >> 6) + wid();
    if (g >= G) return;
    const int lane = threadIdx.x & 63;
    uint8_t* L = smem + wid() * 44 * 1024;
    const uint8_t* src = in + g * K * BB;
    for (int p = 0; p < 43; ++p) {
        const int off = min(p * 1024 + lane * 16, K * BB - 16);
        __builtin_amdgcn_global_load_lds(GPTR(src + off), LPTR(L + p * 1024), 16, 0, 2);
    }
    vmw<0>();
    const int c = lane < NW ? lane : NW - 1;
    uint32_t acc[8] = {0};
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t o = (uint32_t)(L - smem) + x * BB + t * S + 4 * c;
            const uint32_t* q = (const uint32_t*)(smem + (o & ~3u));
            acc[t] ^= __builtin_amdgcn_alignbyte(q[1], q[0], o & 3u);
        }
    }
    store_out(out, g, lane, acc);
}


// (e) lane-flat unaligned dword loads: lanes take consecutive (group, word) pairs across
// group boundaries (every lane busy), PD blocks ahead
template <int PD>
__global__ __launch_bounds__(256) void reg_flat(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    const long long u0 = ((long long)blockIdx.x * 4 + wid()) * 64;
    const int lane = threadIdx.x & 63;
    long long u = u0 + lane;
    if (u0 >= G * NW) return;
    const bool live = u < G * NW;
    if (!live) u = G * NW - 1;
    const long long g = u / NW;
    const int c = (int)(u - g * NW);
    const int off = min(4 * c, S - 4);
    const uint8_t* p = in + g * K * BB + off;
    uint32_t acc[8] = {0}, raw[PD][8];
#pragma unroll
    for (int q = 0; q < PD; ++q)
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[q][t] = *(const u32ua*)(p + q * BB + t * S);
#pragma unroll
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] ^= raw[x % PD][t];
        if (x + PD < K)
#pragma unroll
            for (int t = 0; t < 8; ++t) raw[x % PD][t] = *(const u32ua*)(p + (x + PD) * BB + t * S);
    }
    if (live && c < 42) {
#pragma unroll
        for (int r = 0; r < 8; ++r) *(u32ua*)(out + g * BB + r * S + 4 * c) = acc[r];
    }
}

// (f) one group per wave, one ALIGNED dword per lane per sub-row; the next dword comes from
// lane + 1 over DPP (wave_shl:1) and v_alignbyte realigns
template <int PD>
__global__ __launch_bounds__(256) void reg_dpp(const uint8_t* __restrict__ in, uint8_t* out, long long G) {
    const long long g = (long long)blockIdx.x * 4 + wid();
    if (g >= G) return;
    const int lane = threadIdx.x & 63;
    const int c = lane < 44 ? lane : 43;
    const uint8_t* base = in + g * K * BB;   // 8-byte aligned
    uint32_t acc[8] = {0}, raw[PD][8];
    auto ld = [&](int x, int t) -> uint32_t {
        const int o = x * BB + t * S;   // o & 3 == t & 3 (BB % 8 == 0)
        return *(const uint32_t*)(base + (o & ~3) + 4 * c);
    };
#pragma unroll
    for (int q = 0; q < PD; ++q)
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[q][t] = ld(q, t);
#pragma unroll
    for (int x = 0; x < K; ++x) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t cur = raw[x % PD][t];
            const uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cur, 0x130, 0xf, 0xf, false);
            acc[t] ^= (t & 3) ? __builtin_amdgcn_alignbyte(nxt, cur, t & 3) : cur;
        }
        if (x + PD < K)
#pragma unroll
            for (int t = 0; t < 8; ++t) raw[x % PD][t] = ld(x + PD, t);
    }
    store_out(out, g, lane, acc);
}

template <class F>
void timeit(const char* name, F launch, double bytes, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("%-28s %8.3f ms  %6.0f GB/s (read+write)\n", name, ms, bytes / ms / 1e6);
}

__global__ void fill(uint8_t* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (size_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + 1) * 0x9E3779B97F4A7C15ull;
}

int main() {
    const long long G = 65536;
    const size_t inb = (size_t)G * K * BB;
    uint8_t *in, *out;
    CK(hipMalloc(&in, inb + 4096)); CK(hipMalloc(&out, (size_t)G * BB + 4096));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, inb);
    CK(hipDeviceSynchronize());
    const double bytes = (double)G * (K + 1) * BB;
    const unsigned nb4 = (unsigned)((G + 3) / 4);
    const int reps = 10;
    timeit("a reg_unaligned PD2", [&] { hipLaunchKernelGGL(reg_unaligned<2>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("a reg_unaligned PD4", [&] { hipLaunchKernelGGL(reg_unaligned<4>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    const unsigned nbf = (unsigned)((G * NW + 255) / 256);
    timeit("e reg_flat PD2", [&] { hipLaunchKernelGGL(reg_flat<2>, dim3(nbf), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("e reg_flat PD4", [&] { hipLaunchKernelGGL(reg_flat<4>, dim3(nbf), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("f reg_dpp PD2", [&] { hipLaunchKernelGGL(reg_dpp<2>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("f reg_dpp PD4", [&] { hipLaunchKernelGGL(reg_dpp<4>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("b reg_aligned PD2", [&] { hipLaunchKernelGGL(reg_aligned<2>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("b reg_aligned PD4", [&] { hipLaunchKernelGGL(reg_aligned<4>, dim3(nb4), dim3(256), 0, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS4", [&] { hipLaunchKernelGGL(lds_ring<4>, dim3(nb4), dim3(256), 4 * 4 * 1376, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS6", [&] { hipLaunchKernelGGL(lds_ring<6>, dim3(nb4), dim3(256), 4 * 6 * 1376, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS8", [&] { hipLaunchKernelGGL(lds_ring<8>, dim3(nb4), dim3(256), 4 * 8 * 1376, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS4 clamp", [&] { hipLaunchKernelGGL((lds_ring<4, true>), dim3(nb4), dim3(256), 4 * 4 * 2048, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS8 clamp", [&] { hipLaunchKernelGGL((lds_ring<8, true>), dim3(nb4), dim3(256), 4 * 8 * 2048, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS8 clamp 1w", [&] { hipLaunchKernelGGL((lds_ring<8, true, 1>), dim3((unsigned)G), dim3(64), 8 * 2048, 0, in, out, G); }, bytes, reps);
    timeit("c lds_ring NS16 clamp 1w", [&] { hipLaunchKernelGGL((lds_ring<16, true, 1>), dim3((unsigned)G), dim3(64), 16 * 2048, 0, in, out, G); }, bytes, reps);
    timeit("d lds_group 1w", [&] { hipLaunchKernelGGL(lds_group, dim3((unsigned)G), dim3(64), 44 * 1024, 0, in, out, G); }, bytes, reps);
    timeit("d lds_group 3w", [&] { hipLaunchKernelGGL(lds_group, dim3((unsigned)((G + 2) / 3)), dim3(192), 3 * 44 * 1024, 0, in, out, G); }, bytes, reps);
    return 0;
}
