// Microbenchmark: LDS-DMA (global_load_lds_dwordx4) streaming vs plain loads on gfx950,
// for the m = 1 XOR encode layout (G groups x k blocks x bb bytes).  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 dma_variants.hip -o dma_variants
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N> __device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
    else if constexpr (N == 31) asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
    else if constexpr (N == 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
    else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else static_assert(N < 0, "add a case");
}

// Read-only ingest: each wave streams a contiguous range through an LDS ring of
// NS 1-KiB slots, keeping NS-1 DMA instructions in flight.  No consumer.
template <int AUX, int NS>
__global__ __launch_bounds__(256) void dma_read(const uint8_t* __restrict__ src, size_t bytes_per_wave, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][NS][1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + w;
    const uint8_t* s = src + wave * bytes_per_wave + lane * 16;
    const int n = (int)(bytes_per_wave / 1024);
    for (int i = 0; i < n; ++i) {
        __builtin_amdgcn_global_load_lds(GPTR(s + (size_t)i * 1024), LPTR(lds[w][i % NS]), 16, 0, AUX);
        if (i >= NS - 1) wait_vm<NS - 1 == 15 ? 14 : (NS - 1 == 8 ? 8 : 4)>();
    }
    wait_vm<0>();
    if (((uint32_t*)lds[w][0])[lane] == 0x12345678u) sink[0] = 1;
}

__global__ void read_nt_unroll(const u32x4* __restrict__ a, size_t n, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        u32x4 a0 = __builtin_nontemporal_load(&a[i]);
        u32x4 a1 = __builtin_nontemporal_load(&a[i + stride]);
        u32x4 a2 = __builtin_nontemporal_load(&a[i + 2 * stride]);
        u32x4 a3 = __builtin_nontemporal_load(&a[i + 3 * stride]);
        acc ^= a0 ^ a1 ^ a2 ^ a3;
    }
    if ((acc.x & 0xfffffff) == 0x1234567) sink[0] = acc;
}

// XOR encode (k = 10, bb = 1352): each wave owns groups g = wave, wave + W, ...; a group's
// k*bb bytes are contiguous and 16-aligned (k even), DMA'd into one of 2 LDS slots.
template <int AUX, int WPB>
__global__ __launch_bounds__(WPB * 64) void xor_dma(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, int bb, long long G) {
    constexpr int K = 10;
    constexpr int GB = K * 1352;                  // 13520
    constexpr int NDMA = (GB + 1023) / 1024;      // 14
    constexpr int SLOT = NDMA * 1024;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* myl = smem + (size_t)w * 2 * SLOT;
    const long long W = (long long)gridDim.x * WPB;
    long long g = (long long)blockIdx.x * WPB + w;
    if (g >= G) return;
    auto issue = [&](long long gg, int slot) {
        const uint8_t* s = d + gg * GB;
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
            const int off = min(i * 1024 + lane * 16, GB - 16);   // clamp the last partial piece
            __builtin_amdgcn_global_load_lds(GPTR(s + off), LPTR(myl + slot * SLOT + i * 1024), 16, 0, AUX);
        }
    };
    issue(g, 0);
    int slot = 0;
    for (; g < G; g += W) {
        const long long gn = g + W;
        if (gn < G) { issue(gn, slot ^ 1); wait_vm<NDMA>(); } else wait_vm<0>();
        const uint8_t* L = myl + slot * SLOT;
        uint8_t* o = p + g * 1352;
        for (int q = lane; q < 169; q += 64) {
            uint64_t acc = *(const uint64_t*)(L + q * 8);
#pragma unroll
            for (int x = 1; x < K; ++x) acc ^= *(const uint64_t*)(L + x * 1352 + q * 8);
            *(uint64_t*)(o + q * 8) = acc;
        }
        slot ^= 1;
    }
}


// v2: WPB waves x NSLOT group slots per wave; WAITST = store instructions of the previous
// group that may stay in flight; NTST = non-temporal parity stores.
template <int WPB, int NSLOT, int WAITST, bool NTST>
__global__ __launch_bounds__(WPB * 64) void xor_dma2(const uint8_t* __restrict__ d, uint8_t* __restrict__ p, long long G) {
    constexpr int K = 10, BB = 1352, GB = K * BB, NDMA = (GB + 1023) / 1024, SLOT = NDMA * 1024;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* myl = smem + (size_t)w * NSLOT * SLOT;
    const long long W = (long long)gridDim.x * WPB;
    long long g = (long long)blockIdx.x * WPB + w;
    if (g >= G) return;
    auto issue = [&](long long gg, int slot) {
        const uint8_t* s = d + gg * GB;
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
            const int off = min(i * 1024 + lane * 16, GB - 16);
            __builtin_amdgcn_global_load_lds(GPTR(s + off), LPTR(myl + slot * SLOT + i * 1024), 16, 0, 2);
        }
    };
    // prologue: NSLOT-1 groups in flight
#pragma unroll
    for (int j = 0; j < NSLOT - 1; ++j) if (g + j * W < G) issue(g + j * W, j);
    int slot = 0;
    for (int it = 0; g < G; g += W, ++it) {
        const long long gn = g + (NSLOT - 1) * W;
        const bool more = gn < G;
        if (more) issue(gn, (slot + NSLOT - 1) % NSLOT);
        // wait for group g: younger ops = (NSLOT-1) groups of DMA (if issued) + stores
        if (more) {
            if constexpr (NSLOT == 2) { if constexpr (WAITST) wait_vm<17>(); else wait_vm<14>(); }
            else if constexpr (NSLOT == 3) { if constexpr (WAITST) wait_vm<31>(); else wait_vm<28>(); }
            else wait_vm<0>();
        } else {
            wait_vm<0>();
        }
        const uint8_t* L = myl + slot * SLOT;
        uint8_t* o = p + g * BB;
        for (int q = lane; q < 169; q += 64) {
            uint64_t acc = *(const uint64_t*)(L + q * 8);
#pragma unroll
            for (int x = 1; x < K; ++x) acc ^= *(const uint64_t*)(L + x * BB + q * 8);
            if (NTST) __builtin_nontemporal_store(acc, (uint64_t*)(o + q * 8));
            else *(uint64_t*)(o + q * 8) = acc;
        }
        slot = (slot + 1) % NSLOT;
    }
}

// reference: flat 16B plain loads (the v1 shipped kernel) with/without nt
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


template <typename F, typename R>
static float timeit2(F f, R reset, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); f();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < reps; ++i) {
        reset();
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
    long long G = argc > 1 ? atoll(argv[1]) : 65536;
    int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int k = 10, bb = 1352;
    size_t dbytes = (size_t)G * k * bb, pbytes = (size_t)G * bb;
    size_t big = 4ull << 30;
    uint8_t *d, *p, *x, *flush;
    CK(hipMalloc(&d, dbytes + 4096)); CK(hipMalloc(&p, pbytes + 4096));
    CK(hipMalloc(&x, big)); CK(hipMalloc(&flush, 512ull << 20));
    CK(hipMemset(d, 0x5a, dbytes)); CK(hipMemset(x, 0x33, big));
    uint32_t* sink; CK(hipMalloc(&sink, 64));
    // evict the 256 MiB Infinity Cache between reps so every variant starts cold
    auto reset = [&] { CK(hipMemsetAsync(flush, 1, 512ull << 20)); };
    auto rep = [&](const char* name, float ms, double bytes) {
        printf("%-36s %9.1f us  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", name, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
    };
    int cus = 256;
    // read ceilings: 4 GiB, one 1 MiB contiguous range per wave
    {
        size_t bpw = 1 << 20; int waves = (int)(big / bpw); int blocks = waves / 4;
        rep("dma_read aux0 NS16", timeit2([&] { dma_read<0, 16><<<blocks, 256>>>(x, bpw, sink); }, reset, reps), (double)big);
        rep("dma_read nt NS16", timeit2([&] { dma_read<2, 16><<<blocks, 256>>>(x, bpw, sink); }, reset, reps), (double)big);
        rep("dma_read nt NS9", timeit2([&] { dma_read<2, 9><<<blocks, 256>>>(x, bpw, sink); }, reset, reps), (double)big);
        size_t bpw2 = 64 << 10; int blocks2 = (int)(big / bpw2 / 4);
        rep("dma_read nt NS16 64K/wave", timeit2([&] { dma_read<2, 16><<<blocks2, 256>>>(x, bpw2, sink); }, reset, reps), (double)big);
        rep("read_nt_unroll4", timeit2([&] { read_nt_unroll<<<cus * 16, 256>>>((u32x4*)x, big / 16, (u32x4*)sink); }, reset, reps), (double)big);
    }
    double bx = (double)(dbytes + pbytes);
    int nu = (bb + 15) / 16; unsigned tot = (unsigned)(G * nu);
    rep("v_flat16 (cold)", timeit2([&] { v_flat16<false><<<(tot + 255) / 256, 256>>>(d, p, k, bb, nu, tot); }, reset, reps), bx);
    rep("v_flat16_nt (cold)", timeit2([&] { v_flat16<true><<<(tot + 255) / 256, 256>>>(d, p, k, bb, nu, tot); }, reset, reps), bx);
    constexpr int SLOT = 14 * 1024;
#define RUNV(WPB, NS, WS, NT, PERCU) do { \
        size_t lds = (size_t)WPB * NS * SLOT; \
        char name[80]; snprintf(name, sizeof name, "xor_dma2 w%d s%d ws%d nt%d x%d", WPB, NS, WS, (int)NT, PERCU); \
        rep(name, timeit2([&] { xor_dma2<WPB, NS, WS, NT><<<cus * PERCU, WPB * 64, lds>>>(d, p, G); }, reset, reps), bx); } while (0)
    RUNV(4, 2, 0, false, 1);
    RUNV(4, 2, 1, false, 1);
    RUNV(4, 2, 1, true, 1);
    RUNV(3, 3, 1, false, 1);
    RUNV(3, 3, 1, true, 1);
    RUNV(5, 2, 1, false, 1);
    RUNV(5, 2, 1, true, 1);
    RUNV(2, 2, 1, true, 2);
    RUNV(2, 3, 1, true, 1);
    RUNV(8, 1, 0, true, 1);
    RUNV(4, 1, 0, true, 2);
    RUNV(11, 1, 0, true, 1);
    // correctness of xor_dma vs v_flat16
    {
        std::vector<uint8_t> h(dbytes);
        for (size_t i = 0; i < dbytes; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
        CK(hipMemcpy(d, h.data(), dbytes, hipMemcpyHostToDevice));
        uint8_t* p2; CK(hipMalloc(&p2, pbytes));
        v_flat16<false><<<(tot + 255) / 256, 256>>>(d, p2, k, bb, nu, tot);
        xor_dma2<3, 3, 1, true><<<cus, 192, 3 * 3 * SLOT>>>(d, p, G);
        std::vector<uint8_t> a(pbytes), b(pbytes);
        CK(hipMemcpy(a.data(), p, pbytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), p2, pbytes, hipMemcpyDeviceToHost));
        printf("xor_dma correct: %s\n", a == b ? "yes" : "NO");
    }
    return 0;
}
