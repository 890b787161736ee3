// Microbenchmark: HBM throughput of a read/write MIX on gfx950 (not product code).
//
// The encodes and decodes here differ mainly in how many bytes each group writes per byte it
// reads: config A 1/10, B encode 4/32, the QuicR preset encodes (10,10) 1/1, (10,15) 1.5/1,
// (10,20) 2/1.  This kernel moves the same mixes with NO arithmetic: every wave owns groups
// g0, g0 + W, ... of NR KiB read (one contiguous range) and NW KiB written (another), 16 B per
// lane per instruction (global_load_dwordx4 / global_store_dwordx4, nt), 4 loads in flight
// per lane, so the rate it reaches is the ceiling the mix allows with plain streaming.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 rw_mix.hip -o rw_mix && ./rw_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                       \
            exit(1);                                                            \
        }                                                                       \
    } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NR KiB read and NW KiB written per group; every lane moves 16 B per instruction
template <int NR, int NW>
__global__ __launch_bounds__(256) void mix_kernel(const u32x4* in, u32x4* out, long long groups,
                                                  unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * 4;
    const long long g0 = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (long long g = g0; g < groups; g += W) {
        const u32x4* src = in + g * (NR * 64) + lane;
        u32x4* dst = out + g * (long long)(NW * 64) + lane;
        // reads in batches of 4 in flight
#pragma unroll
        for (int p = 0; p < NR; p += 4) {
            u32x4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (p + q < NR) v[q] = __builtin_nontemporal_load(src + (p + q) * 64);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (p + q < NR) acc ^= v[q];
        }
#pragma unroll
        for (int p = 0; p < NW; ++p) {
            u32x4 o = acc;
            o.x += (uint32_t)p;   // distinct data per written KiB
            __builtin_nontemporal_store(o, dst + p * 64);
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicAdd(sink, 1ull);
}

template <int NR, int NW>
static void run(const char* name, const u32x4* in, u32x4* out, size_t rbytes_max,
                unsigned long long* sink, int cus) {
    const long long groups = (long long)(rbytes_max / (NR * 1024));
    const double bytes = (double)groups * (NR + NW) * 1024.0;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int blocks = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mix_kernel<NR, NW>, 256, 0));
    const unsigned grid = (unsigned)(cus * blocks);
    for (int w = 0; w < 3; ++w) mix_kernel<NR, NW><<<grid, 256>>>(in, out, groups, sink);
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) mix_kernel<NR, NW><<<grid, 256>>>(in, out, groups, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-24s read %2d KiB write %2d KiB per group (write share %.2f): %.3f ms, %.2f TB/s\n",
           name, NR, NW, (double)NW / (NR + NW), ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main() {
    int dev = 0;
    CK(hipSetDevice(dev));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t rbytes = 1ull << 30;   // 1 GiB read per launch (past the 256 MiB L3)
    const size_t wbytes = 2ull << 30;   // up to 2 GiB written
    u32x4 *in = nullptr, *out = nullptr;
    unsigned long long* sink = nullptr;
    CK(hipMalloc(&in, rbytes));
    CK(hipMalloc(&out, wbytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(in, 1, rbytes));
    CK(hipMemset(out, 0, wbytes));
    run<16, 0>("read only", in, out, rbytes, sink, cus);
    run<16, 2>("A-like 1/8", in, out, rbytes, sink, cus);
    run<16, 4>("B-like 1/4", in, out, rbytes, sink, cus);
    run<8, 4>("1/2", in, out, rbytes, sink, cus);
    run<8, 8>("(10,10)-like 1/1", in, out, rbytes, sink, cus);
    run<8, 12>("(10,15)-like 3/2", in, out, rbytes / 2, sink, cus);
    run<8, 16>("(10,20)-like 2/1", in, out, rbytes / 2, sink, cus);
    run<1, 8>("write mostly 8/1", in, out, rbytes / 8, sink, cus);
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(sink));
    return 0;
}
