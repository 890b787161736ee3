// Microbenchmark for gf_ring_kernel variants (timing only; parity is covered by the
// library tests).  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -structurizecfg-skip-uniform-regions=true \
//         -I../../quic_amd/csrc gf_ring_mb.hip -o gf_ring_mb
#include "../../quic_amd/csrc/gf_ring.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

using namespace qfec;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void fill(uint8_t* p, size_t n, uint64_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (size_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
}

struct Shape { const char* name; int k, m, bb, rc; long long G; };

template <int RC, int NS, int CNT, int TEAMS, int SPO, int PROBE>
float run(const Shape& sh, const uint8_t* in, uint8_t* out, const uint8_t* coef, int reps, int wpg_override = 0) {
    RingArgs a{};
    a.k = sh.k; a.m = sh.m; a.bb = sh.bb; a.s = sh.bb / 8;
    a.nw = (a.s + 3) / 4; a.ntiles = (a.nw + 63) / 64;
    a.nchunk = (sh.m + RC - 1) / RC; a.nwaves = a.ntiles * a.nchunk;
    a.in_gstride = (long long)sh.k * sh.bb; a.coef_gstride = 0; a.out_gstride = (long long)sh.m * sh.bb;
    a.groups = sh.G; a.rmax = 0;
    const int units = (sh.bb + 30) / 16, np = (units + 63) / 64;
    size_t lds; unsigned threads;
    if (SPO > 0) {
        a.slot_bytes = units * 16;
        a.team_bytes = NS * a.slot_bytes + ((RC * sh.bb + 4 + 15) / 16) * 16 + 16;
        lds = (size_t)TEAMS * a.team_bytes; threads = TEAMS * 64;
    } else {
        a.slot_bytes = np * 1024; a.team_bytes = NS * a.slot_bytes + 16;
        lds = a.team_bytes; threads = a.nwaves * 64;
    }
    a.in = in; a.out = out; a.coef = coef;
    auto kern = gf_ring_kernel<RC, NS, CNT, TEAMS, SPO, false, PROBE>;
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)threads, lds));
    if (wpg_override) per_cu = std::min(per_cu, wpg_override);
    const long long tpw = SPO > 0 ? TEAMS : 1;
    long long grid = std::min<long long>((sh.G + tpw - 1) / tpw, 256LL * per_cu);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, in, out, coef, (const uint8_t*)nullptr, (const int32_t*)nullptr, a);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, in, out, coef, (const uint8_t*)nullptr, (const int32_t*)nullptr, a);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    const double bytes = (double)sh.G * (sh.k + sh.m) * sh.bb;
    printf("%-6s RC=%d NS=%2d CNT=%d TEAMS=%d SPO=%d PROBE=%d lds=%6zu thr=%4u per_cu=%d grid=%lld : %8.3f ms  %6.0f GB/s\n",
           sh.name, RC, NS, CNT, TEAMS, SPO, PROBE, lds, threads, per_cu, grid, ms, bytes / ms / 1e6);
    return ms;
}

int main(int argc, char** argv) {
    const int reps = 5;
    Shape B{"B", 32, 4, 1352, 4, 65536};
    Shape D{"D", 128, 16, 9008, 8, 8192};
    size_t inB = (size_t)B.G * B.k * B.bb, inD = (size_t)D.G * D.k * D.bb;
    uint8_t *in, *out, *coef;
    size_t inmax = std::max(inB, inD);
    CK(hipMalloc(&in, inmax + 4096)); CK(hipMalloc(&out, inmax / 4 + 4096)); CK(hipMalloc(&coef, 1 << 16));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, inmax, 1ull);
    hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, coef, 1 << 16, 7ull);
    CK(hipDeviceSynchronize());
    // B: one-wave teams, staged outputs
    run<4, 8, 2, 2, 3, 0>(B, in, out, coef, reps);
    run<4, 8, 2, 4, 3, 0>(B, in, out, coef, reps);
    // B: one-wave WGs, direct stores (drain once per group)
    run<4, 4, 2, 1, 0, 0>(B, in, out, coef, reps);
    run<4, 6, 2, 1, 0, 0>(B, in, out, coef, reps);
    run<4, 8, 2, 1, 0, 0>(B, in, out, coef, reps);
    run<4, 6, 2, 1, 0, 1>(B, in, out, coef, reps);
    run<4, 6, 2, 1, 0, 2>(B, in, out, coef, reps);
    run<4, 12, 2, 1, 0, 0>(B, in, out, coef, reps);
    // D: multi-wave teams
    run<8, 8, 1, 1, 0, 0>(D, in, out, coef, reps);
    run<8, 4, 1, 1, 0, 0>(D, in, out, coef, reps);
    return 0;
}
