// Microbenchmark: where the m = 1 decode loses time against the encode (config A,
// 65,536 x (10+1) x 1352 B).  Instantiates xor_dma_kernel with its PROBE bits.  Timing
// only.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 xor_dec_mb.hip -o xor_dec_mb
#include "../../quic_amd/csrc/xor_dma.hip"
#include <stdio.h>

using namespace qfec;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void fill(uint8_t* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (size_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + 1) * 0x9E3779B97F4A7C15ull;
}
__global__ void rows_fill(uint8_t* r, long long G, int k) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < G * k; i += (long long)gridDim.x * blockDim.x) {
        const int slot = (int)(i % k);
        r[i] = slot == 0 ? (uint8_t)k : (uint8_t)slot;   // slot 0 carries the parity, row 0 lost
    }
}

template <bool DEC, bool FUSED, int PROBE>
void run(const char* name, const uint8_t* in, uint8_t* out, const uint8_t* rows, uint8_t* rows_out,
         int32_t* status, long long G, int waves) {
    const int k = 10, bb = 1352;
    const size_t lds = (size_t)waves * 2 * (14 * 1024 + 80) + waves * 64;
    const unsigned nb = 256;
    auto kern = xor_dma_kernel<14, 2, DEC, FUSED, PROBE>;
    const long long ogs = DEC ? (long long)k * bb : bb;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(nb), dim3(waves * 64), lds, 0, in, out, nullptr, rows, rows_out, status, k, bb, G, ogs);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(kern, dim3(nb), dim3(waves * 64), lds, 0, in, out, nullptr, rows, rows_out, status, k, bb, G, ogs);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("%-34s waves=%d %8.4f ms  %6.0f GB/s\n", name, waves, ms, (double)G * 11 * bb / ms / 1e6);
}

int main() {
    const long long G = 65536;
    const size_t nb = (size_t)G * 10 * 1352;
    uint8_t *in, *out, *rows, *rows_out; int32_t* st;
    CK(hipMalloc(&in, nb)); CK(hipMalloc(&out, nb)); CK(hipMalloc(&rows, G * 10)); CK(hipMalloc(&rows_out, G * 10));
    CK(hipMalloc(&st, G * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, nb);
    hipLaunchKernelGGL(rows_fill, dim3(1024), dim3(256), 0, 0, rows, G, 10);
    CK(hipDeviceSynchronize());
    for (int w : {3}) {
        run<true, true, 8>("decode plain stores", in, out, rows, rows_out, st, G, w);
        run<false, false, 8>("encode plain stores", in, out, nullptr, nullptr, nullptr, G, w);
        run<true, true, 0>("decode in place", in, (uint8_t*)in, rows, rows_out, st, G, w);
        run<true, true, 8>("decode in place plain", in, (uint8_t*)in, rows, rows_out, st, G, w);
    }
    for (int w : {3, 4}) {
        run<false, false, 0>("encode", in, out, nullptr, nullptr, nullptr, G, w);
        run<true, true, 0>("decode", in, out, rows, rows_out, st, G, w);
        run<true, true, 1>("decode no-bookkeeping", in, out, rows, rows_out, st, G, w);
        run<true, true, 2>("decode dense-out", in, out, rows, rows_out, st, G, w);
        run<true, true, 3>("decode no-bk dense", in, out, rows, rows_out, st, G, w);
        run<true, true, 7>("decode no-bk dense no-tags", in, out, rows, rows_out, st, G, w);
    }
    return 0;
}
