// Probe: (1) global_load_lds_dwordx4 with 8-byte-aligned sources, (2) unaligned ds_read_b32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <string.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1;} } while (0)
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))
typedef uint32_t u32ua __attribute__((aligned(1)));
__global__ void dma8(const uint8_t* src, uint8_t* out, int shift) {
    __shared__ __attribute__((aligned(16))) uint8_t l[1024];
    int lane = threadIdx.x;
    __builtin_amdgcn_global_load_lds(GPTR(src + shift + lane * 16), LPTR(l), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) out[i] = l[i];
}
__global__ void lds_unaligned(const uint8_t* src, uint32_t* out, int off) {
    __shared__ __attribute__((aligned(16))) uint8_t l[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) l[i] = src[i];
    __syncthreads();
    out[threadIdx.x] = *(const u32ua*)(l + off + threadIdx.x * 4 + 1);   // misaligned by 1..3
}
__global__ void lds_speed(uint32_t* out, int reps, int mis) {
    __shared__ __attribute__((aligned(16))) uint8_t l[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) l[i] = i;
    __syncthreads();
    uint32_t acc = 0;
    const int lane = threadIdx.x & 63;
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc ^= *(const u32ua*)(l + ((t * 169 + lane * 4 + mis * t + r * 4) & 4095));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
    uint8_t *src, *o; uint32_t* o32;
    CK(hipMalloc(&src, 8192)); CK(hipMalloc(&o, 4096)); CK(hipMalloc(&o32, 1 << 24));
    std::vector<uint8_t> h(8192); for (int i = 0; i < 8192; ++i) h[i] = (uint8_t)(i * 7 + 3);
    CK(hipMemcpy(src, h.data(), 8192, hipMemcpyHostToDevice));
    for (int sh : {0, 4, 8, 12}) {
        dma8<<<1, 64>>>(src, o, sh); CK(hipDeviceSynchronize());
        std::vector<uint8_t> r(1024); CK(hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost));
        int bad = 0; for (int i = 0; i < 1024; ++i) bad += r[i] != h[sh + i];
        printf("dma16 src offset %2d: %s (%d bad bytes)\n", sh, bad ? "WRONG" : "ok", bad);
    }
    lds_unaligned<<<1, 64>>>(src, o32, 0); CK(hipDeviceSynchronize());
    std::vector<uint32_t> r32(64); CK(hipMemcpy(r32.data(), o32, 256, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 64; ++i) { uint32_t v; memcpy(&v, &h[i * 4 + 1], 4); bad += v != r32[i]; }
    printf("unaligned ds_read_b32: %s\n", bad ? "WRONG" : "ok");
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mis : {0, 1}) {
        lds_speed<<<2048, 256>>>(o32, 1000, mis); hipDeviceSynchronize();
        hipEventRecord(a); lds_speed<<<2048, 256>>>(o32, 1000, mis); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double reads = 2048.0 * 256 * 1000 * 8;
        printf("lds_speed mis=%d: %.3f ms, %.1f Gread/s (x4B = %.1f TB/s)\n", mis, ms, reads / ms / 1e6, reads * 4 / ms / 1e9);
    }
    return 0;
}
