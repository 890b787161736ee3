// Microbenchmark: chip-wide FNV-1a (mod 2^96) chain rate of limb forms on gfx950 (not product
// code).  Every lane runs one serial chain over NB bytes held in registers (no memory in the
// loop), so the rate is the VALU/latency bound of the chain form alone:
//   limb22: five 22-bit limbs, carry-save, v_mul_u32_u24 (pp_null.hip's Fnv);
//   mad64:  three 32-bit limbs, one 32x32->64 multiply-add per limb (v_mad_u64_u32);
//   mad64b: as mad64, the low limb's product split into mul_lo / mul_hi.
// The chains' tags are compared against each other on the host.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 fnv_rate.hip -o fnv_rate && ./fnv_rate
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

struct Limb22 {
    uint32_t l0, l1, l2, l3, l4;
    __device__ void init() {
        l0 = 0x15c58du, l1 = 0x05d58au, l2 = 0x262b82u, l3 = 0x2ec050u, l4 = 0x272e07u;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        constexpr uint32_t M = (1u << 22) - 1u;
        const uint32_t x0 = l0 ^ b;
        const uint32_t p0 = __umul24(x0, 315u), p1 = __umul24(l1, 315u);
        const uint32_t p2 = __umul24(l2, 315u), p3 = __umul24(l3, 315u);
        const uint32_t p4 = __umul24(l4, 315u);
        l4 = p4 + (p3 >> 22) + x0;
        l1 = (p1 & M) + (p0 >> 22);
        l2 = (p2 & M) + (p1 >> 22);
        l3 = (p3 & M) + (p2 >> 22);
        l0 = p0 & M;
    }
    __device__ void tag(uint32_t* t) const {
        constexpr uint32_t M = (1u << 22) - 1u;
        uint32_t c = 0, n[5];
        const uint32_t l[5] = {l0, l1, l2, l3, l4};
        for (int j = 0; j < 5; ++j) {
            const uint32_t v = l[j] + c;
            n[j] = v & M;
            c = v >> 22;
        }
        const uint64_t lo = (uint64_t)n[0] | ((uint64_t)n[1] << 22) | ((uint64_t)n[2] << 44);
        t[0] = (uint32_t)lo;
        t[1] = (uint32_t)(lo >> 32);
        t[2] = (n[2] >> 20) | (n[3] << 2) | (n[4] << 24);
    }
};

// h mod 2^96 as three 32-bit words; h * P = h * 315 + (h << 88)
struct Mad64 {
    uint32_t h0, h1, h2;
    __device__ void init() {
        // low 96 bits of kOffset, from the 22-bit limbs above
        const uint64_t lo = 0x15c58dull | (0x05d58aull << 22) | (0x262b82ull << 44);
        h0 = (uint32_t)lo;
        h1 = (uint32_t)(lo >> 32);
        h2 = (0x262b82u >> 20) | (0x2ec050u << 2) | (0x272e07u << 24);
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        const uint32_t x0 = h0 ^ b;
        const uint64_t p0 = (uint64_t)x0 * 315u;
        const uint64_t p1 = (uint64_t)h1 * 315u + (p0 >> 32);
        h2 = h2 * 315u + (uint32_t)(p1 >> 32) + (x0 << 24);
        h0 = (uint32_t)p0;
        h1 = (uint32_t)p1;
    }
    __device__ void tag(uint32_t* t) const { t[0] = h0, t[1] = h1, t[2] = h2; }
};

// as Mad64, the carries out of h0 and h1 from the 24-bit high multiply (h * 315 < 2^41)
struct Mad64b {
    uint32_t h0, h1, h2;
    __device__ void init() {
        Mad64 m;
        m.init();
        h0 = m.h0, h1 = m.h1, h2 = m.h2;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        const uint32_t x0 = h0 ^ b;
        const uint32_t lo0 = x0 * 315u, c0 = __umulhi(x0, 315u);
        const uint32_t lo1 = h1 * 315u, c1a = __umulhi(h1, 315u);
        const uint32_t s1 = lo1 + c0;
        const uint32_t c1 = c1a + (s1 < lo1 ? 1u : 0u);
        h2 = h2 * 315u + c1 + (x0 << 24);
        h0 = lo0;
        h1 = s1;
    }
    __device__ void tag(uint32_t* t) const { t[0] = h0, t[1] = h1, t[2] = h2; }
};

template <class H>
__global__ __launch_bounds__(256) void chain_kernel(const uint32_t* data, int reps, uint32_t* tags) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = data[(t * 16 + i) & 4095];
    H h;
    h.init();
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            h.byte(w[i] & 0xFFu);
            h.byte((w[i] >> 8) & 0xFFu);
            h.byte((w[i] >> 16) & 0xFFu);
            h.byte(w[i] >> 24);
        }
    }
    uint32_t tg[3];
    h.tag(tg);
    tags[3 * t] = tg[0], tags[3 * t + 1] = tg[1], tags[3 * t + 2] = tg[2];
}

template <class H>
static double run(const char* name, const uint32_t* d, uint32_t* tags, int blocks, int reps) {
    chain_kernel<H><<<blocks, 256>>>(d, reps, tags);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    chain_kernel<H><<<blocks, 256>>>(d, reps, tags);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)blocks * 256 * reps * 64;
    printf("%-8s %6d blocks: %.3f ms, %.1f GB/s hashed\n", name, blocks, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
    return ms;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t h[4096];
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < 4096; ++i) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        h[i] = (uint32_t)(s >> 32);
    }
    uint32_t *d = nullptr, *t0 = nullptr, *t1 = nullptr, *t2 = nullptr;
    const int maxb = cus * 32;
    CK(hipMalloc(&d, sizeof(h)));
    CK(hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice));
    CK(hipMalloc(&t0, (size_t)maxb * 256 * 12));
    CK(hipMalloc(&t1, (size_t)maxb * 256 * 12));
    CK(hipMalloc(&t2, (size_t)maxb * 256 * 12));
    const int reps = 64;   // 4 KiB per lane
    for (int occ = 4; occ <= 32; occ *= 2) {
        const int blocks = cus * occ;
        run<Limb22>("limb22", d, t0, blocks, reps);
        run<Mad64>("mad64", d, t1, blocks, reps);
        run<Mad64b>("mad64b", d, t2, blocks, reps);
    }
    const size_t n = (size_t)maxb * 256 * 3;
    uint32_t* a = (uint32_t*)malloc(n * 4);
    uint32_t* b = (uint32_t*)malloc(n * 4);
    uint32_t* c = (uint32_t*)malloc(n * 4);
    CK(hipMemcpy(a, t0, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b, t1, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c, t2, n * 4, hipMemcpyDeviceToHost));
    size_t bad1 = 0, bad2 = 0;
    for (size_t i = 0; i < n; ++i) bad1 += a[i] != b[i], bad2 += a[i] != c[i];
    printf("tag mismatches: mad64 %zu, mad64b %zu of %zu words\n", bad1, bad2, n);
    return 0;
}
