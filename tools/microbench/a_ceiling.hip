// Microbenchmark: the HBM ceiling of config A's access shape on gfx950 (not product code).
//
// Config A moves, per group, k = 10 blocks of 1352 B in (13,520 B, one contiguous range)
// and one 1352 B block out; 65,536 groups = 886 MB read + 88.6 MB written per launch.
// The product kernel (xor_dma.hip) streams whole groups into per-wave LDS slots with
// global_load_lds_dwordx4 (nt) and XORs them out of LDS.  This file measures the same
// byte movement with NO arithmetic, over a sweep of shapes, to find the best rate this
// access shape reaches on the box:
//   grp   whole groups into NSLOT LDS slots per wave, W waves per workgroup (one workgroup
//         per CU), optional 1352 B store per group (the A shape minus the XOR)
//   ring  a contiguous range per wave through an NS x 1 KiB LDS ring (read only)
//   reg   global_load_dwordx4 nt into registers, U loads in flight per lane, persistent
//         waves over consecutive 1 KiB pieces, optional 1/10 stores
// Every kernel reads every byte of the 886 MB input exactly once.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 a_ceiling.hip -o a_ceiling && ./a_ceiling
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                       \
            exit(1);                                                            \
        }                                                                       \
    } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N <= 63, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int K = 10, BB = 1352, GB = K * BB;   // 13,520 B per group
constexpr int NP = (GB + 1023) / 1024;          // 14 pieces

// whole groups into NSLOT slots per wave; STORE: write a 1352-B block per group (nt)
// SPOL: store policy 0 = nt, 1 = plain write-back; BLOCKED: wave w takes a contiguous
// run of groups instead of g0, g0 + W, ...
// XMAP: 1 = logical wave ids XCD-major (hardware deals workgroups round-robin over the 8
// XCDs), so groups g and g + 1 run on the same XCD and a 128-B output line shared by two
// groups is written through ONE L2; 2 = the same plus a line-padded output stride (1408 B,
// every group's output whole lines: the upper bound of removing shared lines)
template <int NSLOT, bool STORE, int AUX, int SPOL = 0, bool BLOCKED = false, int XMAP = 0>
__global__ __launch_bounds__(256) void grp_kernel(const uint8_t* in, uint8_t* out, long long groups,
                                                  uint32_t* sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int SLOT = NP * 1024;
    const int nwv = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    uint8_t* myl = smem + (size_t)w * NSLOT * SLOT;
    const long long nw = (long long)gridDim.x * nwv;
    long long wid = (long long)blockIdx.x * nwv + w;
    if (XMAP) {   // requires gridDim.x % 8 == 0
        const int nbx = gridDim.x >> 3, x = blockIdx.x & 7, j = blockIdx.x >> 3;
        wid = ((long long)x * nbx + j) * nwv + w;
    }
    constexpr int OST = XMAP == 2 ? 1408 : BB;
    long long W = nw, g0 = wid, cnt;
    if (BLOCKED) {
        const long long per = (groups + nw - 1) / nw;
        g0 = wid * per;
        W = 1;
        if (g0 >= groups) return;
        cnt = min(per, groups - g0);
    } else {
        if (g0 >= groups) return;
        cnt = (groups - 1 - g0) / W + 1;
    }
    auto issue = [&](long long i, int slot) {
        const uint8_t* src = in + (g0 + i * W) * GB;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const int off = min(p * 1024 + lane * 16, GB - 16);
            __builtin_amdgcn_global_load_lds(GPTR(src + off), LPTR(myl + slot * SLOT + p * 1024), 16,
                                             0, AUX);
        }
    };
    constexpr int SPG = STORE ? 3 : 0;   // stores per group (169 qwords / 64 lanes)
    constexpr int WAIT = (NSLOT - 1) * (NP + SPG);
    static_assert(WAIT <= 63, "vmcnt");
    for (int u = 0; u < NSLOT - 1; ++u)
        if (u < cnt) issue(u, u);
    uint64_t acc = 0;
    for (long long i = 0; i < cnt; ++i) {
        const int u = (int)(i % NSLOT);
        if (i + NSLOT - 1 < cnt) {
            issue(i + NSLOT - 1, (int)((i + NSLOT - 1) % NSLOT));
            wait_vm<WAIT>();
        } else {
            wait_vm<0>();
        }
        const uint8_t* L = myl + u * SLOT;
        if (STORE) {
            uint8_t* o = out + (g0 + i * W) * OST;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int q = min(lane + 64 * j, BB / 8 - 1);
                const uint64_t v = *(const uint64_t*)(L + q * 8);
                if (SPOL == 0) __builtin_nontemporal_store(v, (uint64_t*)(o + q * 8));
                else *(uint64_t*)(o + q * 8) = v;
            }
        } else {
            acc ^= *(const uint64_t*)(L + lane * 8);
        }
    }
    if (!STORE && acc == 0x123456789abcdefull) sink[0] = 1;
}

// contiguous range per wave through an NS-slot ring of 1 KiB pieces (read only)
template <int NS, int AUX>
__global__ __launch_bounds__(256) void ring_kernel(const uint8_t* in, long long pieces_per_wave,
                                                   uint32_t* sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int nwv = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    uint8_t* ring = smem + (size_t)w * NS * 1024;
    const long long wave = (long long)blockIdx.x * nwv + w;
    const uint8_t* s = in + wave * pieces_per_wave * 1024 + lane * 16;
    for (long long i = 0; i < pieces_per_wave; ++i) {
        __builtin_amdgcn_global_load_lds(GPTR(s + i * 1024), LPTR(ring + (i % NS) * 1024), 16, 0,
                                         AUX);
        if (i >= NS - 1) wait_vm<NS - 1>();
    }
    wait_vm<0>();
    if (((uint32_t*)ring)[lane] == 0x12345678u) sink[0] = 1;
}

// register loads: persistent waves, wave w takes pieces w, w + W, ... (1 KiB each), U in
// flight per lane; STORE: every 10th piece is also written out (the A byte ratio)
template <int U, bool STORE>
__global__ __launch_bounds__(256) void reg_kernel(const u32x4* in, u32x4* out, long long pieces,
                                                  uint32_t* sink) {
    const int lane = threadIdx.x & 63;
    const long long W = (long long)gridDim.x * (blockDim.x >> 6);
    const long long w0 = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    u32x4 acc = {0, 0, 0, 0};
    for (long long p = w0; p < pieces; p += U * W) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = min(p + u * W, pieces - 1);
            v[u] = __builtin_nontemporal_load(in + q * 64 + lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = p + u * W;
            if (STORE && q < pieces && q % 10 == 0)
                __builtin_nontemporal_store(v[u], out + (q / 10) * 64 + lane);
            else
                acc ^= v[u];
        }
    }
    if ((acc.x & 0xffffff) == 0x123456) sink[0] = acc.y;
}

struct Timer {
    hipEvent_t a, b;
    Timer() {   // device-scope release: no system-scope cache flush inside the interval
        CK(hipEventCreateWithFlags(&a, hipEventReleaseToDevice));
        CK(hipEventCreateWithFlags(&b, hipEventReleaseToDevice));
    }
};

template <class F>
double time_ms(F&& launch, int reps) {
    Timer t;
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(t.a));
        launch();
        CK(hipEventRecord(t.b));
        CK(hipEventSynchronize(t.b));
        float x;
        CK(hipEventElapsedTime(&x, t.a, t.b));
        ms.push_back(x);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const long long G = 65536;
    const size_t in_bytes = (size_t)G * GB, out_bytes = (size_t)G * BB;
    uint8_t *in, *out;
    uint32_t* sink;
    CK(hipMalloc(&in, in_bytes + 4096));
    CK(hipMalloc(&out, (size_t)G * 1408 + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 0x5a, in_bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 30;
    auto report = [&](const char* name, double ms, size_t bytes) {
        printf("%-34s %8.1f us  %6.3f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    char nm[128];
    // grp: slots x waves (one workgroup per CU), read only and with the A stores
#define GRPX(NSLOT, WV, ST, AUX, SP, BL, WPC) GRPM(NSLOT, WV, ST, AUX, SP, BL, WPC, 0)
#define GRPM(NSLOT, WV, ST, AUX, SP, BL, WPC, XM)                                           \
    {                                                                                       \
        const size_t lds = (size_t)WV * NSLOT * NP * 1024;                                  \
        if (lds * WPC <= 160 * 1024) {                                                      \
            auto kern = grp_kernel<NSLOT, ST, AUX, SP, BL, XM>;                                 \
            if (lds > 64 * 1024)                                                            \
                CK(hipFuncSetAttribute((const void*)kern,                                   \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
            const unsigned nb = (unsigned)std::min<long long>((G + WV - 1) / WV, cus * WPC); \
            double ms = time_ms([&] { kern<<<nb, WV * 64, lds>>>(in, out, G, sink); }, reps); \
            snprintf(nm, sizeof nm, "grp s=%d w=%d x%d %s aux=%d st=%s%s%s", NSLOT, WV, WPC,\
                     ST ? "rd+wr" : "rd", AUX, SP ? "wb" : "nt", BL ? " blocked" : "",     \
                     XM == 1 ? " xcd" : XM == 2 ? " xcd+pad" : "");                       \
            report(nm, ms, in_bytes + (ST ? out_bytes : 0));                                \
        }                                                                                   \
    }
#define GRP(NSLOT, WV, ST, AUX) GRPX(NSLOT, WV, ST, AUX, 0, false, 1)
    GRP(2, 1, true, 2) GRP(3, 1, true, 2) GRP(4, 1, true, 2)
    GRP(2, 2, true, 2) GRP(2, 3, true, 2) GRP(2, 4, true, 2) GRP(3, 2, true, 2)
    GRPX(2, 1, true, 2, 0, false, 2) GRPX(2, 1, true, 2, 0, false, 3)
    GRPX(2, 1, true, 2, 1, false, 1) GRPX(2, 3, true, 2, 1, false, 1)
    GRPX(2, 1, true, 2, 0, true, 1) GRPX(2, 3, true, 2, 0, true, 1)
    GRPX(3, 1, true, 2, 0, true, 1)
    GRP(2, 1, false, 2) GRP(2, 3, false, 2)
    GRPM(2, 1, true, 2, 0, false, 1, 1) GRPM(2, 3, true, 2, 0, false, 1, 1)
    GRPM(2, 1, true, 2, 1, false, 1, 1) GRPM(2, 3, true, 2, 1, false, 1, 1)
    GRPM(2, 1, true, 2, 0, false, 1, 2) GRPM(2, 3, true, 2, 0, false, 1, 2)
    GRPM(2, 1, true, 2, 0, false, 2, 1) GRPM(3, 1, true, 2, 0, false, 1, 1)
    GRP(2, 1, true, 2) GRP(2, 3, true, 2)
    // ring: read only, NS slots x waves per workgroup (workgroups fill the CU by LDS)
#define RING(NS, WV, AUX)                                                                   \
    {                                                                                       \
        const size_t lds = (size_t)WV * NS * 1024;                                          \
        const int per_cu = std::max(1, (int)((160 * 1024) / lds));                          \
        const long long waves = (long long)cus * per_cu * WV;                               \
        const long long ppw = (long long)(in_bytes / 1024) / waves;                         \
        if (lds > 64 * 1024)                                                                \
            CK(hipFuncSetAttribute((const void*)ring_kernel<NS, AUX>,                       \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));  \
        double ms = time_ms([&] {                                                           \
            ring_kernel<NS, AUX><<<(unsigned)(waves / WV), WV * 64, lds>>>(in, ppw, sink);  \
        }, reps);                                                                           \
        snprintf(nm, sizeof nm, "ring slots=%d waves=%d x%d/CU aux=%d", NS, WV, per_cu, AUX); \
        report(nm, ms, (size_t)ppw * waves * 1024);                                         \
    }
    RING(8, 4, 2) RING(16, 4, 2) RING(32, 4, 2) RING(16, 2, 2) RING(40, 1, 2) RING(10, 4, 2)
    RING(16, 4, 0)
    // reg: U loads in flight per lane, waves per CU from the grid
#define REG(U, ST, WPC)                                                                     \
    {                                                                                       \
        const long long pieces = (long long)(in_bytes / 1024);                              \
        double ms = time_ms([&] {                                                           \
            reg_kernel<U, ST><<<(unsigned)(cus * WPC / 4), 256>>>((const u32x4*)in,         \
                                                                 (u32x4*)out, pieces, sink); \
        }, reps);                                                                           \
        snprintf(nm, sizeof nm, "reg U=%d waves/CU=%d %s", U, WPC, ST ? "rd+wr" : "rd");   \
        report(nm, ms, (size_t)pieces * 1024 + (ST ? (size_t)(pieces / 10) * 1024 : 0));   \
    }
    REG(4, false, 8) REG(8, false, 8) REG(8, false, 16) REG(16, false, 8) REG(4, false, 32)
    REG(8, true, 8) REG(8, true, 16) REG(16, true, 8)
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(sink));
    return 0;
}
