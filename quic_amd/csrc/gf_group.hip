// gf_group.hip — m > 1 encode / decode for groups that fit in LDS (k * bb <= ~48 KiB,
// e.g. (32, 4) x 1352 B), the shape of BASELINE config B.
//
// Same arithmetic as gf_apply_kernel (bit-sliced Cauchy code, cauchy_256.cpp:90-125,
// :1502-1601; W/Z nibble expansion of gf_bitslice.h).  What differs is the data path:
// measured on MI355X (tools/microbench/b_mem_mb.hip), reading 169-byte sub-rows with
// per-lane dword loads tops out at ~4.3 TB/s and per-block LDS-DMA windows at ~1.3 TB/s,
// while streaming whole groups into LDS with 1 KiB global_load_lds_dwordx4 pieces
// reaches ~5.3 TB/s.  So:
//
//   * one workgroup of NWV waves owns one group at a time (persistent grid, groups
//     g = blockIdx.x + i * gridDim.x); the waves DMA the group's 16-byte-aligned window
//     into LDS, round-robin over 1 KiB pieces, then wait + barrier;
//   * the k blocks are split between the waves (wave w takes blocks w, w + NWV, ...); each
//     wave reads its blocks' column words from LDS (aligned ds_read2_b32 + v_alignbyte),
//     expands W/Z and applies all RC outputs of the current output chunk;
//   * the per-wave partial outputs are XOR-reduced through LDS (reusing the group
//     buffer once every wave is done reading it) and stored.
// Several workgroups share a CU (LDS ~45 KiB each), so one workgroup's DMA overlaps
// another's arithmetic; within a workgroup the loop is load -> compute -> store.
//
// Decode uses the per-group coefficients of decode_prep_kernel ([G][nchunk][k][RCP]),
// writes recovered block j into slot slots[g][j] and skips groups with nout == 0.  Every
// read of a group completes before any of its outputs is stored, so in place is safe.
#include "fec_kernels.h"
#include "gf_bitslice.h"

namespace qfec {

#define QG_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QG_LPTR(p) ((__attribute__((address_space(3))) void*)(p))
typedef uint32_t u32ua_g __attribute__((aligned(1)));
typedef uint16_t u16ua_g __attribute__((aligned(1)));

template <int N>
__device__ __forceinline__ void group_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to 63): binary dispatch.
template <int LO, int HI>
__device__ __forceinline__ void group_wait_dyn(int n) {
    if constexpr (LO == HI) {
        group_wait_vmcnt<LO>();
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (n <= MID) group_wait_dyn<LO, MID>(n);
        else group_wait_dyn<MID + 1, HI>(n);
    }
}

constexpr unsigned kGDrop = 0x80000000u;   // buffer offset past any range: lane dropped

// Workgroup barrier for LDS data only.  __syncthreads() also waits vmcnt(0), which would
// drain the next group's LDS-DMA that is deliberately still in flight.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// LDS: two group slots of `win` bytes (double buffer) + the reduction area
// red[NWV][RC][8][64] dwords.  Every wave issues exactly CNT DMA pieces per group
// (pieces past the window land in a 1 KiB trash area at the end), so
// `s_waitcnt vmcnt(CNT)` right after issuing group i + 1 retires group i.
template <int RC, int NWV, int CNT, bool DECODE>
__global__ __launch_bounds__(NWV * 64) void gf_group_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int k, int m, int bb, int nchunk, int rmax, long long coef_gstride, long long out_gstride,
    int win) {
    constexpr int RCP = RC < 4 ? 4 : RC;
    constexpr int NCW = RCP / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    const int s = bb >> 3;
    const int nw = (s + 3) >> 2;                    // column words per sub-row (<= 64 here)
    const int nwf = s >> 2;                         // full words
    const long long gb = (long long)k * bb;
    uint32_t* red = (uint32_t*)(smem + 2 * win);
    uint8_t* trash = smem + 2 * win + NWV * RC * 8 * 64 * 4;
    const int c = lane;
    const int cr = c < nw ? c : nw - 1;

    auto issue = [&](long long g, int slot) {
        const uintptr_t base = (uintptr_t)(in + g * gb);
        const uintptr_t a0 = base & ~(uintptr_t)15;
        const int units = (int)(((base + gb + 15) & ~(uintptr_t)15) - a0) >> 4;
#pragma unroll
        for (int i = 0; i < CNT; ++i) {
            const int p = w + i * NWV;
            const bool real = p * 64 < units;       // wave-uniform
            const int u = p * 64 + lane;
            if (real ? (u < units) : (lane == 0))
                __builtin_amdgcn_global_load_lds(
                    QG_GPTR(a0 + (real ? (size_t)u * 16 : 0)),
                    QG_LPTR(real ? smem + slot * win + p * 1024 : trash), 16, 0, 2);
        }
    };

    // Stores go through buffer instructions with out-of-range lanes dropped, so their
    // count per row is fixed (1 dword + 1 short if s & 2 + 1 byte if s & 1) and the wait
    // below can skip exactly the previous group's stores instead of draining them.
    const int spr = 1 + ((s >> 1) & 1) + (s & 1);
    long long g = blockIdx.x;
    if (g >= groups) return;
    issue(g, 0);
    int slot = 0;
    int stores_prev = 0;                             // store instructions of group g - 1
#pragma unroll 1
    for (; g < groups; g += gridDim.x) {
        const long long gn = g + gridDim.x;
        if (gn < groups) {
            issue(gn, slot ^ 1);
            // younger than group g's pieces: the previous group's stores + group gn
            group_wait_dyn<0, 63>(min(63, CNT + stores_prev));
        } else {
            group_wait_vmcnt<0>();
        }
        stores_prev = 0;
        lds_barrier();                             // every wave's pieces of group g
        const int ntot = DECODE ? nout[g] : m;
        const uint8_t* L = smem + slot * win;
        const uint32_t goff = (uint32_t)((uintptr_t)(in + g * gb) & 15) + (uint32_t)(L - smem);
#pragma unroll 1
        for (int ch = 0; ch < nchunk; ++ch) {
            int n = ntot - ch * RC;
            n = n < 0 ? 0 : (n > RC ? RC : n);
            if (n == 0) break;                       // uniform per workgroup
            uint32_t acc[RC][8];
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[j][r] = 0;
            const uint8_t* cg = coef + g * coef_gstride + (long long)ch * k * RCP;
            const bool p0 = !DECODE && ch == 0;      // row 0 = all ones (P0)
#pragma unroll 1
            for (int x = w; x < k; x += NWV) {
                uint32_t cwv[NCW];
#pragma unroll
                for (int q = 0; q < NCW; ++q)
                    cwv[q] = __builtin_amdgcn_readfirstlane(((const uint32_t*)(cg + x * RCP))[q]);
                const uint32_t blk = goff + (uint32_t)(x * bb) + 4 * cr;
                WZ v;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const uint32_t o = blk + t * s;
                    const uint32_t* q = (const uint32_t*)(smem + (o & ~3u));
                    v.W[t] = __builtin_amdgcn_alignbyte(q[1], q[0], o & 3u);
                }
                if (p0) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                }
                expand_wz(v);
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (j < n && !(p0 && j == 0)) {
                        const uint32_t cf = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                        apply_nibble<0>(acc[j], cf & 15u, v);
                        apply_nibble<4>(acc[j], cf >> 4, v);
                    }
                }
            }
            // ---- XOR-reduce the NWV partials through LDS: red[w][j][r][lane]
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) red[((w * RC + j) * 8 + r) * 64 + lane] = acc[j][r];
            lds_barrier();
            for (int j = w; j < n; j += NWV) {       // wave w finalises outputs w, w+NWV..
                const int o = ch * RC + j;
                const int oslot = DECODE ? slots[g * rmax + o] : o;
                uint8_t* dst = out + g * out_gstride + (long long)oslot * bb;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)bb, 0x00020000);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    uint32_t vsum = 0;
#pragma unroll
                    for (int u = 0; u < NWV; ++u) vsum ^= red[((u * RC + j) * 8 + r) * 64 + lane];
                    const unsigned at = (unsigned)(r * s + 4 * c);
                    __builtin_amdgcn_raw_buffer_store_b32(vsum, rs, c < nwf ? at : kGDrop, 0, 2);
                    if (s & 2)
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)vsum, rs,
                                                              c == nwf ? at : kGDrop, 0, 2);
                    if (s & 1)
                        __builtin_amdgcn_raw_buffer_store_b8(
                            (uint8_t)(vsum >> (8 * (s & 2))), rs,
                            c == nwf ? at + (s & 2) : kGDrop, 0, 2);
                }
                stores_prev += 8 * spr;
            }
            lds_barrier();                         // red free; slot of g free after the loop
        }
        slot ^= 1;
    }
}

namespace {

int genv(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

int group_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
    }
    return n;
}

constexpr int kGroupWaves = 8;   // two per SIMD; one workgroup per CU (LDS)

struct GroupPlan {
    int win = 0, cnt = 0;
    size_t lds = 0;
};

GroupPlan group_plan(int k, int bb, int rc) {
    GroupPlan p;
    const int units = (int)(((long long)k * bb + 30) / 16);
    const int npc = (units + 63) / 64;
    p.win = npc * 1024;
    p.cnt = (npc + kGroupWaves - 1) / kGroupWaves;
    p.lds = 2 * (size_t)p.win + (size_t)kGroupWaves * rc * 8 * 64 * 4 + 1024;
    return p;
}

}  // namespace

bool gf_group_supported(int k, int m, int bb, int rc) {
    if (!genv("QFEC_GROUP", 0)) return false;   // opt-in: gf_apply is faster on (32, 4)
    if (bb % 8 || bb / 8 < 4 || bb > 2048 || (rc != 2 && rc != 4)) return false;
    (void)m;
    const GroupPlan p = group_plan(k, bb, rc);
    return p.lds <= 160 * 1024 && p.cnt >= 1 && p.cnt <= 8;
}

hipError_t launch_gf_group(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                           const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                           long long groups, int rc, int nchunk, int rmax,
                           long long coef_gstride, long long out_gstride, bool decode,
                           hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    const GroupPlan p = group_plan(k, bb, rc);
    const unsigned threads = kGroupWaves * 64;
    const long long grid = std::min<long long>(groups, (long long)group_cus());
#define QG_GO(RCV, CNTV, DEC)                                                                \
    hipLaunchKernelGGL((gf_group_kernel<RCV, kGroupWaves, CNTV, DEC>), dim3((unsigned)grid),  \
                       dim3(threads), p.lds, st, in, out, coef, slots, nout, groups, k, m, bb, \
                       nchunk, rmax, coef_gstride, out_gstride, p.win)
#define QG_CNT(RCV, DEC)                                                                     \
    switch (p.cnt) {                                                                         \
        case 1: QG_GO(RCV, 1, DEC); break;                                                   \
        case 2: QG_GO(RCV, 2, DEC); break;                                                   \
        case 3: QG_GO(RCV, 3, DEC); break;                                                   \
        case 4: QG_GO(RCV, 4, DEC); break;                                                   \
        case 5: QG_GO(RCV, 5, DEC); break;                                                   \
        case 6: QG_GO(RCV, 6, DEC); break;                                                   \
        case 7: QG_GO(RCV, 7, DEC); break;                                                   \
        case 8: QG_GO(RCV, 8, DEC); break;                                                   \
        default: return hipErrorInvalidValue;                                                \
    }
    if (rc == 2) {
        if (decode) { QG_CNT(2, true) } else { QG_CNT(2, false) }
    } else if (rc == 4) {
        if (decode) { QG_CNT(4, true) } else { QG_CNT(4, false) }
    } else {
        return hipErrorInvalidValue;
    }
#undef QG_CNT
#undef QG_GO
    return hipGetLastError();
}

}  // namespace qfec
