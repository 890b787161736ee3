// gf_ring.hip — streaming bit-sliced GF(2^8) apply for m > 1 encode and decode (gfx950).
//
// Same arithmetic as the reference's bit-sliced Cauchy code (cauchy_256.cpp:90-125,
// encode :1502-1601): out[r][j] ^= XOR_{t : bit t of c * alpha^r} in[t][j], with the W/Z
// nibble expansion of gf_bitslice.h.  What differs from gf_apply_kernel is how the bytes
// reach the lanes:
//
//   * A "team" of W waves owns a strided sequence of groups (persistent grid) and streams
//     them block after block through an LDS ring of NS block slots with
//     global_load_lds_dwordx4 (1 KiB per wave instruction, nt).  Each block is fetched as
//     the 16-byte-aligned window around it, so no alignment is required of the caller,
//     and the ring keeps NS - 1 blocks in flight across group boundaries.
//   * Every wave issues exactly CNT DMA instructions per block (pieces past the window go
//     to a trash slot), so `s_waitcnt vmcnt((NS - 2) * CNT)` retires exactly the block
//     about to be combined, with no drain at group boundaries.
//   * Lanes read their column word of the 8 sub-rows from LDS with unaligned ds_read_b32
//     (bytes past a sub-row only feed byte columns that are never stored: byte column j
//     of the output depends on byte column j of the inputs alone).
//   * Outputs: teams of one wave write the group's RC output rows to an LDS staging area
//     and store each output block with a fixed count of 8-byte buffer stores (lanes past
//     the block or outputs past n are dropped by the descriptor's range check), so the
//     store count is known at compile time and folds into the counted wait.  Multi-wave
//     teams (large blocks) store their words directly and retire the stores with a full
//     wait, once per group.
//
// One wave = (column tile of 64 words, output chunk of RC rows); a team has
// ntiles * nchunk waves.  Encode coefficients are one shared [nchunk][k][RCP] table;
// decode coefficients are per group (decode_prep_kernel), [G][nchunk][k][RCP].
#include "fec_kernels.h"
#include "gf_bitslice.h"

namespace qfec {

typedef uint32_t u32ua __attribute__((aligned(1)));
typedef uint16_t u16ua __attribute__((aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2a4 __attribute__((aligned(4)));
#define QR_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QR_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void ring_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

constexpr unsigned kDrop = 0x80000000u;   // buffer offset past any range: the lane is dropped

// PROBE (tools/microbench/gf_ring_mb.hip only; the library instantiates 0): 1 = skip the
// coefficient apply, 2 = also skip the LDS reads, 3 = skip the per-block barrier.
template <int RC, int NS, int CNT, int TEAMS, int SPO, bool DECODE, int PROBE = 0>
__global__ __launch_bounds__(1024) void gf_ring_kernel(const uint8_t* in_, uint8_t* out_,
                                                       const uint8_t* __restrict__ coef,
                                                       const uint8_t* __restrict__ slots,
                                                       const int32_t* __restrict__ nout,
                                                       const RingArgs a) {
    constexpr int RCP = RC < 4 ? 4 : RC;
    constexpr int NCW = RCP / 4;
    constexpr int AH = NS - 1;                       // blocks in flight
    constexpr bool STAGE = SPO > 0;                  // one-wave teams, LDS-staged outputs
    constexpr int S_STORES = STAGE ? RC * SPO : 0;
    constexpr int WAIT_STEADY = (AH - 1) * CNT;
    constexpr int WAIT_STORED = (AH - 1) * CNT + S_STORES > 63 ? 63 : (AH - 1) * CNT + S_STORES;
    static_assert(!STAGE || TEAMS >= 1, "staged outputs need one-wave teams");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int wv = wave_id();
    const int team = STAGE ? wv : 0;
    const int w = STAGE ? 0 : wv;
    const int W = STAGE ? 1 : a.nwaves;
    uint8_t* ring = smem + (size_t)team * a.team_bytes;
    uint8_t* stage = ring + NS * a.slot_bytes;       // STAGE: [RC][bb] (+4 pad)
    uint8_t* trash = ring + a.team_bytes - 16;        // landing spot of padding DMA pieces
    const int tile = w % a.ntiles;
    const int chunk = w / a.ntiles;
    const long long tid = STAGE ? (long long)blockIdx.x * TEAMS + team : (long long)blockIdx.x;
    const long long nt = (long long)gridDim.x * (STAGE ? TEAMS : 1);
    if (tid >= a.groups) return;                     // uniform per team (and per WG if W > 1)
    const int k = a.k, bb = a.bb, s = a.s;
    const long long ng = (a.groups - 1 - tid) / nt + 1;
    const long long nsteps = ng * k;

    // ---- DMA issue cursor
    long long ig = 0;
    int ix = 0, islot = 0;
    auto issue = [&]() {
        const long long g = tid + ig * nt;
        const uintptr_t base = (uintptr_t)(in_ + g * a.in_gstride + (long long)ix * bb);
        const uintptr_t b0 = base & ~(uintptr_t)15;
        const int U = (int)(((base + bb + 15) & ~(uintptr_t)15) - b0) >> 4;
        uint8_t* slotp = ring + islot * a.slot_bytes;
#pragma unroll
        for (int i = 0; i < CNT; ++i) {
            const int p = w + i * W;                 // piece of this block (1 KiB)
            const bool real = p * 64 < U;            // wave-uniform
            const int u = p * 64 + lane;
            if (real ? (u < U) : (lane == 0)) {
                const uint8_t* src = (const uint8_t*)b0 + (real ? (size_t)u * 16 : 0);
                __builtin_amdgcn_global_load_lds(QR_GPTR(src),
                                                 QR_LPTR(real ? slotp + p * 1024 : trash), 16, 0,
                                                 2);
            }
        }
        if (++ix == k) { ix = 0; ++ig; }
        if (++islot == NS) islot = 0;
    };

    const int c = tile * 64 + lane;                  // this lane's column word
    const int cr = c < a.nw ? c : a.nw - 1;          // idle lanes read a valid word
    const int nwf = s >> 2;                          // full words per sub-row

    // ---- per-group output state
    long long cg = 0;
    int cx = 0, cslot = 0;
    auto group_n = [&](long long g) -> int {
        int n = DECODE ? nout[g] : a.m;
        n -= chunk * RC;
        return n < 0 ? 0 : (n > RC ? RC : n);
    };
    long long g = tid;
    int n = group_n(g);

    uint32_t acc[RC][8];
#pragma unroll
    for (int j = 0; j < RC; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[j][r] = 0;

    {
        const int pre = nsteps < AH ? (int)nsteps : AH;
        for (int i = 0; i < pre; ++i) issue();
    }
    bool stored = false;
#pragma unroll 1
    for (long long st = 0; st < nsteps; ++st) {
        const bool steady = st + AH <= nsteps;       // AH - 1 younger blocks are in flight
        if (steady) {
            if (STAGE && stored) ring_wait_vmcnt<WAIT_STORED>();
            else if (!stored) ring_wait_vmcnt<WAIT_STEADY>();
            else ring_wait_vmcnt<0>();
        } else {
            ring_wait_vmcnt<0>();
        }
        stored = false;
        if (!STAGE && W > 1 && PROBE != 3) {
            // publish every wave's pieces of block st; proves block st - 1's slot is free
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        if (st + AH < nsteps) issue();               // into the slot of block st - 1

        if (n > 0) {
            const uint32_t* cw = (const uint32_t*)(coef + g * a.coef_gstride +
                                                   ((long long)chunk * k + cx) * RCP);
            uint32_t cwv[NCW];
#pragma unroll
            for (int q = 0; q < NCW; ++q) cwv[q] = __builtin_amdgcn_readfirstlane(cw[q]);
            const uintptr_t base = (uintptr_t)(in_ + g * a.in_gstride + (long long)cx * bb);
            // Sub-row t starts at a byte offset that is not 4-aligned in general
            // (s = 169, 1126, ...), and an unaligned ds_read_b32 replays at ~64 cycles: read
            // the two aligned dwords around the word (one ds_read2_b32) and realign them
            // with v_alignbyte_b32 (the misalignment is uniform per sub-row).
            const uint32_t blk = (uint32_t)(ring - smem) + cslot * a.slot_bytes +
                                 (uint32_t)(base & 15) + 4 * cr;
            WZ v;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t o = blk + t * s;
                const uint32_t* q = (const uint32_t*)(smem + (o & ~3u));
                if (PROBE == 2) v.W[t] = o ^ cwv[0];
                else v.W[t] = __builtin_amdgcn_alignbyte(q[1], q[0], o & 3u);
            }
            if (PROBE == 1 || PROBE == 2) {
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
            } else {
            expand_wz(v);
#pragma unroll
            for (int j = 0; j < RC; ++j) {
                if (j < n) {
                    if (!DECODE && j == 0 && chunk == 0) {
                        // encode row 0 is the all-ones row (P0 = XOR of the data,
                        // cauchy_256.cpp:1519-1523): no coefficient dispatch
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                        continue;
                    }
                    const uint32_t cf = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                    apply_nibble<0>(acc[j], cf & 15u, v);
                    apply_nibble<4>(acc[j], cf >> 4, v);
                }
            }
            }
        }
        if (++cslot == NS) cslot = 0;
        if (++cx == k) {
            // ---- group done: store its n output blocks
            if constexpr (STAGE) {
                // rows -> LDS staging (exact bytes), then SPO 8-byte stores per output
                if (n > 0) {
#pragma unroll
                    for (int j = 0; j < RC; ++j) {
                        if (j < n) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) {
                                uint8_t* d = stage + j * bb + r * s + 4 * c;
                                const uint32_t val = acc[j][r];
                                const uint32_t mis = (uint32_t)(d - smem) & 3u;   // uniform per row
                                if (c < nwf) {
                                    // unaligned ds_write_b32 replays; split by alignment
                                    if (mis == 0) {
                                        *(uint32_t*)d = val;
                                    } else if (mis == 2) {
                                        ((uint16_t*)d)[0] = (uint16_t)val;
                                        ((uint16_t*)d)[1] = (uint16_t)(val >> 16);
                                    } else {
                                        d[0] = (uint8_t)val;
                                        *(u16ua*)(d + 1) = (uint16_t)(val >> 8);
                                        d[3] = (uint8_t)(val >> 24);
                                    }
                                } else if (c == nwf) {
                                    if (s & 2) *(u16ua*)d = (uint16_t)val;
                                    if (s & 1) d[s & 2] = (uint8_t)(val >> (8 * (s & 2)));
                                }
                            }
                        }
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    const int o = chunk * RC + j;
                    int slot = o;
                    if (DECODE && j < n) slot = slots[g * a.rmax + o];
                    uint8_t* dst = out_ + g * a.out_gstride + (long long)slot * bb;
                    const __amdgpu_buffer_rsrc_t rs = ring_rsrc(dst, j < n ? (unsigned)bb : 0u);
#pragma unroll
                    for (int q = 0; q < SPO; ++q) {
                        const int off = (q * 64 + lane) * 8;
                        const int lo = off + 8 <= bb ? off : (bb >= 8 ? bb - 8 : 0);
                        const u32x2 val = *(const u32x2a4*)(stage + j * bb + lo);
                        __builtin_amdgcn_raw_buffer_store_b64(val, rs,
                                                              off + 8 <= bb ? (unsigned)off : kDrop,
                                                              0, 2);
                    }
                }
                stored = true;
            } else {
                if (n > 0) {
#pragma unroll
                    for (int j = 0; j < RC; ++j) {
                        if (j < n) {
                            const int o = chunk * RC + j;
                            const int slot = DECODE ? slots[g * a.rmax + o] : o;
                            uint8_t* dst = out_ + g * a.out_gstride + (long long)slot * bb;
#pragma unroll
                            for (int r = 0; r < 8; ++r) {
                                uint8_t* d = dst + r * s + 4 * c;
                                const uint32_t val = acc[j][r];
                                if (c < nwf) {
                                    __builtin_nontemporal_store(val, (u32ua*)d);
                                } else if (c == nwf) {
                                    if (s & 2) *(u16ua*)d = (uint16_t)val;
                                    if (s & 1) d[s & 2] = (uint8_t)(val >> (8 * (s & 2)));
                                }
                            }
                        }
                    }
                }
                stored = true;   // unknown store count: the next wait drains
            }
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[j][r] = 0;
            cx = 0;
            ++cg;
            if (cg < ng) {
                g = tid + cg * nt;
                n = group_n(g);
            }
        }
    }
}

// ------------------------------------------------------------------------- launcher
namespace {

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

int device_cus() {
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

template <int RC, int NS, int CNT, int TEAMS, int SPO, bool DECODE>
hipError_t ring_go(const RingArgs& a, size_t lds, unsigned threads, hipStream_t st) {
    auto kern = gf_ring_kernel<RC, NS, CNT, TEAMS, SPO, DECODE>;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)threads, lds) !=
            hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    const long long teams_per_wg = SPO > 0 ? TEAMS : 1;
    const long long want = (a.groups + teams_per_wg - 1) / teams_per_wg;
    const long long grid = std::min<long long>(want, (long long)device_cus() * per_cu);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(threads), lds, st, a.in, a.out, a.coef,
                       a.slots, a.nout, a);
    return hipGetLastError();
}

// Launch plan for one (k, bb, rc, nchunk) shape; `ok` is false when no instantiated
// variant covers it (the caller then uses gf_apply_kernel).
struct RingPlan {
    bool ok = false;
    bool staged = false;   // one-wave teams with LDS-staged outputs
    int ns = 8, teams = 1, spo = 0, cnt = 1;
    RingArgs a{};
    size_t lds = 0;
    unsigned threads = 0;
};

template <bool DECODE>
hipError_t ring_run(const RingPlan& p, int rc, bool dry, hipStream_t st) {
    // Instantiated variants.  Staged: (RC, NS, TEAMS, SPO) with CNT = 2 pieces per block.
#define QR_S(RCV, NSV, TV, SV)                                                             \
    if (p.staged && rc == RCV && p.ns == NSV && p.teams == TV && p.spo == SV)             \
        return dry ? hipSuccess : ring_go<RCV, NSV, 2, TV, SV, DECODE>(p.a, p.lds, p.threads, st);
    QR_S(2, 8, 2, 3) QR_S(4, 8, 2, 3) QR_S(8, 8, 2, 3)
    QR_S(2, 8, 4, 3) QR_S(4, 8, 4, 3) QR_S(8, 8, 4, 3)
    QR_S(4, 6, 4, 3) QR_S(4, 12, 2, 3) QR_S(4, 8, 1, 3) QR_S(4, 16, 1, 3) QR_S(4, 12, 1, 3)
    QR_S(2, 8, 2, 2) QR_S(4, 8, 2, 2) QR_S(8, 8, 2, 2)
#undef QR_S
    // Multi-wave teams: (RC, NS, CNT).
#define QR_M(RCV, NSV, CNTV)                                                               \
    if (!p.staged && rc == RCV && p.ns == NSV && p.cnt == CNTV)                            \
        return dry ? hipSuccess : ring_go<RCV, NSV, CNTV, 1, 0, DECODE>(p.a, p.lds, p.threads, st);
    QR_M(8, 8, 1) QR_M(8, 8, 2) QR_M(8, 12, 1) QR_M(8, 16, 1) QR_M(8, 4, 1) QR_M(8, 6, 1)
    QR_M(4, 8, 1) QR_M(4, 8, 2) QR_M(4, 16, 1) QR_M(4, 6, 2)
#undef QR_M
    return hipErrorInvalidValue;
}

RingPlan make_plan(int k, int m, int bb, int rc, int nchunk) {
    RingPlan p;
    if (!env_int("QFEC_RING", 0)) return p;   // opt-in: slower than gf_apply so far
    RingArgs& a = p.a;
    a.k = k; a.m = m; a.bb = bb; a.s = bb / 8;
    if (a.s < 4 || k < 1) return p;
    a.nw = (a.s + 3) / 4;
    a.ntiles = (a.nw + 63) / 64;
    a.nchunk = nchunk;
    a.nwaves = a.ntiles * nchunk;
    a.in_gstride = (long long)k * bb;
    const int units = (bb + 30) / 16;               // 16-byte window of any alignment
    const int np = (units + 63) / 64;
    if (a.ntiles == 1 && nchunk == 1 && np <= 2 && bb <= 1536) {
        p.staged = true;
        p.ns = env_int("QFEC_RING_NS", 8);
        p.teams = env_int("QFEC_RING_TEAMS", 2);
        p.spo = (bb + 511) / 512;
        p.cnt = 2;
        a.slot_bytes = units * 16;
        a.team_bytes = p.ns * a.slot_bytes + ((rc * bb + 4 + 15) / 16) * 16 + 16;
        p.lds = (size_t)p.teams * a.team_bytes;
        p.threads = (unsigned)p.teams * 64;
    } else {
        if (a.nwaves > 16) return p;
        p.ns = env_int("QFEC_RING_NS", 8);
        p.cnt = (np + a.nwaves - 1) / a.nwaves;
        a.slot_bytes = np * 1024;
        a.team_bytes = p.ns * a.slot_bytes + 16;
        p.lds = (size_t)a.team_bytes;
        p.threads = (unsigned)a.nwaves * 64;
    }
    if (p.lds > 160 * 1024) return p;
    p.ok = ring_run<false>(p, rc, true, nullptr) == hipSuccess;
    return p;
}

}  // namespace

bool gf_ring_supported(int k, int m, int bb, int rc, int nchunk) {
    return make_plan(k, m, bb, rc, nchunk).ok;
}

hipError_t launch_gf_ring(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                          const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                          long long groups, int rc, int nchunk, int rmax,
                          long long coef_gstride, long long out_gstride, bool decode,
                          hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    RingPlan p = make_plan(k, m, bb, rc, nchunk);
    if (!p.ok) return hipErrorInvalidValue;
    RingArgs& a = p.a;
    a.in = in; a.out = out; a.coef = coef; a.slots = slots; a.nout = nout;
    a.groups = groups;
    a.coef_gstride = coef_gstride;
    a.out_gstride = out_gstride;
    a.rmax = rmax;
    return decode ? ring_run<true>(p, rc, false, st) : ring_run<false>(p, rc, false, st);
}

}  // namespace qfec
