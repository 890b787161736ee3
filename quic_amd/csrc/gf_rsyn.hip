// gf_rsyn.hip — BASELINE configs B and C decode, (32 data + 4 parity) x 1352 B, on the static
// ring stream of the B/C encode (gf_ring_kernel, gf_stream.hip), in SLOT order.
//
// gf_bsyn streams a group's received blocks in row order, one block DMA per slot from wherever
// the slot lies (1 KiB + 336 B per block, each at its own address): that stream tops out near
// 4.8-5.2 TB/s.  The encode streams a group as contiguous 1 KiB pieces
// on a compile-time schedule (every wait an immediate) at 5.5 TB/s.  Here the decode streams the
// received group exactly like that and consumes it slot by slot, which needs the coefficient
// of slot i's ROW at compile time.  In the receive sets the receiver builds from packets in
// packet-number order (quic_fec_group.cc:259-274: the first k packets received, in arrival
// order), slot i holds the present data row i + e with e the number of erased rows below it,
// 0 <= e <= 4, or a parity row after the data.  So each slot dispatches (a binary tree of
// uniform branches) to one of the 5 compile-time coefficient sets C[y][i + e] for its row:
//   T_y = sum_{data slots i} C[y][row_i] D_i  ^  sum_{parity slots, row k + y} R_y
// which is the syndrome gf_bsyn forms, summed in another order (each received block enters
// with its own row's coefficient, cauchy_256.cpp:1269-1420; a repeated data row too).  Then
// E_j = sum_i Sinv[j][i] T_{y_i} (r^2 run-time products by nibble jumps, gf_winjump.h).
//
// The prep (decode_prep_bsyn_kernel) marks the groups this kernel takes (bsyn::kFast: every
// data slot's row lies in [i, i + 4]) and lists the other changed groups for gf_bsyn
// (shuffled arrival, repeated rows far from their slot).  A group not taken here is streamed
// from an empty buffer range (no HBM traffic), so the static schedule stays intact.
//
// Row 0 of the code is all ones (the XOR parity, cauchy_256.cpp:1519-1523): its syndrome
// takes every data block as is, outside the dispatch.
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

namespace {

constexpr int kRsynWaves = 4;
constexpr unsigned kRsDrop = 0x80000000u;   // buffer offset past any range: lane dropped

template <int N>
__device__ __forceinline__ void rs_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16 bytes per lane from buffer rs at voff + soff into LDS at lds + 16 * lane (nt); lanes past
// the range read zeros.  (Device only: in a lambda the builtin would void the host stub.)
__device__ __forceinline__ void rs_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds, uint32_t voff,
                                         int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 2);
#else
    (void)rs, (void)lds, (void)voff, (void)soff;
#endif
}

// a dword of a table the kernel never writes, through the scalar cache
__device__ __forceinline__ uint32_t rs_cload_u32(const void* base, long long byte_off) {
    return ((const __attribute__((address_space(4))) uint32_t*)(base))[byte_off >> 2];
}

// f(integral_constant<int, v>) for the run-time v in [LO, HI]: a tree of uniform branches
template <int LO, int HI, class F>
__device__ __forceinline__ void rs_dispatch(int v, F&& f) {
    if constexpr (LO == HI) {
        f(std::integral_constant<int, LO>{});
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (v <= MID) rs_dispatch<LO, MID>(v, f);
        else rs_dispatch<MID + 1, HI>(v, f);
    }
}

template <int S>
struct RsynShape {
    static constexpr int R = 8, RB = R * 1024;   // ring: 8 one-KiB pieces per wave
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4, NWF = S / 4;
    static constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);   // stores per sub-row
    static constexpr int pf(int x) { return (x * BB) >> 10; }             // first piece of slot x
    static constexpr int pl(int x) { return ((x + 1) * BB - 1) >> 10; }   // its last piece
};

// K, MC: the compiled code; S: sub-row bytes.  At most RC = 4 recovered blocks per group.
// The piece schedule is gf_ring_run's (gf_stream.hip): before slot x's compute the ring holds
// every piece from slot x's first one on and is filled up to pf(x) + R - 1 (the next group's
// first pieces included); every group issues NST stores (outputs past n: empty range), so
// every wait is an immediate.
template <int K, int MC, int S>
__global__ __launch_bounds__(kRsynWaves * 64) void gf_rsyn_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int rmax, long long out_gstride) {
    using SH = RsynShape<S>;
    constexpr int R = SH::R, RB = SH::RB, BB = SH::BB, NW = SH::NW, NWF = SH::NWF;
    constexpr int GB = K * BB;
    constexpr int NP = (GB + 1023) / 1024;
    constexpr int E = bsyn::kRsynE;
    constexpr int RC = 4;
    constexpr int NST = RC * 8 * SH::SPR;
    constexpr int FM1 = SH::pf(K - 1) + R - 1 - NP;    // next-group pieces issued early
    static_assert(GB % 16 == 0, "16-byte aligned groups (even k at 1352-byte blocks)");
    static_assert(FM1 >= SH::pl(0), "block 0 of the next group is prefetched in full");
    static_assert(SH::pf(K - 1) + R - 1 < 2 * NP, "the frontier stays within the next group");
    static_assert(K <= 64 && MC <= 8 && RC <= MC && K % 4 == 0, "compiled small-block code");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    uint8_t* ring = smem + (size_t)w * RB;
    const long long W = (long long)gridDim.x * kRsynWaves;
    const long long g0 = (long long)blockIdx.x * kRsynWaves + w;
    if (g0 >= groups) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));
    const int c = lane < NW ? lane : NW - 1;           // idle lanes shadow the last word
    const uint32_t v16 = 16u * (uint32_t)lane;

    // the current and the next group's buffer resources: range GB when gf_rsyn decodes the
    // group, 0 otherwise (its pieces read as zeros, no traffic), and 0 past the last group
    auto group_rsrc = [&](long long gi) __attribute__((always_inline)) {
        const bool inside = gi < cnt;
        const long long g = inside ? g0 + gi * W : g0;   // no table load past the last group
        const bool live = (rs_cload_u32(tab + g * (long long)bsyn::kBytes, bsyn::kFast) != 0) && inside;
        return __builtin_amdgcn_make_buffer_rsrc((void*)(in + g * (long long)GB), 0,
                                                 live ? (unsigned)GB : 0u, 0x00020000);
    };
    __amdgpu_buffer_rsrc_t rs_cur = group_rsrc(0), rs_next = group_rsrc(1);
    int phase = 0;                                     // ring slot of the group's piece 0

    // piece n of the current group (n >= NP: piece n - NP of the next)
    auto issue = [&](auto nc) __attribute__((always_inline)) {
        constexpr int n = decltype(nc)::value;
        uint8_t* dst = ring + ((phase + n) & (R - 1)) * 1024;
        if constexpr (n < NP) rs_dma16(rs_cur, dst, v16, n * 1024);
        else rs_dma16(rs_next, dst, v16, (n - NP) * 1024);
    };
    // slot x at ring byte (phase * 1024 + x * BB) mod RB (a slot that wraps round the ring end
    // is read with per-lane wrapped addresses)
    auto read_block = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8]) __attribute__((always_inline)) {
        constexpr int x = decltype(xc)::value;
        uint32_t c4 = 4u * (uint32_t)c;
        asm volatile("" : "+v"(c4));   // opaque: addresses are not hoisted across blocks
        const uint32_t bp = ((uint32_t)phase * 1024u + (uint32_t)(x * BB)) & (uint32_t)(RB - 1);
        if (bp + (uint32_t)BB + 4u <= (uint32_t)RB) {
            const uint8_t* L = ring + bp + c4;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                const uint32_t* q = (const uint32_t*)(L + (o & ~3));
                lo[t] = q[0];
                hi[t] = (o & 3) ? q[1] : 0u;
            }
        } else {
            const uint32_t base = bp + c4;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                const uint32_t a0 = base + (uint32_t)(o & ~3);
                lo[t] = *(const uint32_t*)(ring + min(a0, a0 - (uint32_t)RB));
                if (o & 3) {
                    const uint32_t a1 = a0 + 4u;
                    hi[t] = *(const uint32_t*)(ring + min(a1, a1 - (uint32_t)RB));
                } else {
                    hi[t] = 0u;
                }
            }
        }
    };

    // ---- prologue: the first group's early pieces, then the stores a previous group would
    // have issued (empty range), so every group sees the same VMEM history
    static_for<FM1 + 1>([&](auto nc) __attribute__((always_inline)) { issue(nc); });
    asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
    {
        const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
        for (int q = 0; q < NST; ++q)   // distinct offsets: not merged as duplicate stores
            __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
    }

    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = g0 + (long long)i * W;
        const uint8_t* tb = tab + g * (long long)bsyn::kBytes;
        const bool fast = rs_cload_u32(tb, bsyn::kFast) != 0;
        int n = fast ? (int)rs_cload_u32(nout, 4 * g) : 0;
        n = n > rmax ? rmax : n;
        n = n > RC ? RC : n;
        uint32_t rw[K / 4];                            // the slots' row tags
#pragma unroll
        for (int q = 0; q < K / 4; ++q) rw[q] = rs_cload_u32(tb, bsyn::kRows + 4 * q);
        uint32_t acc[MC][8];
#pragma unroll
        for (int y = 0; y < MC; ++y)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[y][r] = 0;
        // slot 0: its pieces were issued before the previous group's stores
        rs_wait_vmcnt<(FM1 - SH::pl(0) + NST > 63 ? 63 : FM1 - SH::pl(0) + NST)>();
        read_block(std::integral_constant<int, 0>{}, lo0, hi0);

        auto step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                        uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            constexpr int F0 = x == 0 ? FM1 : SH::pf(x - 1) + R - 1;   // frontier before
            constexpr int F1 = SH::pf(x) + R - 1;                       // and after this step
            static_for<F1 - F0>([&](auto qc) __attribute__((always_inline)) {
                issue(std::integral_constant<int, F0 + 1 + decltype(qc)::value>{});
            });
            if constexpr (x + 1 < K) {
                constexpr int pl1 = SH::pl(x + 1);
                constexpr int yng = F1 - pl1 + (pl1 <= FM1 ? NST : 0);
                rs_wait_vmcnt<(yng > 63 ? 63 : yng)>();
                read_block(std::integral_constant<int, x + 1>{}, nlo, nhi);
            }
            if (n <= 0) return;   // nothing to recover here (or not this kernel's group)
            uint32_t wv[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                wv[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
            const int row = (int)((rw[x / 4] >> (8 * (x % 4))) & 0xFFu);
            if (row >= K) {
                // a parity block: T_{row - K} ^= it (the prep checked row < K + MC)
                const int y = row - K;
                static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                    constexpr int yy = decltype(yc)::value;
                    if (y == yy) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[yy][r] ^= wv[r];
                    }
                });
            } else {
                // a data block of row x + e, 0 <= e <= E (the prep's kFast test)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[0][r] ^= wv[r];   // row 0: all ones
                Win win;
                win_build(wv, win);
                rs_dispatch<0, E>(row - x, [&](auto ec) __attribute__((always_inline)) {
                    constexpr int xr = x + decltype(ec)::value;
                    if constexpr (xr < K) {
                        asm volatile("");
                        static_for<MC - 1>([&](auto yc) __attribute__((always_inline)) {
                            constexpr int y = decltype(yc)::value + 1;
                            win_apply<cauchy_coef(MC, y, xr)>(acc[y], win);
                        });
                    }
                });
            }
        };
        static_for<K>([&](auto xc) __attribute__((always_inline)) {
            // accumulators opaque at every block boundary (no cross-block XOR reassociation)
#pragma unroll
            for (int y = 0; y < MC; ++y)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[y][r]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(xc)::value % 2 == 0) step(xc, lo0, hi0, lo1, hi1);
            else step(xc, lo1, hi1, lo0, hi0);
        });

        // ---- E_j = sum_i Sinv[j][i] T_{y_i}; RC x 8 x SPR store instructions whatever n is
        // (outputs past n: empty range), kept after the last step's DMAs and before the next
        // group's (issue order)
        asm volatile("" ::: "memory");
        const uint32_t ymap = rs_cload_u32(tb, bsyn::kY);
        uint32_t vo = lane < NWF ? 4u * (uint32_t)lane : kRsDrop;
        uint32_t vt = (lane == NWF && NWF < NW) ? 4u * (uint32_t)lane : kRsDrop;
        asm volatile("" : "+v"(vo), "+v"(vt));
#pragma unroll 1
        for (int j = 0; j < RC; ++j) {
            const bool on = j < n;
            uint32_t o[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) o[r] = 0;
            if (on) {
                const uint32_t sw = rs_cload_u32(tb, bsyn::kSinv + 4 * j);   // Sinv[j][0..3]
#pragma unroll 1
                for (int ii = 0; ii < n; ++ii) {
                    const int y = (int)((ymap >> (8 * ii)) & 0xFFu);
                    WZ v;
                    static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int yy = decltype(yc)::value;
                        if (y == yy) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) v.W[r] = acc[yy][r];
                        }
                    });
                    expand_wz(v);
                    wz_mul_acc_rt(o, v, (sw >> (8 * ii)) & 0xFFu);
                }
            }
            const long long sj = g * rmax + j;
            const int oslot = (slots && on) ? (int)((rs_cload_u32(slots, sj & ~3LL) >> (8 * (sj & 3))) & 0xFFu)
                                            : j;
            uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(dst, 0, on ? (unsigned)BB : 0u, 0x00020000);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                __builtin_amdgcn_raw_buffer_store_b32(o[r], rs, vo, r * S, 2);
                if (S & 2) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)o[r], rs, vt, r * S, 2);
                if (S & 1)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(o[r] >> (8 * (S & 2))), rs, vt,
                                                         r * S + (S & 2), 2);
            }
        }
        asm volatile("" ::: "memory");
        rs_cur = rs_next;
        rs_next = group_rsrc(i + 2);
        phase = (phase + NP) & (R - 1);
    }
    rs_wait_vmcnt<0>();
}

constexpr int kRsynS = 169;   // bb = 1352: 1350-byte payloads (BASELINE configs B, C)

}  // namespace

hipError_t launch_gf_rsyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                          long long groups, int rmax, long long out_gstride, hipStream_t st,
                          const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_bsyn_supported(k, m, bb, rmax, t)) return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)slots | (uintptr_t)nout) & 3))
        return hipErrorInvalidValue;
    using SH = RsynShape<kRsynS>;
    const size_t lds = (size_t)kRsynWaves * SH::RB;
    const long long want = (groups + kRsynWaves - 1) / kRsynWaves;
    long long cap = (long long)t.cus * (long long)((160 * 1024) / lds);
    if (t.stream_grid > 0) cap = t.stream_grid;          // tests: many groups per wave
    const unsigned grid = (unsigned)std::min<long long>(want, cap);
    if ((groups + (long long)grid * kRsynWaves - 1) / ((long long)grid * kRsynWaves) >= (1LL << 31))
        return hipErrorInvalidValue;
    note_kernel("gf_rsyn_kernel<decode,k32m4>");
    note_grid("gf_rsyn_kernel", grid);
    qlaunch((gf_rsyn_kernel<32, 4, kRsynS>), dim3(grid), dim3(kRsynWaves * 64), lds, st, in, out,
            tab, slots, nout, groups, rmax, out_gstride);
    return hipGetLastError();
}

}  // namespace qfec
