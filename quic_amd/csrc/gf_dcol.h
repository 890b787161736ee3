// gf_dcol.hip — BASELINE config D, (128 data + 16 parity) x 9008 B blocks (9000 B payloads,
// quic_fec_group.cc:344-352): encode and syndrome decode of the compiled (128, 16) code with
// ONE wave per column tile computing ALL 16 rows.
//
// Arithmetic: the bit-sliced Cauchy code of cauchy_256.cpp:90-125 in the windowed form of
// gf_bitslice.h with compile-time coefficients (cauchy_const.h, cauchy_256.cpp:422-480):
// per block a lane builds the 2 x 15 XOR combinations of its column word's 4-sub-row
// halves (22 VALU) and then every (row, sub-row) is one v_bitop3, 128 per block.
//
// Why this shape.  The D kernels are bound by VALU issue: the instruction
// count per block and the cycles each VALU instruction costs at the kernel's occupancy
// (tools/microbench/valu_rate.hip, profiles/r04/valu_rate.txt: 4.6 shader cycles per VALU per
// SIMD at two waves per SIMD, 3.3 at four, 2.7 at eight).  gf_tile split the 16 rows over two waves per column
// tile, which builds every block's window twice (2 x 97 VALU per tile and block against
// ~157 here) and needs a workgroup barrier per block pair and, in the decode, an 80 KB LDS
// exchange of the syndromes.  Here a wave holds all 128 accumulators (about 190 VGPRs,
// two waves per SIMD), so:
//   - every window is built once;
//   - the decode's syndromes of all 16 parity rows sit in one wave: the r x r solve needs
//     no exchange, and no per-(row, block) "is this row needed" branch (gf_tile_syn's);
//   - the waves are independent: each streams its own column segments of every block
//     (8 sub-row envelopes of 256 B, two buffer_load_dwordx4 ... lds per block) into a
//     private LDS ring, with no barriers.
//
// Units.  A group is NT = 5 column tiles of 60 words (the last one 42 words); a unit is one
// (group, tile).  Wave lw owns units lw, lw + W, lw + 2W, ... (W = waves in the grid), with
// an XCD-aware workgroup order so the tiles of one group run on one XCD (their 16-byte
// alignment envelopes overlap by a few bytes: L2 hits).
//
// Decode (cauchy_256.cpp:1269-1420): the k received blocks are streamed by DATA ROW: row x's
// block (from the slot the prep table names) at position x, an erased row as a zero block
// (a DMA from an empty buffer range, no HBM traffic), so position x's coefficients stay
// compile-time and the block pass is the encode's.  Its 16 accumulators are then
// P'_y = sum_{present x} C[y][x] D_x; the extras follow (received parity blocks: T_y =
// P'_y ^ R_y; a repeated data row adds C[y][row] times its block, run-time coefficients);
// finally E_j = sum_i Sinv[j][i] T_{y_i} with run-time coefficients (nibble dispatch), r^2
// applies per group against 128 block steps.
//
// vmcnt bookkeeping: a block is NDMA = 2 DMA instructions, issued D blocks ahead; waiting
// for block b + 1 leaves (D - 1) * NDMA younger.  A unit ends with at least NSTMIN stores
// (every store instruction is issued, lanes and rows without output dropped; the first unit
// finds NSTMIN empty stores from the prologue), so the waits for a unit's blocks 1 .. D - 1,
// which were issued before those stores, use vmcnt(63): (D - 1) * NDMA + NSTMIN >= 63
// younger instructions.  tests/test_isa.py checks
// that the compiler adds no VMEM instruction or vmcnt wait of its own.
#pragma once
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

namespace {

#define QD_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void dc_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16 bytes per lane from buffer rs at voff into LDS at lds + 16 * lane (nt).  Lanes whose
// offset lies past the buffer's range load zeros.  (Device only: in a lambda the builtin
// would void the kernel's host stub.)
template <int AUX>
__device__ __forceinline__ void dc_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QD_LPTR(lds), 16, voff, 0, 0, AUX);
#else
    (void)rs, (void)lds, (void)voff;
#endif
}

// a wave-uniform value made opaque to the optimiser (device only, as above)
__device__ __forceinline__ void dc_opaque_v(uint32_t& x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#else
    (void)x;
#endif
}

// the lane id, recomputed where it is used (not kept live across the block loop)
__device__ __forceinline__ int dc_lane_here() {
    int l = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
#endif
    return l;
}

// byte i / dword at byte offset o of a table the kernel never writes, through the scalar
// cache (constant address space)
__device__ __forceinline__ uint32_t dc_cload_u32(const uint8_t* base, long long o) {
    return ((const __attribute__((address_space(4))) uint32_t*)(base))[o >> 2];
}
__device__ __forceinline__ int dc_cload_u8(const uint8_t* base, long long i) {
    return (int)((dc_cload_u32(base, i & ~3LL) >> (8 * (i & 3))) & 0xFFu);
}

constexpr unsigned kDDrop = 0x80000000u;   // buffer offset past any range: lane dropped
constexpr int kDcWaves = 4;                // waves per workgroup (independent)

template <int S>
struct DcShape {
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4;            // column words per sub-row
    static constexpr int NWF = S / 4;                 // full words
    // a tile is TW = 60 column words (240 bytes, a multiple of 16), so the 16-byte aligned
    // envelope of its part of a sub-row ((t * S) % 16 <= 14 bytes of skew, the words, and
    // the dword after the last word for the realignment) is exactly 256 bytes: 16 lanes of
    // one buffer_load_dwordx4 ... lds, a block is two such instructions (2 KiB of LDS), with
    // no partial instruction.  Lanes 60..63 idle (the tile count per group is 5 either way)
    static constexpr int TW = 60;
    static constexpr int NT = (NW + TW - 1) / TW;     // column tiles
    static constexpr int TAILW = NW - TW * (NT - 1);  // words of the last tile
    static constexpr int SEGL = 16, SEGB = 16 * SEGL;
    static constexpr int TAILL = (14 + 4 * TAILW + 2 + 15) / 16;   // lanes, last tile
    static constexpr int BUFB = 8 * SEGB;                           // LDS bytes per block
    static constexpr int NDMA = 8 * SEGL / 64;                      // DMA instructions / block
    static_assert(S % 2 == 0 && BB % 16 == 0 && TAILL <= SEGL && 14 + 4 * TW + 2 <= SEGB &&
                  NDMA * 64 == 8 * SEGL, "shape");
};

// CACHE: bit 0 = the DMA loads are plain (cached) instead of non-temporal, bit 1 = the
// stores are plain instead of non-temporal.  Neighbouring tiles' 256-byte envelopes share
// cache lines, which a non-temporal load evicts first.
// About 190 VGPRs: two waves per SIMD.  Block b + 1 is read from LDS into registers while
// block b is combined (prefetch).
template <int S, int D, bool DECODE, int CACHE>
__global__ __launch_bounds__(kDcWaves * 64, 2) void gf_dcol_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout,
    const uint8_t* __restrict__ cenc, long long groups, int rmax, long long in_bytes,
    long long tab_gstride, long long out_gstride) {
    using SH = DcShape<S>;
    constexpr int KC = 128, MC = 16;
    constexpr int RW = MC;                           // parity rows per wave: all of them
    constexpr int BB = SH::BB, NW = SH::NW, NWF = SH::NWF, NT = SH::NT;
    constexpr int SEGL = SH::SEGL, SEGB = SH::SEGB, TAILL = SH::TAILL, BUFB = SH::BUFB;
    constexpr int NDMA = SH::NDMA;
    constexpr int NBUF = D + 1;                      // D in flight + the one being read
    constexpr int WAITN = (D - 1) * NDMA;            // younger than the awaited block b + 1
    constexpr int NSTMIN = 64 - WAITN;               // stores a unit ends with, at least
    static_assert(WAITN + NSTMIN >= 63 && WAITN <= 63 && D >= 2 && KC % 4 == 0 && D <= KC / 2,
                  "pipeline");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int wv = wave_id();
    uint8_t* ring = smem + (size_t)wv * NBUF * BUFB;
    // XCD-aware workgroup order: hardware workgroup b runs on XCD b % 8; logical workgroups
    // of one XCD are consecutive, so a group's tiles share an L2
    const unsigned nwg = gridDim.x, hb = blockIdx.x;
    const unsigned xcd = hb & 7u, q8 = nwg >> 3, r8 = nwg & 7u;
    const unsigned lwg = xcd * q8 + min(xcd, r8) + (hb >> 3);
    const long long W = (long long)nwg * kDcWaves;
    const long long u0 = (long long)lwg * kDcWaves + wv;
    const long long NU = groups * NT;
    if (u0 >= NU) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((NU - 1 - u0) / W + 1));

    // ---- issue side.  The DMA stream runs exactly D blocks ahead of the compute side, so
    // while unit i is combined the stream is in unit i (positions D ..) or, for the last D
    // blocks, in unit i + 1: both units' stream state is kept.  A unit past the last one
    // streams empty-range DMAs (zeros, no traffic).
    struct Unit {
        const uint8_t* src;   // the group's first block
        const uint8_t* tb;    // its syndrome table (decode)
        int room;             // bytes from src to the end of the input (capped)
        int len;              // stream positions: KC rows (+ extras, decode)
        bool none;            // past the last unit
    };
    // per-lane DMA offsets of a unit's tile p: lane gl = 64 q + L of the block's 8 * SEGL
    // lanes is lane j of segment t = gl / SEGL (an unused lane: empty-range offset)
    static_assert(NDMA == 2, "two DMA instructions per block (named offset registers)");
    auto tile_voff = [&](int p, uint32_t& v0, uint32_t& v1) __attribute__((always_inline)) {
        const int segl = p == NT - 1 ? TAILL : SEGL;
        const int t = lane / SEGL, j = lane - t * SEGL;   // instruction 1: segment t + 4
        const uint32_t base = (uint32_t)(4 * SH::TW * p + 16 * j);
        v0 = j < segl ? (uint32_t)((t * S) & ~15) + base : kDDrop;
        v1 = j < segl ? (uint32_t)(((t + 4) * S) & ~15) + base : kDDrop;
    };
    auto make_unit = [&](int i, Unit& un, uint32_t& v0, uint32_t& v1) __attribute__((always_inline)) {
        un.none = i >= cnt;
        const long long u = un.none ? u0 : u0 + (long long)i * W;   // (group, tile)
        const long long g = u / NT;
        const int p = (int)(u - g * NT);
        un.src = in + g * (long long)KC * BB;
        un.tb = DECODE ? tab + g * tab_gstride : tab;
        un.room = (int)min(in_bytes - g * (long long)KC * BB, (long long)KC * BB + 16);
        un.len = KC;
        if constexpr (DECODE)
            if (!un.none) un.len = KC + (int)(dc_cload_u32(un.tb, syn::kNExt) & 0xFFu);
        tile_voff(p, v0, v1);
    };
    Unit cu, nu;                                     // the unit combined now, and the next
    uint32_t vc0, vc1, vn0, vn1;                     // their DMA lane offsets
    int iss_off = 0;                                 // LDS ring offset of the next DMA
    // one block: the DMA of the block at byte offset boff of unit un into the next ring
    // buffer (zero: an erased row, or past the last unit)
    auto dma_block = [&](const Unit& un, uint32_t v0, uint32_t v1, int boff, bool zero)
                         __attribute__((always_inline)) {
        const bool z = zero || un.none;
        const unsigned nrec = z ? 0u : (unsigned)min(un.room - boff, BB + 16);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(un.src + boff), 0, nrec, 0x00020000);
        uint8_t* dst = ring + iss_off;
        constexpr int LAUX = (CACHE & 1) ? 0 : 2;
        dc_dma16<LAUX>(rs, dst, v0);
        dc_dma16<LAUX>(rs, dst + 1024, v1);
        iss_off += BUFB;
        if (iss_off == NBUF * BUFB) iss_off = 0;
    };
    // decode: the slot of data row x comes from the table, 4 rows per scalar load, loaded
    // one word ahead (rw: rows x .. x + 3 once x % 4 == 0, rn: the next four)
    uint32_t rw_c = 0, rn_c = 0, rw_n = 0, rn_n = 0;
    // data row x of unit un (x compile-time)
    auto issue_row = [&](auto xc, const Unit& un, uint32_t v0, uint32_t v1, uint32_t& rw,
                         uint32_t& rn) __attribute__((always_inline)) {
        constexpr int x = decltype(xc)::value;
        if constexpr (DECODE) {
            if constexpr (x % 4 == 0) {
                rw = rn;
                if constexpr (x + 4 < KC) rn = dc_cload_u32(un.tb, syn::kRowSlot + x + 4);
            }
            const int slot = (int)((rw >> (8 * (x % 4))) & 0xFFu);
            dma_block(un, v0, v1, min(slot, KC - 1) * BB, slot >= KC);
        } else {
            dma_block(un, v0, v1, x * BB, false);
        }
    };
    // first word of a unit's row slots (before its row 0 is issued: rn = rows 0..3)
    auto rows_start = [&](const Unit& un, uint32_t& rn) __attribute__((always_inline)) {
        if constexpr (DECODE) rn = un.none ? 0u : dc_cload_u32(un.tb, syn::kRowSlot);
    };
    // extra e of unit un (decode, run time)
    auto issue_extra = [&](int e, const Unit& un, uint32_t v0, uint32_t v1)
                           __attribute__((always_inline)) {
        // extras follow the present rows in the stream order: kPerm[np + e], np = KC - ne
        const int slot = dc_cload_u8(un.tb, syn::kPerm + e + 2 * KC - un.len);
        dma_block(un, v0, v1, min(slot, KC - 1) * BB, false);
    };
    // run-time stream position q of the current unit (q >= KC): an extra, or the next unit's
    // row q - len (< D: the rows issued before the next unit starts)
    auto issue_tail = [&](int q) __attribute__((always_inline)) {
        if (q < cu.len) {
            issue_extra(q - KC, cu, vc0, vc1);
        } else {
            const int x = q - cu.len;
            static_for<D>([&](auto xc) __attribute__((always_inline)) {
                if (x == decltype(xc)::value) issue_row(xc, nu, vn0, vn1, rw_n, rn_n);
            });
        }
    };

    // ---- read side: column word c of the 8 sub-rows of the block at ring offset rd_off
    // (segment t at SEGB * t, the word at its skew (t * S) % 16 + 4c; odd sub-rows are 2
    // bytes off a dword: two aligned dwords, realigned at use)
    int rd_off = 0;
    auto read_block = [&](uint32_t (&lo)[8], uint32_t (&hi)[8]) __attribute__((always_inline)) {
        uint32_t c4 = 4u * (uint32_t)lane + (uint32_t)rd_off;
        dc_opaque_v(c4);   // no hoisting across blocks
        const uint8_t* L = ring + c4;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = SEGB * t + ((t * S) & 15);
            const uint32_t* qp = (const uint32_t*)(L + (o & ~3));
            lo[t] = qp[0];
            hi[t] = (o & 3) ? qp[1] : 0u;
        }
    };
    auto realign = [&](const uint32_t (&lo)[8], const uint32_t (&hi)[8], uint32_t (&w8)[8])
                       __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = (t * S) & 15;
            w8[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
        }
    };
    // wait for block b + 1 and read it into (nlo, nhi); `early` (compile time): it was issued
    // before the previous unit's stores
    auto next_block = [&](auto early, uint32_t (&nlo)[8], uint32_t (&nhi)[8])
                          __attribute__((always_inline)) {
        if constexpr (decltype(early)::value) dc_wait_vmcnt<63>();
        else dc_wait_vmcnt<WAITN>();
        rd_off += BUFB;
        if (rd_off == NBUF * BUFB) rd_off = 0;
        read_block(nlo, nhi);
    };

    // ---- prologue: unit 0's first D rows, then the stores a previous unit would have issued
    // (empty range), so every unit's blocks 1 .. D - 1 have at least NSTMIN stores younger
    make_unit(0, cu, vc0, vc1);
    rows_start(cu, rn_c);
    static_for<D>([&](auto xc) __attribute__((always_inline)) { issue_row(xc, cu, vc0, vc1, rw_c, rn_c); });
    asm volatile("" ::: "memory");
    {
        const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
        for (int q = 0; q < NSTMIN; ++q)   // distinct offsets: not merged as duplicate stores
            __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
    }
    asm volatile("" ::: "memory");
    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
    dc_wait_vmcnt<WAITN>();
    read_block(lo0, hi0);

#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long u = u0 + (long long)i * W;
        const long long g = u / NT;
        const int p = (int)(u - g * NT);
        const uint8_t* tb = tab + (DECODE ? g * tab_gstride : 0);
        make_unit(i + 1, nu, vn0, vn1);
        rows_start(nu, rn_n);
        // decode: the syndrome rows the solve uses (the received parity rows, syn::kNeed) and
        // the present data rows (syn::kMask); rows outside them are skipped by uniform
        // branches (cauchy_256.cpp:712-795: only received recovery rows enter the system)
        uint32_t need = 0xFFFFu, pm0 = ~0u, pm1 = ~0u, pm2 = ~0u, pm3 = ~0u;
        if constexpr (DECODE) {
            need = dc_cload_u32(tb, syn::kNeed);
            pm0 = dc_cload_u32(tb, syn::kMask);
            pm1 = dc_cload_u32(tb, syn::kMask + 4);
            pm2 = dc_cload_u32(tb, syn::kMask + 8);
            pm3 = dc_cload_u32(tb, syn::kMask + 12);
        }
        uint32_t acc[RW][8];
#pragma unroll
        for (int y = 0; y < RW; ++y)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[y][r] = 0;

        // data row x (compile time): issue stream position x + D, read block x + 1, and
        // every row's windowed apply of block x
        auto step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                        uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            if constexpr (x + D < KC) {
                issue_row(std::integral_constant<int, x + D>{}, cu, vc0, vc1, rw_c, rn_c);
            } else if constexpr (!DECODE) {
                issue_row(std::integral_constant<int, x + D - KC>{}, nu, vn0, vn1, rw_n, rn_n);
            } else {
                issue_tail(x + D);
            }
            uint32_t w8[8];
            next_block(std::bool_constant<(x + 1 <= D - 1)>{}, nlo, nhi);
            if constexpr (DECODE) {
                // an erased row's zero block adds nothing; a row the solve does not use is
                // not accumulated (the empty asm keeps each branch a branch: no select)
                const uint32_t pw = x < 32 ? pm0 : x < 64 ? pm1 : x < 96 ? pm2 : pm3;
                if (__builtin_expect((pw >> (x % 32)) & 1u, 1)) {
                    realign(lo, hi, w8);
                    Win win;
                    win_build(w8, win);
                    static_for<RW>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int y = decltype(yc)::value;
#ifndef QFEC_DCOL_ROWSKIP
#define QFEC_DCOL_ROWSKIP 1
#endif
                        if (!QFEC_DCOL_ROWSKIP || __builtin_expect((need >> y) & 1u, 1)) {
                            asm volatile("");
                            win_apply<cauchy_coef(MC, y, x)>(acc[y], win);
                        }
                    });
                }
            } else {
                realign(lo, hi, w8);
                Win win;
                win_build(w8, win);
                static_for<RW>([&](auto yc) __attribute__((always_inline)) {
                    constexpr int y = decltype(yc)::value;
                    win_apply<cauchy_coef(MC, y, x)>(acc[y], win);
                });
            }
        };
        static_for<KC>([&](auto xc) __attribute__((always_inline)) {
            // accumulators opaque at every block boundary: with constant coefficients the XOR
            // reassociation would otherwise merge the blocks' sums and keep every block's
            // window live; and nothing is scheduled across blocks (register pressure)
#pragma unroll
            for (int y = 0; y < RW; ++y)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[y][r]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(xc)::value % 2 == 0) step(xc, lo0, hi0, lo1, hi1);
            else step(xc, lo1, hi1, lo0, hi0);
        });

        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
        const int lane_e = dc_lane_here();
        const int wcol = SH::TW * p + lane_e;          // this lane's column word
        const bool mine = lane_e < SH::TW;
        uint32_t vo = mine && wcol < NWF ? 4u * (uint32_t)wcol : kDDrop;
        uint32_t vt = (mine && wcol == NWF && NWF < NW) ? 4u * (uint32_t)wcol : kDDrop;
        dc_opaque_v(vo);
        dc_opaque_v(vt);
        // one output block: 8 sub-row dword stores, plus the tail word's 16-bit store in the
        // last tile (S % 4 == 2)
        static_assert(S % 4 == 2, "the tail word of a sub-row holds 2 bytes");
        constexpr int SAUX = (CACHE & 2) ? 0 : 2;
        auto store_out = [&](uint8_t* dst, bool on, const uint32_t (&o)[8])
                             __attribute__((always_inline)) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(dst, 0, on ? (unsigned)BB : 0u, 0x00020000);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(o[r], rs, vo, r * S, SAUX);
            if (p == NT - 1) {
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)o[r], rs, vt, r * S, SAUX);
            }
        };

        if constexpr (!DECODE) {
            static_assert(RW * 8 >= NSTMIN, "store count");
#pragma unroll
            for (int y = 0; y < RW; ++y)
                store_out(out + g * out_gstride + (long long)y * BB, true, acc[y]);
        } else {
            const int ne = cu.len - KC;
            const int n = min((int)dc_cload_u32((const uint8_t*)nout, 4 * g), rmax);
            // extras: a received parity row y adds its block to T_y; a repeated data row adds
            // C[y][row] times its block to every row (run-time coefficients, cenc = [m][k])
            auto extra = [&](int e, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                             uint32_t (&nhi)[8]) __attribute__((always_inline)) {
                issue_tail(KC + e + D);
                WZ v;
                next_block(std::false_type{}, nlo, nhi);
                realign(lo, hi, v.W8);
                const int row = dc_cload_u8(tb, syn::kERow + e);
                if (row >= KC) {
                    const int y = row - KC;
                    static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int yy = decltype(yc)::value;
                        if (y == yy) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) acc[yy][r] ^= v.W[r];
                        }
                    });
                } else {
                    expand_wz(v);
                    static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int yy = decltype(yc)::value;
                        if ((need >> yy) & 1u) {
                            const uint32_t cf = (uint32_t)dc_cload_u8(cenc, yy * KC + row);
                            apply_nibble<0>(acc[yy], cf & 15u, v);
                            apply_nibble<4>(acc[yy], cf >> 4, v);
                        }
                    });
                }
            };
#pragma unroll 1
            for (int e = 0; e + 1 < ne; e += 2) {
                extra(e, lo0, hi0, lo1, hi1);
                extra(e + 1, lo1, hi1, lo0, hi0);
            }
            if (ne & 1) {
                extra(ne - 1, lo0, hi0, lo1, hi1);
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    lo0[t] = lo1[t];
                    hi0[t] = hi1[t];
                }
            }
            // E_j = sum_i Sinv[j][i] T_{y_i}, in passes of 4 outputs; every pass issues its
            // 4 x 8 dword stores (outputs past n: empty range), padded to NSTMIN per unit
            asm volatile("" ::: "memory");
            constexpr int PO = 4;
            const int npass = n > PO ? (n + PO - 1) / PO : 1;
#pragma unroll 1
            for (int ps = 0; ps < npass; ++ps) {
                uint32_t o[PO][8];
#pragma unroll
                for (int q = 0; q < PO; ++q)
#pragma unroll
                    for (int r = 0; r < 8; ++r) o[q][r] = 0;
#pragma unroll 1
                for (int ii = 0; ii < n; ++ii) {
                    const int y = dc_cload_u8(tb, syn::kYmap + ii);
                    WZ v;
#pragma unroll
                    for (int r = 0; r < 8; ++r) v.W[r] = 0;
                    static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int yy = decltype(yc)::value;
                        if (y == yy) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) v.W[r] = acc[yy][r];
                        }
                    });
                    expand_wz(v);
#pragma unroll
                    for (int q = 0; q < PO; ++q) {
                        const int j = PO * ps + q;
                        if (j < n) {
                            // nibble jumps (gf_winjump.h): one indirect jump per nibble
                            // instead of a 16-way branch tree
                            const uint32_t cf = (uint32_t)dc_cload_u8(tb, syn::kSinv + j * 16 + ii);
                            wz_mul_acc_rt(o[q], v, cf);
                        }
                    }
                }
                asm volatile("" ::: "memory");
#pragma unroll
                for (int q = 0; q < PO; ++q) {
                    const int j = PO * ps + q;
                    const bool on = j < n;
                    const int oslot = slots ? (on ? dc_cload_u8(slots, g * rmax + j) : 0) : j;
                    store_out(out + g * out_gstride + (long long)oslot * BB, on, o[q]);
                }
                asm volatile("" ::: "memory");
            }
            if constexpr (NSTMIN > PO * 8) {
                if (npass == 1) {
                    // pad: a unit ends with at least NSTMIN stores (empty range)
                    const __amdgpu_buffer_rsrc_t none =
                        __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
                    for (int q = 0; q < NSTMIN - PO * 8; ++q)
                        __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
                }
            }
        }
        asm volatile("" ::: "memory");
        cu = nu;
        rw_c = rw_n;
        rn_c = rn_n;
        vc0 = vn0;
        vc1 = vn1;
    }
    dc_wait_vmcnt<0>();
}

}  // namespace

constexpr int kDcolS = 1126;   // bb = 9008: 9000-byte payloads (BASELINE config D)

// One instantiation of gf_dcol_kernel per translation unit (gf_dcol_<e|d><D><C>.hip): each
// takes minutes to compile, and separate objects build in parallel.
#define QD_LAUNCH_ARGS                                                                          \
    dim3 grid, size_t lds, hipStream_t st, const uint8_t *in, uint8_t *out, const uint8_t *tab, \
        const uint8_t *slots, const int32_t *nout, const uint8_t *cenc, long long groups,       \
        int rmax, long long in_bytes, long long tab_gstride, long long out_gstride
hipError_t dcol_go_e63(QD_LAUNCH_ARGS);
hipError_t dcol_go_e83(QD_LAUNCH_ARGS);
hipError_t dcol_go_d62(QD_LAUNCH_ARGS);
hipError_t dcol_go_d82(QD_LAUNCH_ARGS);

#define QD_DEFINE_GO(NAME, DV, DEC, C, ...)                                                     \
    hipError_t NAME(QD_LAUNCH_ARGS) {                                                           \
        qlaunch((gf_dcol_kernel<kDcolS, DV, DEC, C, ##__VA_ARGS__>), grid, dim3(kDcWaves * 64),  \
                lds, st, in,                                                                    \
                out, tab, slots, nout, cenc, groups, rmax, in_bytes, tab_gstride, out_gstride); \
        return hipGetLastError();                                                               \
    }

}  // namespace qfec
