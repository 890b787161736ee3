// gf_stream.hip — m > 1 encode / decode for groups of small blocks (bb <= 2 KiB, one column
// word of each sub-row per lane): the shape of BASELINE configs B and C ((32 + 4) x 1352 B)
// and of every group whose padded packets are at most 2 KiB.
//
// Same arithmetic as gf_apply_kernel (bit-sliced Cauchy code, cauchy_256.cpp:90-125,
// :1502-1601, W/Z nibble expansion of gf_bitslice.h).  What differs is the memory path.
// Reading 169-byte sub-rows with per-lane dword loads tops out at ~4.5 TB/s on MI355X
// (tools/microbench/b_mem_mb.hip, variants a/e), while 1 KiB global_load_lds_dwordx4 pieces
// of whole groups stream at 6.5-6.8 TB/s read-only (tools/microbench/a_ceiling.hip).
//
// Every wave owns whole groups (g0, g0 + W, ...) and streams them through a private LDS
// ring of R one-KiB slots plus a mirror of the first two (a piece DMA'd into slot s < 2 is
// also DMA'd into slot R + s), so any block that starts inside the ring lies contiguous in
// LDS and is read with fixed offsets.  The wave consumes the blocks of a group in order;
// before block x it tops the ring up with the next pieces of its stream (crossing into its
// next group) and waits, with a counted `s_waitcnt vmcnt`, only for the pieces block x
// covers.  No barriers, no cross-wave traffic.  Lane c takes column word c of the 8
// sub-rows of a block as two aligned dwords and v_alignbyte (sub-row t starts t * s bytes
// into the block), expands W/Z and applies the outputs.  The group's outputs are stored
// when its last block is done, through buffer stores whose out-of-range lanes are
// dropped, so the number of VMEM instructions per group is fixed and the vmcnt
// bookkeeping is exact.
//
// vmcnt bookkeeping: `vm` counts every VMEM instruction the wave issued (DMA pieces, their
// mirror copies, stores); lane s of `vmv` holds the value of `vm` at the last instruction
// that wrote slot s.  VMEM instructions retire in issue order, so waiting for
// vmcnt <= vm - 1 - vmv[slot] retires that piece.  No other VMEM instruction may be
// emitted in the loop (coefficients, nout and slots come through s_load); the ISA check
// in tests/test_isa.py guards that.
//
// Decode: per-group coefficients from the decode prep ([G][1][k][RCP]), outputs go to
// slots[g][j] (or j, recovered-blocks layout) and groups with nout == 0 are skipped.  All of
// a group's blocks are in LDS before any of its stores, so in place is safe.
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

#define QS_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QS_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void stream_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform run-time n in [LO, HI]: binary dispatch.
template <int LO, int HI>
__device__ __forceinline__ void stream_wait_dyn(int n) {
    if constexpr (LO == HI) {
        stream_wait_vmcnt<LO>();
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (n <= MID) stream_wait_dyn<LO, MID>(n);
        else stream_wait_dyn<MID + 1, HI>(n);
    }
}

// 16 bytes per lane from buffer rs at voff into LDS at lds + 16 * lane (nt); offsets past
// the buffer's range load zeros.  (Device only: in a lambda the builtin would void the
// kernel's host stub.)
template <int AUX = 2>
__device__ __forceinline__ void stream_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds,
                                             uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QS_LPTR(lds), 16, voff, 0, 0, AUX);
#else
    (void)rs, (void)lds, (void)voff;
#endif
}

// Byte i of a 4-byte-aligned kernel-argument array through s_load_dword: a byte load
// (global_load_ubyte, or flat_load after an integer-to-pointer cast) would be a VMEM
// instruction outside the vmcnt bookkeeping, and its use would drain the ring.
__device__ __forceinline__ int sload_u8(const uint8_t* __restrict__ base, long long i) {
    const uint32_t wv = ((const uint32_t*)base)[i >> 2];
    return (int)((wv >> (8 * (i & 3))) & 0xFFu);
}

constexpr unsigned kSDrop = 0x80000000u;   // buffer offset past any range: lane dropped
constexpr int kStreamWaves = 4;            // waves per workgroup (independent)
constexpr int kMirror = 2;                 // mirrored slots: a block (<= 2 KiB + 3 B of
                                           // over-read) starting in the ring never wraps

// S = sub-row bytes (bb / 8) at compile time, or 0: s_rt at run time (any s <= 256).
// RC = outputs per group (one chunk: m <= RC for encode, rmax <= RC for decode).
// RCPT = byte stride of a coefficient row in the table (max(4, table rc)).  Encode is
// instantiated with RC = m exactly, so the per-output `j < n` test folds away.
// KC > 0 (encode only): the code is fixed, k = KC and m = RC <= 6, and the coefficients come
// from cauchy_const.h at compile time.  The block loop is then fully unrolled and every
// 8x8 bit expansion folds into its straight-line XORs: no coefficient loads and no scalar
// nibble dispatch (about 9 scalar instructions per nibble in the run-time form).
//
// Units: a group's outputs are cut into nchunk chunks of RC (encode m > 8, decode rmax > 8);
// a unit is one (group, chunk) and streams the whole group (the chunks of one group run on
// neighbouring waves, so the re-reads hit L2).  Groups whose byte offset is 8 mod 16 (odd k
// with bb = 8 mod 16: the reference's (5, 5) and (15, 15) presets at 1352-byte blocks) are
// streamed from the 16-byte boundary below them, their blocks 8 bytes into the stream.
// NJ (decode): each run-time product is two nibble jumps straight into its output's
// accumulator (gf_winjump.h wz_mul_acc_rt) instead of two 16-way uniform branch trees.
// WIDE (compiled encode, S = 169): each output block is assembled in a per-wave LDS staging
// buffer (inline-asm ds ops) and written with 3 dwordx2 stores of contiguous bytes instead
// of 8 x (b32 + b8) sub-row stores (the (5, 5) encode).
constexpr int kStreamStage = 1360;
template <int RC, int S, bool DECODE, int RCPT = (RC < 4 ? 4 : RC), int KC = 0, bool NJ = false,
          bool WIDE = false>
__global__ __launch_bounds__(kStreamWaves * 64) void gf_stream_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int k, int m, int rmax, long long coef_gstride, long long out_gstride, int R, int s_rt,
    int nchunk) {
    static_assert(KC == 0 || (!DECODE && RC >= 2 && RC <= 20 && S > 0),
                  "compile-time codes: encode, m <= 6, fixed block size");
    static_assert(S <= 256, "one column word of each sub-row per lane");
    const int s = S ? S : s_rt;                     // sub-row bytes
    const int BB = 8 * s;
    const int NW = (s + 3) >> 2;                    // column words per sub-row
    const int NWF = s >> 2;                         // full words
    constexpr int NCW = RCPT / 4;
    static_assert(RCPT % 4 == 0 && RCPT >= RC, "coefficient row stride");
    // store instructions per sub-row: b32 (full words) + b16 / b8 (the tail word)
    constexpr int SPR = S ? 1 + ((S >> 1) & 1) + (S & 1) : 3;
    constexpr int SAUX = DECODE ? 0 : 2;   // encode's dense parity stream: nt stores
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // the lane id, recomputed where it is used (v_mbcnt): nothing lane-derived stays live
    // across the block loop (register pressure of the compiled encodes with many outputs)
    auto lane_here = []() __attribute__((always_inline)) -> int {
        int l = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
#endif
        return l;
    };
    const int w = wave_id();
    const int RB = R * 1024;
    uint8_t* ring = smem + (size_t)w * (R + kMirror) * 1024;
    static_assert(!WIDE || (S == 169 && !DECODE), "wide stores: 1352-byte encode blocks");
    const uint32_t stage =   // this wave's staging buffer (LDS address), after every wave's ring
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(
            smem + (size_t)kStreamWaves * (R + kMirror) * 1024 + (size_t)w * kStreamStage);
    const long long W = (long long)gridDim.x * kStreamWaves;
    const long long g0 = (long long)blockIdx.x * kStreamWaves + w;   // the wave's first unit
    const long long NU = groups * nchunk;
    if (g0 >= NU) return;
    const long long cnt =   // wave-uniform, kept in SGPRs (the division runs on the VALU)
        __builtin_amdgcn_readfirstlane((int)((NU - 1 - g0) / W + 1));   // units of this wave
    if constexpr (KC > 0) k = KC;
    const int gb = k * BB;
    const int skew8 = (gb & 15) ? 8 : 0;               // groups may start 8 mod 16
    const int NP = (gb + skew8 + 1023) >> 10;          // pieces per unit
    // column word of a lane (idle lanes shadow the last word)
    auto col_here = [&]() __attribute__((always_inline)) -> int { return min(lane_here(), NW - 1); };

    // ---- issue side (wave-uniform): next piece iss_p of the stream, into slot iss_slot
    int iss_p = 0, iss_slot = 0;
    int issued = 0;                                    // pieces issued
    int vm = 0;                                        // VMEM instructions issued
    uint32_t vmv = 0;                                  // lane s: vm index of slot s's last write
    // the 16-byte aligned start of unit u's group, and its last 16-byte chunk (clamp)
    // A decode unit without output (a group with nothing lost, or a chunk past its losses) is
    // left out of the stream: its group is not read at all.
    const long long u_end = g0 + cnt * W;              // past the wave's last unit
    auto unit_live = [&](long long u) -> bool {
        if constexpr (!DECODE) return true;
        const long long g = u / nchunk;
        return nout[g] - (int)(u - g * nchunk) * RC > 0;
    };
    long long iss_u = g0;
    while (iss_u < u_end && !unit_live(iss_u)) iss_u += W;
    // The loads go through a buffer resource bounded by the end of the input: the last
    // 16-byte chunk of a group whose size is 8 mod 16 reaches 8 bytes past it, which past the
    // last group of the buffer reads as zeros instead of touching unmapped memory.
    const long long in_bytes = groups * (long long)gb;
    auto unit_src = [&](long long u, int& last, unsigned& nrec) -> const uint8_t* {
        const long long a = (u / nchunk) * (long long)gb;
        const int sk = (int)(a & 15);
        last = (sk + gb - 1) & ~15;
        nrec = (unsigned)min(in_bytes - (a - sk), (long long)gb + 32);
        return in + (a - sk);
    };
    int ilast = 0;
    unsigned inrec = 0;
    const uint8_t* isrc = unit_src(iss_u < u_end ? iss_u : g0, ilast, inrec);

    auto issue_one = [&]() {
        const int lane = lane_here();
        const int off = min(iss_p * 1024 + lane * 16, ilast);   // last piece: clamp inside
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)isrc, 0, inrec, 0x00020000);
        stream_dma16(rs, ring + iss_slot * 1024, (uint32_t)off);
        ++vm;
        if (iss_slot < kMirror) {
            stream_dma16(rs, ring + (R + iss_slot) * 1024, (uint32_t)off);
            ++vm;
        }
        vmv = lane == iss_slot ? (uint32_t)(vm - 1) : vmv;
        ++issued;
        if (++iss_slot == R) iss_slot = 0;
        if (++iss_p == NP) {
            iss_p = 0;
            do {
                iss_u += W;
            } while (iss_u < u_end && !unit_live(iss_u));
            isrc = unit_src(iss_u, ilast, inrec);
        }
    };
    // top the ring up: every piece from `head` on stays, the rest of the R slots refill
    auto fill = [&](int head) {
        while (iss_u < u_end && issued - head < R) issue_one();
    };
    // wait until the block at ring position bp has landed (its last piece retired)
    auto wait_block = [&](uint32_t bp) {
        int sl = (int)((bp + BB - 1) >> 10);
        sl = sl >= R ? sl - R : sl;
        const int idx = __builtin_amdgcn_readlane((int)vmv, sl);
        const int pending = vm - 1 - idx;
        // coarse steps (a smaller count only waits longer): 4 scalar branch levels
        if (pending >= 16) {
            if (pending >= 32) {
                if (pending >= 48) stream_wait_vmcnt<48>();
                else stream_wait_vmcnt<32>();
            } else {
                if (pending >= 24) stream_wait_vmcnt<24>();
                else stream_wait_vmcnt<16>();
            }
        } else {
            stream_wait_dyn<0, 15>(pending < 0 ? 0 : pending);
        }
    };
    // column word c of the 8 sub-rows as aligned dword pairs (block starts are 8-byte
    // aligned in the ring: slots are 1 KiB and BB % 8 == 0; sub-row t is misaligned by
    // (t * s) & 3, realigned with v_alignbyte at use).  The block lies contiguous in
    // [bp, bp + BB + 3] thanks to the mirror.
    auto read_block = [&](uint32_t bp, uint32_t (&lo)[8], uint32_t (&hi)[8]) {
        // the lane's byte offset, opaque to the optimiser: in the fully unrolled (KC > 0)
        // form it would otherwise precompute every block's addresses up front
        uint32_t c4 = 4u * (uint32_t)col_here();
        if constexpr (KC > 0) asm volatile("" : "+v"(c4));
        const uint8_t* L = ring + bp + c4;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = t * s;
            const uint32_t* q = (const uint32_t*)(L + (o & ~3));
            lo[t] = q[0];
            hi[t] = (S == 0 || (o & 3)) ? q[1] : 0u;
        }
    };
    auto next_pos = [&](uint32_t bp) -> uint32_t {
        bp += BB;
        return bp >= (uint32_t)RB ? bp - (uint32_t)RB : bp;
    };

    // ---- consume side
    int gbase = 0;                                     // first piece of the current group
    int gslot0 = 0;                                    // its slot
#pragma unroll 1
    for (long long i = 0; i < cnt; ++i) {
        const long long u = g0 + i * W;
        const long long g = u / nchunk;
        const int ch = (int)(u - g * nchunk);            // output chunk: outputs ch * RC + j
        const int sk = (int)((g * gb) & 15);             // the group's bytes start sk into its stream
        int n = (DECODE ? nout[g] : m) - ch * RC;
        n = n > RC ? RC : n;
        if (n > 0) {
            const uint32_t* cw = (const uint32_t*)(coef + (DECODE ? g * coef_gstride : 0) +
                                                   (long long)ch * k * RCPT);
            uint32_t acc[RC][8];
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[j][r] = 0;
            // Block x + 1's LDS reads are issued before block x is combined (software
            // pipeline); the ring keeps every piece from block x's first on, so block x's
            // pieces are not refilled while its reads may still be in flight.
            uint32_t bpos = (uint32_t)gslot0 * 1024u + (uint32_t)sk;   // ring position of block x
            uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
            fill(gbase);
            wait_block(bpos);
            read_block(bpos, lo0, hi0);
            // xc: the block index, an int or (KC > 0) an integral_constant
            // run-time coefficients two blocks ahead: the scalar load for block x + 2 is
            // issued while block x is combined, so its latency is hidden
            uint32_t cA[NCW], cB[NCW];
            if constexpr (KC == 0) {
#pragma unroll
                for (int q = 0; q < NCW; ++q) {
                    cA[q] = cw[q];
                    cB[q] = cw[(k > 1 ? 1 : 0) * NCW + q];
                }
            }
            auto step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8],
                            uint32_t (&nlo)[8], uint32_t (&nhi)[8], uint32_t (&cc)[NCW]) {
                const int x = xc;
                const uint32_t bn = next_pos(bpos);
                if (x + 1 < k) {
                    fill(gbase + ((sk + x * BB) >> 10));
                    wait_block(bn);
                    read_block(bn, nlo, nhi);
                }
                bpos = bn;
                WZ v;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int o = t * s;
                    v.W[t] = (S == 0 || (o & 3)) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3)
                                                 : lo[t];
                }
                if constexpr (KC > 0) {
                    // windowed form (gf_bitslice.h): one v_bitop3 per (output, sub-row); row 0
                    // is P0, all coefficients 1 (cauchy_256.cpp:1519-1523)
                    Win win;
                    win_build(v.W8, win);
                    static_for<RC>([&](auto jc) __attribute__((always_inline)) {
                        constexpr int j = decltype(jc)::value;
                        win_apply<cauchy_coef(RC, j, decltype(xc)::value)>(acc[j], win);
                    });
                    return;
                }
                uint32_t cwv[NCW];
                const int xn = x + 2 < k ? x + 2 : k - 1;
#pragma unroll
                for (int q = 0; q < NCW; ++q) {
                    cwv[q] = cc[q];
                    cc[q] = cw[xn * NCW + q];
                }
                expand_wz(v);
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (!DECODE && j == 0 && ch == 0) {
                        // encode row 0 is P0, all coefficients 1 (cauchy_256.cpp:1519-1523):
                        // a plain XOR, no scalar nibble dispatch
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                    } else if (j < n) {
                        const uint32_t cf = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                        if constexpr (NJ) {
                            wz_mul_acc_rt(acc[j], v, cf);
                        } else {
                            apply_nibble<0>(acc[j], cf & 15u, v);
                            apply_nibble<4>(acc[j], cf >> 4, v);
                        }
                    }
                }
            };
            if constexpr (KC > 0) {
                // the block loop inline, not through a lambda (the fully unrolled 250-block
                // loop of (250, 5) spills to scratch through one)
                static_for<KC>([&](auto xc) {
                    // the accumulators are opaque at every block boundary: with all
                    // coefficients constant, the XOR reassociation would otherwise flatten the
                    // blocks' sums into one tree and keep every block's W/Z live (~490 VGPRs)
#pragma unroll
                    for (int j = 0; j < RC; ++j)
#pragma unroll
                        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[j][r]));
                    if constexpr (decltype(xc)::value % 2 == 0)
                        step(xc, lo0, hi0, lo1, hi1, cA);
                    else
                        step(xc, lo1, hi1, lo0, hi0, cB);
                });
            } else {
#pragma unroll 1
                for (int x = 0; x < k; x += 2) {
                    step(x, lo0, hi0, lo1, hi1, cA);
                    if (x + 1 < k) step(x + 1, lo1, hi1, lo0, hi0, cB);
                }
            }
            asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
            // ---- outputs: fixed instruction count per output (dropped lanes, no branches).
            // Lane offsets 4c (full words) and the tail lane's, sub-row in the scalar offset:
            // two address VGPRs, opaque so they are not hoisted as 8 x RC precomputed ones.
            const int lane = lane_here(), c = min(lane, NW - 1);
            uint32_t vo = lane < NWF ? 4u * (uint32_t)c : kSDrop;
            uint32_t vt = lane == NWF && NWF < NW ? 4u * (uint32_t)c : kSDrop;
            asm volatile("" : "+v"(vo), "+v"(vt));
            if constexpr (WIDE) {
                // 8 ds_write_b32 per lane at the sub-row offsets (the tail word's 3 extra bytes
                // land on the next sub-row's start, overwritten by its later write; the last
                // one's inside the staging pad), then 3 x 512 B read back and stored as
                // contiguous 8-byte lanes (past the block: dropped by the buffer range; the
                // reads past 1360 B touch the next wave's buffer or read zeros, unused)
                const uint32_t ra = stage + 8u * (uint32_t)lane;
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    const int jo = ch * RC + j;
                    uint8_t* dst = out + g * out_gstride + (long long)jo * BB;
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
                    if (lane < NW) stage_block_169(stage, acc[j], lane);
                    uint64_t v0, v1, v2;
                    asm volatile("ds_read_b64 %0, %3\n\t"
                                 "ds_read_b64 %1, %3 offset:512\n\t"
                                 "ds_read_b64 %2, %3 offset:1024\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=&v"(v0), "=&v"(v1), "=&v"(v2)
                                 : "v"(ra)
                                 : "memory");
                    const uint64_t vv[3] = {v0, v1, v2};
#pragma unroll
                    for (int h = 0; h < 3; ++h)
                        __builtin_amdgcn_raw_buffer_store_b64(
                            qf_u32x2(vv[h]),
                            rs, 512u * h + 8u * (uint32_t)lane, 0, SAUX);
                    vm += 3;
                }
                asm volatile("" ::: "memory");
                gbase += NP;
                gslot0 = (gslot0 + NP) % R;
                continue;
            }
#pragma unroll
            for (int j = 0; j < RC; ++j) {
                if (j < n) {
                    const int jo = ch * RC + j;
                    const int oslot = (DECODE && slots) ? sload_u8(slots, g * rmax + jo) : jo;
                    uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const uint32_t vsum = acc[j][r];
                        __builtin_amdgcn_raw_buffer_store_b32(vsum, rs, vo, r * s, SAUX);
                        if (S == 0 || (S & 2))
                            __builtin_amdgcn_raw_buffer_store_b16(
                                (uint16_t)vsum, rs, (s & 2) ? vt : kSDrop, r * s, SAUX);
                        if (S == 0 || (S & 1))
                            __builtin_amdgcn_raw_buffer_store_b8(
                                (uint8_t)(vsum >> (8 * (s & 2))), rs, (s & 1) ? vt : kSDrop,
                                r * s + (s & 2), SAUX);
                    }
                    vm += 8 * SPR;
                }
            }
            asm volatile("" ::: "memory");
            gbase += NP;                                 // units without output stream nothing
            gslot0 = (gslot0 + NP) % R;
        }
    }
    stream_wait_vmcnt<0>();
}

// ------------------------------------------------------------------ static ring
// gf_ring_kernel: the same stream for one FIXED shape (k = K blocks of 8 * S bytes: the
// BASELINE B/C groups, (32 + 4) x 1352 B), with the whole per-group schedule known at
// compile time.  A group is NP one-KiB pieces; piece n of a wave's stream lands in ring slot
// (phase + n) mod R, phase = the group's first slot (advances by NP mod R per group).
// Before block x's compute the ring holds every piece from block x's first one on and is
// filled up to F(x) = pf(x) + R - 1 (the next group's first pieces included), so the number
// of pieces per step, and the count of VMEM instructions younger than the next block's
// last piece (plus the previous group's fixed-count stores where they sit in between), are
// constants: every wait is an immediate `s_waitcnt vmcnt`, with no run-time bookkeeping.
// The stream's ends are made regular too: the first group finds NST dummy stores (empty
// buffer range) where a previous group's stores would be, and the last group issues
// dummy pieces (a reread of its own last piece) for the group that does not follow.
// No mirror: a block that wraps round the ring end (uniform test) is read with per-lane
// wrapped addresses.
constexpr int kRingWaves = 4;

// SK: the group's bytes start SK bytes into its stream (odd k at 1352-byte blocks: groups
// alternate between 0 and 8 bytes past a 16-byte boundary)
template <int S, int SK = 0>
struct RingShape {
    static constexpr int R = 8, RB = R * 1024;
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4, NWF = S / 4;
    static constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);
    static constexpr int pf(int x) { return (SK + x * BB) >> 10; }             // first piece of block x
    static constexpr int pl(int x) { return (SK + (x + 1) * BB - 1) >> 10; }   // its last piece
    // smallest count of VMEM instructions younger than a block's last piece when the wave
    // waits for it (K blocks per group, NST stores per group): one conservative immediate
    // for the rolled (run-time block index) form
    static constexpr int min_younger(int K, int NST) {
        const int NP = (K * BB + 1023) / 1024;
        const int FM1 = pf(K - 1) + R - 1 - NP;
        int mn = FM1 - pl(0) + NST;
        for (int x = 0; x + 1 < K; ++x) {
            const int y = pf(x) + R - 1 - pl(x + 1) + (pl(x + 1) <= FM1 ? NST : 0);
            mn = y < mn ? y : mn;
        }
        return mn > 63 ? 63 : mn;
    }
};

// NT: the encode's parity stores are non-temporal (decode stores plain).  SK: see RingShape.
// A group whose size is 8 mod 16 is streamed as GBS = GB + 8 bytes from the 16-byte boundary
// at or below its start; the loads then go through a buffer resource bounded by the end of
// the input (the last group's stream may end 8 bytes past it: those lanes read zeros).
// NCH > 1 (encode): a group's MC parity rows are NCH chunks of RC rows, one unit each; unit
// u = NCH * g + ch, and a wave's units u0, u0 + W, ... (W a multiple of NCH) all have chunk
// Y0 / RC = u0 % NCH, so the chunk's rows are compile-time; the NCH units of a group run on
// neighbouring waves, whose reads of the group meet in L2.
template <int K, int S, int RC, bool DECODE, int MC, bool NT, int SK, bool WIDE, int NCH = 1,
          int Y0 = 0>
__device__ __forceinline__ void gf_ring_run(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int rmax, long long coef_gstride, long long out_gstride, uint8_t* smem) {
    using SH = RingShape<S, SK>;
    constexpr int R = SH::R, RB = SH::RB, BB = SH::BB, NW = SH::NW, NWF = SH::NWF;
    constexpr int GB = K * BB;
    constexpr bool SKEW = GB % 16 != 0;
    constexpr int GBS = (GB + 15) / 16 * 16;              // stream bytes per group
    constexpr int NP = (GBS + 1023) / 1024;
    static_assert(SKEW ? GB % 16 == 8 : SK == 0, "groups 0 or 8 bytes off 16");
    // stores per group, fixed: 8 sub-rows x SPR per output, or (WIDE) 3 runs of 512 bytes
    constexpr int NST = WIDE ? RC * 3 : RC * 8 * SH::SPR;
    static_assert(!WIDE || (S == 169 && !DECODE), "wide stores: 1352-byte encode blocks");
    constexpr int RCP = RC < 4 ? 4 : RC, NCW = RCP / 4;
    constexpr int SAUX = (DECODE || !NT) ? 0 : 2;         // encode's parity stream: nt
    constexpr int FM1 = SH::pf(K - 1) + R - 1 - NP;       // next-group pieces issued early
    static_assert(!DECODE || MC == 0, "decode coefficients are per group");
    static_assert(DECODE || MC == RC * NCH, "encode: one output per register set");
    static_assert(NCH == 1 || (!DECODE && Y0 % RC == 0 && Y0 < MC), "chunked encode");
    static_assert(FM1 >= SH::pl(0), "block 0 of the next group is prefetched in full");
    static_assert(SH::pf(K - 1) + R - 1 < 2 * NP, "the frontier stays within the next group");
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    uint8_t* ring = smem + (size_t)w * RB;
    const uint32_t stage =   // (WIDE) this wave's staging buffer (LDS address), after the rings
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(
            smem + (size_t)kRingWaves * RB + (size_t)w * kStreamStage);
    const long long W = (long long)gridDim.x * kRingWaves / NCH;   // group stride of the wave
    const long long g0 = ((long long)blockIdx.x * kRingWaves + w) / NCH;
    if (g0 >= groups) return;
    const long long cnt =   // wave-uniform, kept in SGPRs (the division runs on the VALU)
        __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));      // groups of this wave
    const int c = lane < NW ? lane : NW - 1;              // idle lanes shadow the last word
    const long long gstep = W * GB;

    const uint8_t* gsrc = in + g0 * GB - SK;              // current group's stream
    const uint8_t* in_end = in + groups * GB;
    int phase = 0;                                        // ring slot of its piece 0
    long long i = 0;                                      // current group

    // piece p of the stream that starts at src into ring slot `slot`.  The skewed form puts
    // the piece's offset into the descriptor's base (the range check then bounds the piece,
    // and the lane offsets are two loop-invariant VGPRs instead of one per piece)
    const uint32_t v16 = 16u * (uint32_t)lane;
    const uint32_t vlast = min(16u * (uint32_t)lane, (uint32_t)(GBS - 16 - (NP - 1) * 1024));
    // non-temporal loads, but default policy when a group's chunks are read by NCH waves
    // (the sibling's reads then hit the lines in L2)
    constexpr int LAUX = NCH > 1 ? 0 : 2;
    auto dma = [&](const uint8_t* src, int p, int slot) __attribute__((always_inline)) {
        if constexpr (SKEW) {
            const uint8_t* b = src + p * 1024;
            const long long left = in_end - b;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)b, 0, (unsigned)(left < 1024 ? left : 1024), 0x00020000);
            stream_dma16<LAUX>(rs, ring + slot * 1024, p == NP - 1 ? vlast : v16);
        } else {
            const int off = min(p * 1024 + lane * 16, GBS - 16);
            __builtin_amdgcn_global_load_lds(QS_GPTR(src + off), QS_LPTR(ring + slot * 1024), 16,
                                             0, LAUX);
        }
    };

    // piece n of the current group (n >= NP: piece n - NP of the next, or a dummy reread
    // of the current group's last piece when there is no next group)
    auto issue = [&](auto nc) __attribute__((always_inline)) {
        constexpr int n = decltype(nc)::value;
        if constexpr (n < NP) {
            dma(gsrc, n, (phase + n) & (R - 1));
        } else {
            const bool next = i + 1 < cnt;
            dma(next ? gsrc + gstep : gsrc, next ? n - NP : NP - 1, (phase + n) & (R - 1));
        }
    };
    // the same for a run-time piece index (rolled decode loop)
    auto issue_rt = [&](int n) __attribute__((always_inline)) {
        const uint8_t* src = gsrc;
        int p = n;
        if (n >= NP) {
            const bool next = i + 1 < cnt;
            src = next ? gsrc + gstep : gsrc;
            p = next ? n - NP : NP - 1;
        }
        dma(src, p, (phase + n) & (R - 1));
    };
    // block x (an int or an integral_constant) at ring byte (phase * 1024 + x * BB) mod RB
    auto read_block = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8])
                          __attribute__((always_inline)) {
        const int x = xc;
        uint32_t c4 = 4u * (uint32_t)c;
        asm volatile("" : "+v"(c4));   // opaque: addresses are not hoisted across blocks
        uint32_t bp = ((uint32_t)phase * 1024u + (uint32_t)(SK + x * BB)) & (uint32_t)(RB - 1);
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

    // ---- prologue: the first group's early pieces, then the stores a previous group
    // would have issued (dropped: empty range), so every group sees the same VMEM history
    static_for<FM1 + 1>([&](auto nc) __attribute__((always_inline)) { issue(nc); });
    // The waits count VMEM instructions in issue order: the compiler must not move a
    // buffer store across a DMA (it may: they touch different memory).
    asm volatile("" ::: "memory");
    {
        const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
        for (int q = 0; q < NST; ++q)   // distinct offsets: not merged as duplicate stores
            __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
    }

    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
#pragma unroll 1
    for (; i < cnt; ++i) {
        const long long g = g0 + i * W;
        int n = DECODE ? nout[g] : RC;
        n = n > RC ? RC : n;
        const uint32_t* cw = (const uint32_t*)(coef + (DECODE ? g * coef_gstride : 0));
        uint32_t acc[RC][8];
#pragma unroll
        for (int j = 0; j < RC; ++j)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[j][r] = 0;
        // block 0: its pieces were issued before the previous group's stores
        stream_wait_vmcnt<(FM1 - SH::pl(0) + NST > 63 ? 63 : FM1 - SH::pl(0) + NST)>();
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
                stream_wait_vmcnt<(yng > 63 ? 63 : yng)>();
                read_block(std::integral_constant<int, x + 1>{}, nlo, nhi);
            }
            if (DECODE && n <= 0) return;   // no loss in this group: nothing to combine
            WZ v;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                v.W[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
            if constexpr (!DECODE) {
                Win win;
                win_build(v.W8, win);
                static_for<RC>([&](auto jc) __attribute__((always_inline)) {
                    constexpr int j = decltype(jc)::value;
                    win_apply<cauchy_coef(MC, Y0 + j, x)>(acc[j], win);
                });
            } else {
                uint32_t cwv[NCW];
#pragma unroll
                for (int q = 0; q < NCW; ++q) cwv[q] = cw[x * NCW + q];
                expand_wz(v);
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (j < n) {
                        const uint32_t cf = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                        apply_nibble<0>(acc[j], cf & 15u, v);
                        apply_nibble<4>(acc[j], cf >> 4, v);
                    }
                }
            }
        };
        if constexpr (!DECODE) {
            static_for<K>([&](auto xc) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < RC; ++j)
#pragma unroll
                    for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[j][r]));
                if constexpr (decltype(xc)::value % 2 == 0) step(xc, lo0, hi0, lo1, hi1);
                else step(xc, lo1, hi1, lo0, hi0);
            });
        } else {
            // Decode: run-time coefficients make an unrolled group long (~30K instructions,
            // past the instruction cache's comfort); the rolled loop issues the same pieces
            // (frontier pf(x) + R - 1) and waits with the smallest younger count any block
            // sees, a constant: conservative by at most one piece.
            constexpr int WMIN = SH::min_younger(K, NST);
            int fr = FM1;                                  // pieces issued so far (last index)
            // coefficient rows two blocks ahead (scalar loads have a long latency; the
            // value for block x is loaded while block x - 2 is combined)
            static_assert(NCW == 1, "rmax <= 4: one coefficient dword per block");
            uint32_t cA = cw[0], cB = cw[1];
            auto rstep = [&](int x, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                             uint32_t (&nhi)[8], uint32_t& cc) __attribute__((always_inline)) {
                const int f1 = ((x * BB) >> 10) + R - 1;
                for (; fr < f1; ++fr) issue_rt(fr + 1);
                if (x + 1 < K) {
                    stream_wait_vmcnt<WMIN>();
                    read_block(x + 1, nlo, nhi);
                }
                if (n <= 0) return;   // no loss in this group: nothing to combine
                WZ v;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int o = t * S;
                    v.W[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
                }
                const uint32_t cwv = cc;
                cc = cw[min(x + 2, K - 1)];
                expand_wz(v);
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (j < n) {
                        const uint32_t cf = (cwv >> (8 * (j & 3))) & 0xFFu;
                        apply_nibble<0>(acc[j], cf & 15u, v);
                        apply_nibble<4>(acc[j], cf >> 4, v);
                    }
                }
            };
            static_assert(K % 2 == 0, "register double buffer parity");
#pragma unroll 1
            for (int x = 0; x < K; x += 2) {
                rstep(x, lo0, hi0, lo1, hi1, cA);
                rstep(x + 1, lo1, hi1, lo0, hi0, cB);
            }
        }

        // ---- outputs: NST store instructions whatever n is (unused outputs: empty range),
        // kept after the last step's DMAs and before the next group's (issue order)
        asm volatile("" ::: "memory");
        if constexpr (WIDE) {
            // each parity block staged in LDS as its contiguous bytes (stage_block_169), read
            // back as 3 x 512 bytes and stored as 8-byte lanes (past the block: dropped by the
            // buffer range)
            const uint32_t ra = stage + 8u * (uint32_t)lane;
#pragma unroll
            for (int j = 0; j < RC; ++j) {
                uint8_t* dst = out + g * out_gstride + (long long)(Y0 + j) * BB;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
                if (lane < NW) stage_block_169(stage, acc[j], lane);
                uint64_t v0, v1, v2;
                asm volatile("ds_read_b64 %0, %3\n\t"
                             "ds_read_b64 %1, %3 offset:512\n\t"
                             "ds_read_b64 %2, %3 offset:1024\n\t"
                             "s_waitcnt lgkmcnt(0)"
                             : "=&v"(v0), "=&v"(v1), "=&v"(v2)
                             : "v"(ra)
                             : "memory");
                const uint64_t vv[3] = {v0, v1, v2};
#pragma unroll
                for (int h = 0; h < 3; ++h)
                    __builtin_amdgcn_raw_buffer_store_b64(qf_u32x2(vv[h]), rs,
                                                          512u * h + 8u * (uint32_t)lane, 0, SAUX);
            }
            asm volatile("" ::: "memory");
            gsrc += gstep;
            phase = (phase + NP) & (R - 1);
            continue;
        }
        uint32_t vo = lane < NWF ? 4u * (uint32_t)c : kSDrop;
        uint32_t vt = lane == NWF && NWF < NW ? 4u * (uint32_t)c : kSDrop;
        asm volatile("" : "+v"(vo), "+v"(vt));
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            const bool on = j < n;
            const int oslot = (DECODE && slots) ? (on ? sload_u8(slots, g * rmax + j) : 0) : Y0 + j;
            uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(dst, 0, on ? (unsigned)BB : 0u, 0x00020000);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t vsum = acc[j][r];
                __builtin_amdgcn_raw_buffer_store_b32(vsum, rs, vo, r * S, SAUX);
                if (S & 2)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)vsum, rs, vt, r * S, SAUX);
                if (S & 1)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(vsum >> (8 * (S & 2))), rs, vt,
                                                         r * S + (S & 2), SAUX);
            }
        }
        asm volatile("" ::: "memory");
        gsrc += gstep;
        phase = (phase + NP) & (R - 1);
    }
    stream_wait_vmcnt<0>();
}

#ifndef QF_RING_SKEW_INLINE
#define QF_RING_SKEW_INLINE __forceinline__
#endif
#ifndef QF_RING_ATTR
#define QF_RING_ATTR
#endif
template <int K, int S, int RC, bool DECODE, int MC, bool NT, bool WIDE, int NCH, int Y0>
__device__ QF_RING_SKEW_INLINE void gf_ring_skew(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int rmax, long long coef_gstride, long long out_gstride, uint8_t* smem) {
    if constexpr ((K * 8 * S) % 16 == 0) {
        gf_ring_run<K, S, RC, DECODE, MC, NT, 0, WIDE, NCH, Y0>(in, out, coef, slots, nout, groups,
                                                              rmax, coef_gstride, out_gstride, smem);
    } else {
        // group g starts 8 * (g & 1) bytes past a 16-byte boundary; a wave's groups g0,
        // g0 + W, ... (W = 4 x the grid / NCH, even) all share g0's skew
        const long long g0 = ((long long)blockIdx.x * kRingWaves + wave_id()) / NCH;
        if (g0 & 1)
            gf_ring_run<K, S, RC, DECODE, MC, NT, 8, WIDE, NCH, Y0>(in, out, coef, slots, nout,
                                                                  groups, rmax, coef_gstride,
                                                                  out_gstride, smem);
        else
            gf_ring_run<K, S, RC, DECODE, MC, NT, 0, WIDE, NCH, Y0>(in, out, coef, slots, nout,
                                                                  groups, rmax, coef_gstride,
                                                                  out_gstride, smem);
    }
}

// NCH: parity-row chunks per group (encode; RC = MC / NCH rows each, chunk = the wave's unit
// index mod NCH)
template <int K, int S, int RC, bool DECODE, int MC, bool NT = true, bool WIDE = false, int NCH = 1>
__global__ __launch_bounds__(kRingWaves * 64) QF_RING_ATTR void gf_ring_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int rmax, long long coef_gstride, long long out_gstride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    static_assert(NCH == 1 || NCH == 2, "one or two chunks");
    if constexpr (NCH == 1) {
        gf_ring_skew<K, S, RC, DECODE, MC, NT, WIDE, 1, 0>(in, out, coef, slots, nout, groups,
                                                         rmax, coef_gstride, out_gstride, smem);
    } else {
        if ((blockIdx.x * kRingWaves + wave_id()) & 1)
            gf_ring_skew<K, S, RC, DECODE, MC, NT, WIDE, 2, RC>(in, out, coef, slots, nout,
                                                              groups, rmax, coef_gstride,
                                                              out_gstride, smem);
        else
            gf_ring_skew<K, S, RC, DECODE, MC, NT, WIDE, 2, 0>(in, out, coef, slots, nout,
                                                             groups, rmax, coef_gstride,
                                                             out_gstride, smem);
    }
}

// Ring slots the stream needs: before block x's compute the ring keeps every piece from
// block x's first on, and block x + 1 must land in it too.  Blocks x and x + 1 span
// (o + 2 * bb + 1023) / 1024 pieces from block x's head piece, o its start offset in that
// piece; o is a multiple of gcd(bb, 1024), so at most 1024 - gcd(bb, 1024).
int gf_stream_min_ring(int bb) {
    int a = bb, b = 1024;
    while (b) {
        const int r = a % b;
        a = b;
        b = r;
    }
    const int max_o = 1024 - a;
    return (max_o + 2 * bb + 1023) / 1024;
}

// Codes whose encode is compiled (cauchy_const.h coefficients, windowed form) at 1352-byte
// blocks: BASELINE B/C's (32, 4) and the QuicR presets (quic_fec_group.cc:22-82).
bool gf_stream_compiled(int k, int m, int bb) {
    if (bb != 8 * 169) return false;
    return (k == 32 && m == 4) || (k == 5 && m == 5) || (k == 10 && (m == 10 || m == 15 || m == 20)) ||
           (k == 15 && m == 15) || (k == 250 && m == 5);
}

bool gf_stream_supported(int k, int m, int bb, int rc, bool decode, const Tune& t) {
    (void)m;
    (void)decode;
    if (!t.stream) return false;
    if (bb % 8 != 0 || bb < 8 || bb > 2048) return false;   // s <= 256: a word per lane
    if (rc != 2 && rc != 4 && rc != 8 && rc != 16) return false;
    if ((long long)k * bb < 16) return false;   // groups 8 mod 16 apart stream skewed
    if (t.stream_ring < gf_stream_min_ring(bb)) return false;   // gf_apply instead
    return true;
}

#ifndef QF_KERNELS_ONLY   // (register-use experiments compile single instantiations)
hipError_t launch_gf_stream(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                            const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                            long long groups, int rc, int rmax, long long coef_gstride,
                            long long out_gstride, bool decode, hipStream_t st,
                            const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_stream_supported(k, m, bb, rc, decode, t)) return hipErrorInvalidValue;
    if (((uintptr_t)in & 15) != 0 || ((uintptr_t)slots & 3) != 0) return hipErrorInvalidValue;
    const int R = t.stream_ring;
    if (R < 4 || R > 36) return hipErrorInvalidValue;
    // wide (LDS-staged 8-byte) parity stores: measured faster only for the (5, 5) encode
    // (0.203 -> 0.180 ms; within +-5 % on the other presets)
    const bool wide_enc = !decode && t.const_enc && k == 5 && m == 5 && bb == 1352 &&
                          (((uintptr_t)out | (uintptr_t)out_gstride) & 7) == 0;
    const size_t lds = (size_t)kStreamWaves * ((R + kMirror) * 1024 + (wide_enc ? kStreamStage : 0));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int per_cu = (int)((160 * 1024) / lds);
    // units: (group, chunk of rc outputs); encode chunks of 8 for m > 8 (m <= 8: one chunk
    // of exactly m outputs), decode chunks of rc for rmax > rc
    const int s = bb / 8;
    const bool compiled = !decode && t.const_enc && gf_stream_compiled(k, m, bb);
    const int nchunk = decode ? (rmax + rc - 1) / rc
                              : (compiled || m <= 8 || (rc == 16 && m <= 16)) ? 1 : (m + 7) / 8;
    const long long units = groups * nchunk;
    const long long want = (units + kStreamWaves - 1) / kStreamWaves;
    long long cap = (long long)t.cus * per_cu;
    // oversubscribed: about swg units per wave ((250, 5) decode 5.02 -> 4.36 ms, DESIGN.md
    // section 4.5); large groups only by default
    const int swg = t.stream_wg >= 0 ? t.stream_wg : ((long long)k * bb >= 65536 ? 1 : 0);
    if (swg > 0) cap = (units + (long long)kStreamWaves * swg - 1) / ((long long)kStreamWaves * swg);
    if (t.stream_grid > 0) cap = t.stream_grid;          // tests: many groups per wave
    const unsigned grid = (unsigned)std::min<long long>(want, cap);
    const unsigned threads = kStreamWaves * 64;
    // the wave's 32-bit piece counters: cnt * NP, and (gf_ring) cnt groups
    {
        const long long waves = (long long)grid * kStreamWaves;
        const long long np = ((long long)k * bb + 8 + 1023) / 1024;
        if ((units + waves - 1) / waves * np >= (1LL << 31)) return hipErrorInvalidValue;
    }
#define QS_GO(RCV, SV, DEC, RCPV, KCV)                                                        \
    qlaunch((gf_stream_kernel<RCV, SV, DEC, RCPV, KCV>), dim3(grid), dim3(threads), \
                       lds, st, in, out, coef, slots, nout, groups, k, m, rmax, coef_gstride,   \
                       out_gstride, R, s, nchunk)
#define QS_GOJ(RCV, SV, DEC, RCPV, KCV)                                                       \
    qlaunch((gf_stream_kernel<RCV, SV, DEC, RCPV, KCV, true>), dim3(grid), dim3(threads), \
                       lds, st, in, out, coef, slots, nout, groups, k, m, rmax, coef_gstride,   \
                       out_gstride, R, s, nchunk)
#define QS_DECJ(SV)                                       \
    switch (rc) {                                         \
        case 2: QS_GOJ(2, SV, true, 4, 0); break;         \
        case 4: QS_GOJ(4, SV, true, 4, 0); break;         \
        case 8: QS_GOJ(8, SV, true, 8, 0); break;         \
        default: return hipErrorInvalidValue;             \
    }
#define QS_DEC(SV)                                        \
    switch (rc) {                                         \
        case 2: QS_GO(2, SV, true, 4, 0); break;          \
        case 4: QS_GO(4, SV, true, 4, 0); break;          \
        case 8: QS_GO(8, SV, true, 8, 0); break;          \
        default: return hipErrorInvalidValue;             \
    }
    // encode: one output per register set, RC = m; the table row stride is max(4, rc)
#define QS_ENC(SV)                                        \
    switch (m) {                                          \
        case 2: QS_GO(2, SV, false, 4, 0); break;         \
        case 3: QS_GO(3, SV, false, 4, 0); break;         \
        case 4: QS_GO(4, SV, false, 4, 0); break;         \
        case 5: QS_GO(5, SV, false, 8, 0); break;         \
        case 6: QS_GO(6, SV, false, 8, 0); break;         \
        case 7: QS_GO(7, SV, false, 8, 0); break;         \
        case 8: QS_GO(8, SV, false, 8, 0); break;         \
        default: QS_GO(8, SV, false, 8, 0); break;        \
    }
    // the static ring schedule is used for the encode only: its rolled decode measured
    // slower than gf_stream's (0.644 vs 0.619 ms on config B)
    const bool ring_shape = (k == 32 && m == 4) || (k == 10 && (m == 10 || m == 15 || m == 20)) ||
                            (k == 250 && m == 5) || (k == 15 && m == 15) || (k == 5 && m == 5);
    if (t.stream_static && !decode && s == 169 && ring_shape && t.const_enc) {
        // the fixed B/C shape and the even-k QuicR presets: compile-time ring schedule
        // (gf_ring_kernel)
        // wide (LDS-staged 8-byte) parity stores: 3 store instructions per block instead of
        // 16, so the group's store count stays under the 63 a counted wait can name.  Not for
        // (10, 20): 290 VGPRs, one wave per SIMD (0.754 vs 0.673 ms); B/C keep 4 x 16 stores
        // 
        // (10, 20) in two units of 10 parity rows per group (ring_split): 10 accumulators
        // per wave instead of 20, so wide stores fit the registers
        const bool rsplit = t.ring_split && k == 10 && m == 20;
        const bool rwide = t.ring_wide && !(k == 32 && m == 4) && (rsplit || !(k == 10 && m == 20)) &&
                           (((uintptr_t)out | (uintptr_t)out_gstride) & 7) == 0;
        const size_t rlds = (size_t)kRingWaves * (RingShape<169>::RB + (rwide ? kStreamStage : 0));
        const long long rwant = (groups * (rsplit ? 2 : 1) + kRingWaves - 1) / kRingWaves;
        long long rcap = (long long)t.cus * (int)((160 * 1024) / rlds);
        // oversubscribed: about rwg units per wave; measured faster for these encodes
        // (B 0.58 -> 0.55 ms, (10,10) 0.361 -> 0.330; (10,20) and (15,15) no better,
        // DESIGN.md section 4.5)
        const int rwg = t.ring_wg >= 0 ? t.ring_wg
                        : ((k == 32 && m == 4) || (k == 10 && m == 10) || (k == 5 && m == 5) ||
                           (k == 250 && m == 5)) ? 1 : 0;
        if (rwg > 0)
            rcap = (groups * (rsplit ? 2 : 1) + (long long)kRingWaves * rwg - 1) /
                   ((long long)kRingWaves * rwg);
        if (t.stream_grid > 0) rcap = t.stream_grid;
        const unsigned rgrid = (unsigned)std::min<long long>(rwant, rcap);
        if ((groups * (rsplit ? 2 : 1) + (long long)rgrid * kRingWaves - 1) / ((long long)rgrid * kRingWaves) >=
            (1LL << 31))
            return hipErrorInvalidValue;
        if (rsplit) {
            note_kernel("gf_ring_kernel<encode,k10m20,split>");
            if (rwide)
                qlaunch((gf_ring_kernel<10, 169, 10, false, 20, true, true, 2>), dim3(rgrid),
                        dim3(kRingWaves * 64), rlds, st, in, out, coef, slots, nout, groups, rmax,
                        coef_gstride, out_gstride);
            else
                qlaunch((gf_ring_kernel<10, 169, 10, false, 20, true, false, 2>), dim3(rgrid),
                        dim3(kRingWaves * 64), rlds, st, in, out, coef, slots, nout, groups, rmax,
                        coef_gstride, out_gstride);
            return hipGetLastError();
        }
#define QR_GO1(KV, MCV, WV)                                                                     \
    qlaunch((gf_ring_kernel<KV, 169, MCV, false, MCV, true, WV>), dim3(rgrid),                   \
                       dim3(kRingWaves * 64), rlds, st, in, out, coef, slots, nout, groups, rmax, \
                       coef_gstride, out_gstride)
#define QR_GO(KV, MCV)                  \
    do {                                \
        if (rwide) QR_GO1(KV, MCV, true); \
        else QR_GO1(KV, MCV, false);      \
    } while (0)
        // nt parity stores (plain: 0.673 vs 0.578 ms on B)
        switch (k * 256 + m) {
            case 32 * 256 + 4: note_kernel("gf_ring_kernel<encode,k32m4>"); QR_GO1(32, 4, false); break;
            case 10 * 256 + 10: note_kernel("gf_ring_kernel<encode,k10m10>"); QR_GO(10, 10); break;
            case 10 * 256 + 15: note_kernel("gf_ring_kernel<encode,k10m15>"); QR_GO(10, 15); break;
            case 250 * 256 + 5: note_kernel("gf_ring_kernel<encode,k250m5>"); QR_GO(250, 5); break;
            case 15 * 256 + 15: note_kernel("gf_ring_kernel<encode,k15m15>"); QR_GO(15, 15); break;
            case 5 * 256 + 5: note_kernel("gf_ring_kernel<encode,k5m5>"); QR_GO(5, 5); break;
            default: note_kernel("gf_ring_kernel<encode,k10m20>"); QR_GO1(10, 20, false); break;
        }
#undef QR_GO
#undef QR_GO1
        return hipGetLastError();
    }
    if (decode) {
        if (s == 169) {
            note_kernel("gf_stream_kernel<decode>");
            QS_DECJ(169)
        } else {
            note_kernel("gf_stream_kernel<decode,s>");
            QS_DEC(0)
        }
    } else {
        if (compiled) {
            // BASELINE configs B/C and the QuicR presets at 1350-byte payloads: the code is
            // fixed at compile time (windowed form, every output in one unit)
            note_kernel("gf_stream_kernel<encode,compiled>");
            if (wide_enc) {
                qlaunch((gf_stream_kernel<5, 169, false, 8, 5, false, true>), dim3(grid),
                        dim3(threads), lds, st, in, out, coef, slots, nout, groups, k, m, rmax,
                        coef_gstride, out_gstride, R, s, nchunk);
                return hipGetLastError();
            }
            switch (k * 256 + m) {
                case 32 * 256 + 4: QS_GO(4, 169, false, 4, 32); break;
                case 5 * 256 + 5: QS_GO(5, 169, false, 8, 5); break;
                case 10 * 256 + 10: QS_GO(10, 169, false, 12, 10); break;
                case 10 * 256 + 15: QS_GO(15, 169, false, 16, 10); break;
                case 10 * 256 + 20: QS_GO(20, 169, false, 20, 10); break;
                case 15 * 256 + 15: QS_GO(15, 169, false, 16, 15); break;
                case 250 * 256 + 5: QS_GO(5, 169, false, 8, 250); break;
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
        if (m > 8) {
            // one unit of up to 16 outputs (table rows of 16), or chunks of 8
            if (rc == 16 && m <= 16) {
                note_kernel(s == 169 ? "gf_stream_kernel<encode>" : "gf_stream_kernel<encode,s>");
                if (s == 169) QS_GO(16, 169, false, 16, 0);
                else QS_GO(16, 0, false, 16, 0);
                return hipGetLastError();
            }
            if (rc != 8) return hipErrorInvalidValue;
        } else if ((rc < 4 ? 4 : rc) != (m <= 4 ? 4 : 8)) {
            return hipErrorInvalidValue;
        }
        if (s == 169) {
            note_kernel("gf_stream_kernel<encode>");
            QS_ENC(169)
        } else {
            note_kernel("gf_stream_kernel<encode,s>");
            QS_ENC(0)
        }
    }
#undef QS_ENC
#undef QS_DEC
#undef QS_DECJ
#undef QS_GOJ
#undef QS_GO
    return hipGetLastError();
}

#endif
}  // namespace qfec
