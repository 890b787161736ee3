// gf_tile.hip — encode and decode of jumbo blocks: BASELINE config D,
// (128 data + 16 parity) x 9008 B blocks (9000 B payloads, quic_fec_group.cc:344-352).
//
// Same bit-sliced Cauchy arithmetic as gf_stream / gf_apply (cauchy_256.cpp:90-125,
// :1419-1601, W/Z nibble expansion of gf_bitslice.h).  What differs is the shape:
//
// * A sub-row is s = 1126 bytes = 282 column words, so one group spans NT = 5 column tiles
//   of 64 words, and 16 outputs need two chunks of 8 accumulators (8 outputs x 8 sub-rows
//   = 64 VGPRs).  A workgroup is NT x NCH waves (tile, chunk) that process ONE group at a
//   time, block by block, out of a shared LDS stream: the NPB = 9 one-KiB pieces of every
//   block are DMA'd (global_load_lds_dwordx4, nt) into one of D + 1 block buffers, spread
//   over the waves (each wave issues PPW pieces per block; where the pieces do not divide,
//   the last one is loaded twice into the same LDS bytes).  D blocks are in flight; a
//   wave waits with a counted `s_waitcnt vmcnt` for its own pieces of the next block, then
//   one s_barrier tells it every wave's pieces landed.  Each block is read from HBM once
//   (16-byte aligned pieces: bb % 16 == 0), its sub-rows are realigned in LDS (v_alignbyte),
//   and the waves of one workgroup stay within one block of each other, which keeps the
//   large unrolled encode program inside the instruction cache.
// * Encode of the compiled code (KC, MC) = (128, 16): the coefficients are compile-time
//   constants (cauchy_const.h, cauchy_256.cpp:422-480), the block loop is unrolled and every
//   8x8 expansion folds into straight-line XORs (the windowed form), with no scalar nibble
//   dispatch — about half the instructions of the run-time form, which is issue-bound on
//   this shape (and spills at the 10-wave occupancy; other codes stay on gf_apply).
// * Decode: gf_tile_syn_kernel below (syndromes of the same compiled code).
//
// vmcnt bookkeeping: per block a wave issues exactly PPW DMA instructions; per group it
// issues exactly RC * 8 * SPR stores (lanes of unused outputs dropped), so the count of
// VMEM instructions younger than the pieces of block b + 1 is (D - 1) * PPW, plus the
// group's stores for the first D - 1 blocks of a group (capped at 63: a smaller count only
// waits longer).  tests/test_isa.py checks that the compiler adds no VMEM instruction or
// vmcnt wait of its own.
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf_bitslice.h"

namespace qfec {

#define QT_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QT_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void tile_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_barrier with a compiler memory fence only (__syncthreads would also drain vmcnt,
// i.e. the whole DMA pipeline)
__device__ __forceinline__ void tile_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ int tile_sload_u8(const uint8_t* __restrict__ base, long long i) {
    const uint32_t wv = ((const uint32_t*)base)[i >> 2];
    return (int)((wv >> (8 * (i & 3))) & 0xFFu);
}

// byte i of a table the kernel never writes, through the scalar cache (constant address
// space: the compiler may not prove a pointer computed in a loop is read-only otherwise)
__device__ __forceinline__ int tile_cload_u8(const uint8_t* base, long long i) {
    const __attribute__((address_space(4))) uint32_t* p =
        (const __attribute__((address_space(4))) uint32_t*)(base);
    return (int)((p[i >> 2] >> (8 * (i & 3))) & 0xFFu);
}
__device__ __forceinline__ uint32_t tile_cload_u32(const uint8_t* base, int byte_off) {
    return ((const __attribute__((address_space(4))) uint32_t*)(base))[byte_off >> 2];
}

constexpr unsigned kTDrop = 0x80000000u;   // buffer offset past any range: lane dropped

// The lane id recomputed where it is used (v_mbcnt), in a volatile asm the compiler may not
// hoist: values derived from it at a group's end are not kept live (or spilled) across the
// block loop.
// (The host pass parses these bodies too, and an AMDGPU register constraint there would void
// the kernel's host stub; the asm is emitted for the device only.)
__device__ __forceinline__ int tile_lane_here() {
    int l = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
#endif
    return l;
}

// 16 bytes per lane from buffer rs at voff + soff into LDS at lds + 16 * lane (nt), i.e.
// buffer_load_dwordx4 ... lds: one VGPR of address (device only, as above: in a lambda the
// builtin voids the host stub)
__device__ __forceinline__ void tile_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds,
                                           uint32_t voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QT_LPTR(lds), 16, voff, soff, 0, 2);
#else
    (void)rs, (void)lds, (void)voff, (void)soff;
#endif
}

// an SGPR value made opaque to the optimiser (device only, as above)
__device__ __forceinline__ void tile_opaque_s(int& x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(x));
#else
    (void)x;
#endif
}

template <int S>
struct TileShape {
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4;          // column words per sub-row
    static constexpr int NWF = S / 4;               // full words
    static constexpr int NT = (NW + 63) / 64;       // column tiles (waves per chunk)
    static constexpr int NPB = (BB + 1023) / 1024;  // DMA pieces per block
    static constexpr int BBP = NPB * 1024;          // LDS bytes per block buffer
    static constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);   // stores per sub-row
};

// S: sub-row bytes (compile time).  RC: outputs per chunk wave, NCH chunks.  D: blocks in
// flight (D + 1 + BP LDS buffers).  Encode of the compiled code (k, m) = (KC, MC).
// BP: blocks per workgroup barrier (1, or 2: even steps wait for the next two blocks'
// pieces and pass one barrier for both; odd steps neither wait nor synchronise).
// DB: block b + 1's LDS reads are issued before block b is combined (register double
// buffer, 111 VGPRs: one 10-wave workgroup per CU).  !DB: a block is read right before it
// is combined and the kernel is held to 96 VGPRs, so two workgroups share a CU (5 waves per
// SIMD, the SIMDs evenly loaded; the other workgroup's waves hide the LDS latency).
template <int S, int RC, int NCH, int D, int KC, int MC, int BP = 1, bool DB = true>
__global__ __launch_bounds__(TileShape<S>::NT * NCH * 64, DB ? 3 : 5) void gf_tile_kernel(
    const uint8_t* in, uint8_t* out, long long groups, long long out_gstride) {
    using T = TileShape<S>;
    constexpr int BB = T::BB, NW = T::NW, NWF = T::NWF, NT = T::NT, NPB = T::NPB;
    constexpr int BBP = T::BBP, SPR = T::SPR;
    constexpr int NWV = NT * NCH;
    constexpr int PPW = (NPB + NWV - 1) / NWV;     // pieces per wave per block
    // D blocks in flight plus 1 + BP buffers: the one being read and those the slowest wave
    // may still have LDS reads outstanding on (a wave issues the DMA of block b + D after it
    // passed a barrier that every wave reached after consuming block b - 1 - BP)
    constexpr int NBUF = D + 1 + BP;
    constexpr int NST = RC * 8 * SPR;               // stores per wave per group
    // block b + 1's LDS reads are issued before block b is combined (register double buffer)
    constexpr int AHEAD = D - 1;                     // blocks issued after the awaited one
    constexpr int WAITN = AHEAD * PPW;
    constexpr int WAITG = AHEAD * PPW + NST > 63 ? 63 : AHEAD * PPW + NST;
    // pair barriers: an even step waits for block b + 2, with D - 2 blocks issued after it
    constexpr int WAITN2 = (D - 2) * PPW;
    constexpr int WAITG2 = (D - 2) * PPW + NST > 63 ? 63 : (D - 2) * PPW + NST;
    // !DB: the step waits for its own block (D issued after it), pairs for b + 1 (D - 1)
    constexpr int WAITNS = D * PPW;
    constexpr int WAITGS = D * PPW + NST > 63 ? 63 : D * PPW + NST;
    constexpr int WAITN2S = (D - 1) * PPW;
    constexpr int WAITG2S = (D - 1) * PPW + NST > 63 ? 63 : (D - 1) * PPW + NST;
    static_assert(DB || WAITNS <= 63, "pipeline depth");
    static_assert(BP == 1 || (BP == 2 && D >= 3 && KC % 2 == 0), "pair barriers");
    constexpr int SAUX = 2;                          // the dense parity stream: nt stores
    static_assert(S % 2 == 0 && BB % 16 == 0, "16-byte aligned blocks, 2-byte aligned sub-rows");
    static_assert(MC > 0 && (MC + RC - 1) / RC == NCH && KC % 2 == 0, "compiled code");
    static_assert(WAITN <= 63 && D >= 2, "pipeline depth");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    // wave-uniform (SGPRs: a VGPR copy of the chunk would be one more live register)
    const int tile = __builtin_amdgcn_readfirstlane(w % NT);
    const int chunk = __builtin_amdgcn_readfirstlane(w / NT);
    const int c = min(tile * 64 + lane, NW - 1);     // idle lanes shadow the last word
    constexpr int k = KC;
    const long long G0 = blockIdx.x, GS = gridDim.x;
    if (G0 >= groups) return;                        // uniform over the workgroup
    // wave-uniform 32-bit stream counters, in SGPRs (the launcher checks cnt * k < 2^31):
    // 64-bit or VGPR-resident counters cost a VALU compare and a branch per block
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - G0) / GS + 1));
    const int nblocks = cnt * k;                     // this workgroup's block stream

    // ---- DMA side: block b of the stream = block iss_x of group G0 + iss_i * GS, into
    // ring buffer iss_slot = b mod NBUF
    // The stream is extended past its end by re-reads of its last block (at most D of them),
    // so every block step issues, waits and reads the same way: no tail tests per block, and
    // the counted waits stay exact up to the last real block.
    int iss_slot = 0;
    int iss_x = 0;
    int iss_left = nblocks;                          // real blocks not issued yet
    const uint8_t* iss_src = in + G0 * (long long)k * BB;
    const long long gstride = GS * (long long)k * BB;
    // buffer_load ... lds: the group's base in a buffer resource (SGPRs), the block offset in
    // soffset, the lane's piece offset (fixed per wave) in one VGPR
    uint32_t voff[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int p = min(w + q * NWV, NPB - 1);   // surplus waves reload the last piece
        voff[q] = (uint32_t)min(p * 1024 + lane * 16, BB - 16);
    }
    auto issue_next = [&]() {
        uint8_t* dst = smem + iss_slot * BBP;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)iss_src, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int p = min(w + q * NWV, NPB - 1);
            tile_dma16(rs, dst + p * 1024, voff[q], iss_x * BB);
        }
        if (++iss_slot == NBUF) iss_slot = 0;
        if (--iss_left > 0 && ++iss_x == k) {        // after the last block: stay on it
            iss_x = 0;
            iss_src += gstride;
        }
    };

    // ---- LDS side: column word c of the 8 sub-rows of block b (aligned dwords; sub-row t
    // starts t * S bytes into the buffer, misaligned by (t * S) & 3, realigned at use)
    auto read_block = [&](int b, uint32_t (&lo)[8], uint32_t (&hi)[8]) {
        uint32_t c4 = 4u * (uint32_t)c;
        asm volatile("" : "+v"(c4));   // no hoisting across blocks
        const uint8_t* L = smem + (int)((unsigned)b % NBUF) * BBP + c4;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = t * S;
            const uint32_t* q = (const uint32_t*)(L + (o & ~3));
            lo[t] = q[0];
            hi[t] = (o & 3) ? q[1] : 0u;
        }
    };
    // wait for block bw's pieces (this wave's), then for every wave's
    auto wait_block = [&](bool after_stores) {
        if (after_stores) tile_wait_vmcnt<WAITG>();
        else tile_wait_vmcnt<WAITN>();
        tile_barrier();
    };

    static_assert(KC >= D, "a group covers the prefetch depth");
#pragma unroll 1
    for (int u = 0; u < D; ++u) issue_next();
    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
    if constexpr (DB) {
        wait_block(false);
        read_block(0, lo0, hi0);
    }

    int b = 0;   // stream index of the current block
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = G0 + i * GS;
        const int n = min(MC - chunk * RC, RC);      // chunk h owns outputs h * RC + j
        uint32_t acc[RC][8];
#pragma unroll
        for (int j = 0; j < RC; ++j)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[j][r] = 0;

        // one block: prefetch block b + D, pull block b + 1 into registers, combine block b
        // (xc: the block index in the group, an integral_constant)
        auto step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                        uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            issue_next();
            // blocks 0 .. D - 1 of a group were DMA'd before the previous group's stores
            // were issued, so those stores are younger than their pieces (past the stream's
            // last block this reads a re-read copy nobody uses)
            if constexpr (!DB) {
                // block b itself: D blocks issued after it; pair barriers wait at even steps
                // for blocks b and b + 1 (D - 1 after it; both of this group: KC is even)
                if constexpr (BP == 1) {
                    if (i > 0 && x <= D - 1) tile_wait_vmcnt<WAITGS>();
                    else tile_wait_vmcnt<WAITNS>();
                    tile_barrier();
                } else if constexpr (x % 2 == 0) {
                    if (i > 0 && x + 1 <= D - 1) tile_wait_vmcnt<WAITG2S>();
                    else tile_wait_vmcnt<WAITN2S>();
                    tile_barrier();
                }
                read_block(b, lo, hi);
            } else if constexpr (BP == 1) {
                wait_block(i > 0 && x + 1 <= D - 1);
            } else if constexpr (x % 2 == 0) {
                // blocks b + 1 and b + 2 (in order: waiting for b + 2 covers b + 1); block
                // x + 2 of this group, or block 0 of the next (whose preceding stores are
                // not issued yet)
                if (i > 0 && x + 2 <= D - 1) tile_wait_vmcnt<WAITG2>();
                else tile_wait_vmcnt<WAITN2>();
                tile_barrier();
            }
            if constexpr (DB) read_block(b + 1, nlo, nhi);
            ++b;
            WZ v;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                v.W[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
            // windowed form (gf_bitslice.h): one v_bitop3 per (output, sub-row); row 0 is P0,
            // all coefficients 1 (cauchy_256.cpp:1519-1523).  The blocks' common work (DMA,
            // waits, LDS reads, the combinations) is shared; only the apply differs per
            // chunk, behind a uniform branch.
            Win win;
            win_build(v.W8, win);
            // the chunk test on an SGPR value per block (a loop-invariant condition is kept
            // as a lane mask across the block loop, i.e. in a VGPR)
            int chv = chunk;
            tile_opaque_s(chv);
            static_for<NCH>([&](auto chc) __attribute__((always_inline)) {
                constexpr int CH = decltype(chc)::value;
                if (chv == CH) {
                    static_for<RC>([&](auto jc) __attribute__((always_inline)) {
                        constexpr int o = CH * RC + decltype(jc)::value;
                        if constexpr (o < MC)
                            win_apply<cauchy_coef(MC, o, x)>(acc[decltype(jc)::value], win);
                    });
                }
            });
        };
        static_for<KC>([&](auto xc) __attribute__((always_inline)) {
            // accumulators opaque at every block boundary: with constant coefficients the
            // XOR reassociation would otherwise merge the blocks' sums into one tree and keep
            // every block's combinations live
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[j][r]));
            // and no instruction scheduled across blocks (register pressure)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!DB || decltype(xc)::value % 2 == 0)
                step(xc, lo0, hi0, lo1, hi1);
            else
                step(xc, lo1, hi1, lo0, hi0);
        });
        // KC is even: the next group's first block is in lo0/hi0 again (DB)

        // ---- outputs: a fixed number of store instructions (unused outputs, idle lanes
        // and the lanes outside a word's valid bytes are dropped)
        // Lane offsets: 4c for the full words, the tail word's lane, everyone else dropped;
        // the sub-row goes into the scalar offset and an unused output gets an empty range,
        // so the whole phase needs two VGPRs of addresses (opaque: not hoisted out of the
        // group loop as 8 x RC precomputed offsets).
        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
        const int lane_e = tile_lane_here();
        const bool live = tile * 64 + lane_e < NW;
        uint32_t vo = live && c < NWF ? 4u * (uint32_t)c : kTDrop;
        uint32_t vt = live && c == NWF && NWF < NW ? 4u * (uint32_t)c : kTDrop;
        asm volatile("" : "+v"(vo), "+v"(vt));
#pragma unroll
        for (int j = 0; j < RC; ++j) {
            const bool on = j < n;
            uint8_t* dst = out + g * out_gstride + (long long)(chunk * RC + j) * BB;
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
    }
    tile_wait_vmcnt<0>();
}

// ------------------------------------------------------------------ syndrome decode
// Decode of the compiled (128, 16) code in the reference's order (cauchy_256.cpp:1269-1420:
// the received originals are eliminated from the recovery rows, then the r x r system is
// solved).  With y_i the parity row of received recovery block R_i:
//   T_i = R_i ^ sum_{data slots s} C[y_i][row_s] D_s        (syndromes, C compile-time)
//   E_j = sum_i Sinv[j][i] T_i                               (once per group, run time)
// The block pass runs the windowed form of the compiled encode (one v_bitop3 per (syndrome
// row, sub-row)) for the received parity rows only, instead of r run-time coefficients per
// block through the scalar nibble dispatch; the r x r solve costs r^2 nibble applies per
// group against 128 block steps.
// Stream: the prep's syndrome table (fec_kernels.h, syn::) orders each group's k slots as
// the present data rows ascending, then the extras (recovery blocks, repeated data rows).
// The unrolled block loop tests row x's present bit and consumes the next streamed block
// only if it is set, so the coefficients stay compile-time; an erased row moves the waiting
// block to the other register set instead.
// Waves: NT column tiles x 2 chunks; chunk h owns syndrome rows y = 2t + h and outputs
// j = 2q + h (t, q < 8), so the usual losses (the first r parity rows received) split
// evenly.  Syndromes cross chunks through LDS after the block ring, 8 at a time.
template <int S, int D>
__global__ __launch_bounds__(TileShape<S>::NT * 2 * 64, (TileShape<S>::NT * 2 + 3) / 4) void
gf_tile_syn_kernel(const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
                   const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout,
                   const uint8_t* __restrict__ cenc, long long groups, int rmax,
                   long long tab_gstride, long long out_gstride) {
    using T = TileShape<S>;
    constexpr int KC = 128, MC = 16, NCH = 2;
    constexpr int ROWS = MC / NCH;                  // syndrome rows y = NCH * t + chunk
    constexpr int RO = MC / NCH;                    // outputs j = NCH * q + chunk
    constexpr int TH = 8;                           // syndromes per LDS exchange round
    constexpr int BB = T::BB, NW = T::NW, NWF = T::NWF, NT = T::NT, NPB = T::NPB;
    constexpr int BBP = T::BBP, SPR = T::SPR;
    constexpr int NWV = NT * NCH;
    constexpr int PPW = (NPB + NWV - 1) / NWV;
    constexpr int NBUF = D + 2;
    constexpr int NST = RO * 8 * SPR;               // stores per wave per group
    constexpr int AHEAD = D - 1;
    constexpr int WAITN = AHEAD * PPW;
    constexpr int WAITG = AHEAD * PPW + NST > 63 ? 63 : AHEAD * PPW + NST;
    static_assert(WAITN <= 63 && D >= 2, "pipeline depth");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* tl = (uint32_t*)(smem + NBUF * BBP);  // [TH][NT][8][64] syndrome words

    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    // wave-uniform (SGPRs: a VGPR copy of the chunk would be one more live register)
    const int tile = __builtin_amdgcn_readfirstlane(w % NT);
    const int chunk = __builtin_amdgcn_readfirstlane(w / NT);
    const int c = min(tile * 64 + lane, NW - 1);
    const long long G0 = blockIdx.x, GS = gridDim.x;
    if (G0 >= groups) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - G0) / GS + 1));
    const int nblocks = cnt * KC;                    // 32-bit, in SGPRs (see gf_tile_kernel)

    // ---- DMA side: stream block x of group G0 + i * GS = its slot perm[x]
    int iss_slot = 0;
    int iss_x = 0;
    int iss_left = nblocks;                          // real blocks not issued yet (see above)
    const uint8_t* iss_src = in + G0 * (long long)KC * BB;
    const uint8_t* iss_tab = tab + G0 * tab_gstride;
    const long long gstride = GS * (long long)KC * BB;
    // the stream-order bytes come 4 at a time: one scalar load (and its lgkmcnt wait) per
    // four issued blocks instead of one per block (KC % 4 == 0: a word never spans groups)
    uint32_t perm_w = 0;
    static_assert(KC % 4 == 0 && syn::kPerm % 4 == 0, "stream-order words");
    auto issue_next = [&]() __attribute__((always_inline)) {
        uint8_t* dst = smem + iss_slot * BBP;
        if ((iss_x & 3) == 0) perm_w = tile_cload_u32(iss_tab, syn::kPerm + iss_x);
        const int slot = min((int)((perm_w >> (8 * (iss_x & 3))) & 0xFFu), KC - 1);
        const uint8_t* src = iss_src + (long long)slot * BB;
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int p = min(w + q * NWV, NPB - 1);
            const int off = min(p * 1024 + lane * 16, BB - 16);
            __builtin_amdgcn_global_load_lds(QT_GPTR(src + off), QT_LPTR(dst + p * 1024), 16, 0,
                                             2);
        }
        if (++iss_slot == NBUF) iss_slot = 0;
        if (--iss_left > 0 && ++iss_x == KC) {
            iss_x = 0;
            iss_src += gstride;
            iss_tab += GS * tab_gstride;
        }
    };
    auto read_block = [&](int bi, uint32_t (&lo)[8], uint32_t (&hi)[8])
                          __attribute__((always_inline)) {
        uint32_t c4 = 4u * (uint32_t)c;
        asm volatile("" : "+v"(c4));   // no hoisting across blocks
        const uint8_t* L = smem + (int)((unsigned)bi % NBUF) * BBP + c4;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = t * S;
            const uint32_t* q = (const uint32_t*)(L + (o & ~3));
            lo[t] = q[0];
            hi[t] = (o & 3) ? q[1] : 0u;
        }
    };
    auto wait_block = [&](bool after_stores) __attribute__((always_inline)) {
        if (after_stores) tile_wait_vmcnt<WAITG>();
        else tile_wait_vmcnt<WAITN>();
        tile_barrier();
    };

#pragma unroll 1
    for (int u = 0; u < D; ++u) issue_next();
    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
    wait_block(false);
    read_block(0, lo0, hi0);

    int b = 0;
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = G0 + i * GS;
        const uint8_t* tb = tab + g * tab_gstride;
        uint32_t pm[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pm[q] = tile_cload_u32(tb, syn::kMask + 4 * q);
        const uint32_t need = tile_cload_u32(tb, syn::kNeed);
        const int n = min(nout[g], rmax);
        const int ne = KC - (__builtin_popcount(pm[0]) + __builtin_popcount(pm[1]) +
                             __builtin_popcount(pm[2]) + __builtin_popcount(pm[3]));
        uint32_t acc[ROWS][8];
#pragma unroll
        for (int t = 0; t < ROWS; ++t)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[t][r] = 0;

        // next block: prefetch block b + D, pull block b + 1 into (nlo, nhi); returns the
        // realigned words of block b
        auto advance = [&](const uint32_t (&lo)[8], const uint32_t (&hi)[8], uint32_t (&nlo)[8],
                           uint32_t (&nhi)[8], uint32_t (&wv)[8]) __attribute__((always_inline)) {
            issue_next();
            // positions 0 .. D - 1 of a group were DMA'd before the previous group's stores
            // were issued, so those stores are younger than their pieces
            const int p1 = b + 1 - i * KC;
            wait_block(i > 0 && p1 <= D - 1);
            read_block(b + 1, nlo, nhi);
            ++b;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                wv[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
        };
        // data row x (compile time): its block, if present, into every received syndrome row
        auto row_step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                            uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            if ((pm[x >> 5] >> (x & 31)) & 1u) {
                uint32_t wv[8];
                advance(lo, hi, nlo, nhi, wv);
                Win win;
                win_build(wv, win);
                static_for<NCH>([&](auto chc) __attribute__((always_inline)) {
                    constexpr int CH = decltype(chc)::value;
                    if (chunk == CH) {
                        static_for<ROWS>([&](auto tc) __attribute__((always_inline)) {
                            constexpr int t = decltype(tc)::value, y = NCH * t + CH;
                            if ((need >> y) & 1u)
                                win_apply<cauchy_coef(MC, y, x)>(acc[t], win);
                        });
                    }
                });
            } else {
                // row x erased: the block waiting in (lo, hi) is row x + 1's
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    nlo[t] = lo[t];
                    nhi[t] = hi[t];
                }
            }
        };
        static_for<KC>([&](auto xc) __attribute__((always_inline)) {
            // accumulators opaque at every block boundary (see gf_tile_kernel)
#pragma unroll
            for (int t = 0; t < ROWS; ++t)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[t][r]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(xc)::value % 2 == 0)
                row_step(xc, lo0, hi0, lo1, hi1);
            else
                row_step(xc, lo1, hi1, lo0, hi0);
        });
        static_assert(KC % 2 == 0, "register double buffer parity");

        // extras: a received parity row y adds its block to T_y; a repeated data row adds
        // C[y][row] times its block to every syndrome row (run-time coefficients)
        auto extra = [&](int e, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                         uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            WZ v;
            advance(lo, hi, nlo, nhi, v.W8);
            const int row = tile_cload_u8(tb + syn::kERow, e);
            if (row >= KC) {
                // a mask per row, not a branch: `if (y == 2t + h) acc[t] ^= ...` is folded
                // into a computed index, which sends acc to scratch memory
                const uint32_t ybit = 1u << (row - KC);
                static_for<NCH>([&](auto chc) __attribute__((always_inline)) {
                    constexpr int CH = decltype(chc)::value;
                    if (chunk == CH) {
                        static_for<ROWS>([&](auto tc) __attribute__((always_inline)) {
                            constexpr int t = decltype(tc)::value, y = NCH * t + CH;
                            if ((need >> y) & 1u) {
                                const uint32_t mk = (ybit >> y) & 1u ? ~0u : 0u;
#pragma unroll
                                for (int r = 0; r < 8; ++r)
                                    acc[t][r] ^= v.W[r] & mk;
                            }
                        });
                    }
                });
            } else {
                expand_wz(v);
                static_for<NCH>([&](auto chc) __attribute__((always_inline)) {
                    constexpr int CH = decltype(chc)::value;
                    if (chunk == CH) {
                        static_for<ROWS>([&](auto tc) __attribute__((always_inline)) {
                            constexpr int t = decltype(tc)::value, y = NCH * t + CH;
                            if ((need >> y) & 1u) {
                                const uint32_t cf = (uint32_t)tile_cload_u8(cenc, y * KC + row);
                                apply_nibble<0>(acc[t], cf & 15u, v);
                                apply_nibble<4>(acc[t], cf >> 4, v);
                            }
                        });
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

        // ---- E_j = sum_i Sinv[j][i] T_i.  The syndromes go through LDS, TH per round.  Up
        // to NCH * 4 outputs (the usual case): one round, 4 outputs per wave.  More: passes of
        // 2 outputs per wave over every round, so that only 2 x 8 output words are live next
        // to the syndrome rows still to be exchanged (no spills at 3 waves per SIMD).  Every
        // path issues the same store count (outputs past n with an empty range).
        uint32_t* tlw = tl + tile * 8 * 64 + lane;   // + (i * NT * 8 + r) * 64
        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
        const int lane_e = tile_lane_here();
        const bool live = tile * 64 + lane_e < NW;
        uint32_t vo = live && c < NWF ? 4u * (uint32_t)c : kTDrop;
        uint32_t vt = live && c == NWF && NWF < NW ? 4u * (uint32_t)c : kTDrop;
        asm volatile("" : "+v"(vo), "+v"(vt));
        // this wave's syndromes i in [h0, h0 + TH) to LDS, then a workgroup barrier
        auto exchange = [&](int h0) __attribute__((always_inline)) {
            static_for<NCH>([&](auto chc) __attribute__((always_inline)) {
                constexpr int CH = decltype(chc)::value;
                if (chunk == CH) {
                    static_for<ROWS>([&](auto tc) __attribute__((always_inline)) {
                        constexpr int t = decltype(tc)::value, y = NCH * t + CH;
                        if ((need >> y) & 1u) {
                            const int ii = tile_cload_u8(tb + syn::kISlot, y) - h0;
                            if (ii >= 0 && ii < TH) {
#pragma unroll
                                for (int r = 0; r < 8; ++r) tlw[(ii * NT * 8 + r) * 64] = acc[t][r];
                            }
                        }
                    });
                }
            });
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            tile_barrier();
        };
        // o[q] ^= Sinv[j][i] T_i for the round's syndromes, outputs j = NCH * (q0 + q) + chunk
        auto solve = [&](int h0, int q0, auto& o) __attribute__((always_inline)) {
            constexpr int NQ = sizeof(o) / sizeof(o[0]);
            // rolled: the branchy nibble dispatch stays a small loop body in the instruction
            // cache (the unrolled block pass before it has evicted everything else)
            const int iend = min(TH, n - h0);
#pragma unroll 1
            for (int ii = 0; ii < iend; ++ii) {
                WZ v;
#pragma unroll
                for (int r = 0; r < 8; ++r) v.W[r] = tlw[(ii * NT * 8 + r) * 64];
                expand_wz(v);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int j = NCH * (q0 + q) + chunk;
                    if (j < n) {
                        const uint32_t cf =
                            (uint32_t)tile_cload_u8(tb + syn::kSinv, j * 16 + h0 + ii);
                        apply_nibble<0>(o[q], cf & 15u, v);
                        apply_nibble<4>(o[q], cf >> 4, v);
                    }
                }
            }
        };
        // outputs q0 .. q0 + NQ - 1 of this wave (a fixed number of store instructions)
        auto store = [&](int q0, const auto& o) __attribute__((always_inline)) {
            constexpr int NQ = sizeof(o) / sizeof(o[0]);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int j = NCH * (q0 + q) + chunk;
                const bool on = j < n;
                const int oslot = slots ? (on ? tile_sload_u8(slots, g * rmax + j) : 0) : j;
                uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    dst, 0, on ? (unsigned)BB : 0u, 0x00020000);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint32_t vsum = o[q][r];
                    __builtin_amdgcn_raw_buffer_store_b32(vsum, rs, vo, r * S, 0);
                    if (S & 2)
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)vsum, rs, vt, r * S, 0);
                    if (S & 1)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(vsum >> (8 * (S & 2))), rs,
                                                             vt, r * S + (S & 2), 0);
                }
            }
            asm volatile("" ::: "memory");
        };
        static_assert(RO == 8 && TH == NCH * 4, "output passes");
        if (n <= TH) {
            uint32_t o[4][8];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 8; ++r) o[q][r] = 0;
            if (n > 0) {   // uniform: the barrier
                exchange(0);
                solve(0, 0, o);
            }
            store(0, o);
            store(4, o);   // q >= 4: no output (j >= 8 >= n), empty range
        } else {
            static_for<4>([&](auto pc) __attribute__((always_inline)) {
                constexpr int q0 = 2 * decltype(pc)::value;
                uint32_t o[2][8];
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int r = 0; r < 8; ++r) o[q][r] = 0;
#pragma unroll 1
                for (int h0 = 0; h0 < n; h0 += TH) {
                    exchange(h0);
                    solve(h0, q0, o);
                    // every wave has read this round before the next one rewrites the area
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    tile_barrier();
                }
                store(q0, o);
            });
        }
    }
    tile_wait_vmcnt<0>();
}

namespace {
constexpr int kTileS = 1126;   // bb = 9008: 9000-byte payloads (BASELINE config D)
}  // namespace

bool gf_tile_supported(int k, int m, int bb, const Tune& t) {
    return t.tile && t.const_enc && k == 128 && m == 16 && bb == 8 * kTileS;
}

hipError_t launch_gf_tile_encode(const uint8_t* in, uint8_t* out, int k, int m, int bb,
                                 long long groups, long long out_gstride, hipStream_t st,
                                 const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_tile_supported(k, m, bb, t)) return hipErrorInvalidValue;
    if (((uintptr_t)in & 15) != 0) return hipErrorInvalidValue;
    if (t.tile_depth != 4 && t.tile_depth != 6 && !(t.tile_occ2 && t.tile_depth == 5))
        return hipErrorInvalidValue;
    const bool pair = t.tile_pair && t.tile_depth >= 5;   // depth 4: one barrier per block
    using TS = TileShape<kTileS>;
    constexpr int nch = 2;
    const int bp = pair ? 2 : 1;
    const size_t lds = (size_t)(t.tile_depth + 1 + bp) * TS::BBP;
    const unsigned threads = (unsigned)(TS::NT * nch * 64);
    // workgroups per CU: LDS and waves (<= 128 VGPRs: 16 waves; occ2: <= 96 VGPRs, 20 waves)
    const int wave_cap = t.tile_occ2 ? 20 : 16;
    const int per_cu = std::max(1, std::min((int)((160 * 1024) / lds), wave_cap / (TS::NT * nch)));
    long long cap = (long long)t.cus * per_cu;
    if (t.tile_grid > 0) cap = t.tile_grid;              // tests: many groups per workgroup
    const unsigned grid = (unsigned)std::min<long long>(groups, cap);
    if ((groups + grid - 1) / grid * k >= (1LL << 31)) return hipErrorInvalidValue;
    note_kernel(t.tile_occ2 ? "gf_tile_kernel<encode,k128m16,occ2>" : "gf_tile_kernel<encode,k128m16>");
    if (t.tile_occ2) {
        // two workgroups per CU: LDS <= 80 KB each, the register double buffer dropped
        if (lds > 80 * 1024) return hipErrorInvalidValue;
        if (pair && t.tile_depth == 5)
            qlaunch((gf_tile_kernel<kTileS, 8, nch, 5, 128, 16, 2, false>), dim3(grid),
                    dim3(threads), lds, st, in, out, groups, out_gstride);
        else if (!pair && t.tile_depth == 6)
            qlaunch((gf_tile_kernel<kTileS, 8, nch, 6, 128, 16, 1, false>), dim3(grid),
                    dim3(threads), lds, st, in, out, groups, out_gstride);
        else if (!pair && t.tile_depth == 4)
            qlaunch((gf_tile_kernel<kTileS, 8, nch, 4, 128, 16, 1, false>), dim3(grid),
                    dim3(threads), lds, st, in, out, groups, out_gstride);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (t.tile_depth == 5) return hipErrorInvalidValue;
    if (pair)
        qlaunch((gf_tile_kernel<kTileS, 8, nch, 6, 128, 16, 2>), dim3(grid), dim3(threads),
                lds, st, in, out, groups, out_gstride);
    else if (t.tile_depth == 4)
        qlaunch((gf_tile_kernel<kTileS, 8, nch, 4, 128, 16>), dim3(grid), dim3(threads),
                           lds, st, in, out, groups, out_gstride);
    else
        qlaunch((gf_tile_kernel<kTileS, 8, nch, 6, 128, 16>), dim3(grid), dim3(threads),
                           lds, st, in, out, groups, out_gstride);
    return hipGetLastError();
}

bool gf_tile_syndrome_supported(int k, int m, int bb, int rmax, const Tune& t) {
    return gf_tile_supported(k, m, bb, t) && rmax <= 16;
}

hipError_t launch_gf_tile_syndrome(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                                   const uint8_t* slots, const int32_t* nout,
                                   const uint8_t* cenc, int k, int m, int bb, long long groups,
                                   int rmax, long long tab_gstride, long long out_gstride,
                                   hipStream_t st, const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_tile_syndrome_supported(k, m, bb, rmax, t) || tab_gstride < syn::kBytes)
        return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)tab_gstride |
                                     (uintptr_t)cenc | (uintptr_t)slots) & 3))
        return hipErrorInvalidValue;
    using TS = TileShape<kTileS>;
    constexpr int D = 6;
    const size_t lds = (size_t)(D + 2) * TS::BBP + (size_t)8 * TS::NT * 8 * 64 * 4;
    const unsigned threads = (unsigned)(TS::NT * 2 * 64);
    long long cap = (long long)t.cus * std::max(1, (int)((160 * 1024) / lds));
    if (t.tile_grid > 0) cap = t.tile_grid;
    const unsigned grid = (unsigned)std::min<long long>(groups, cap);
    if ((groups + grid - 1) / grid * k >= (1LL << 31)) return hipErrorInvalidValue;
    note_kernel("gf_tile_syn_kernel<decode,k128m16>");
    qlaunch((gf_tile_syn_kernel<kTileS, D>), dim3(grid), dim3(threads), lds, st, in,
                       out, tab, slots, nout, cenc, groups, rmax, tab_gstride, out_gstride);
    return hipGetLastError();
}

}  // namespace qfec
