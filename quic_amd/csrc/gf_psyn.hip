// gf_psyn.hip — syndrome decode of the QuicR preset codes at 1350-byte payloads:
// FEC_10_10, FEC_10_15, FEC_10_20, FEC_15_15 (quic_fec_group.cc:22-82), bb = 1352, any
// erasure count up to min(k, m).
//
// The reference decodes in two stages (cauchy_256_decode, cauchy_256.cpp:1269-1420; for
// more than 4 erasures its windowed forms win_original :578-653 and
// win_gaussian_elimination :809-1018): eliminate the received originals from the recovery
// rows, then solve the r x r system over the erased rows.  Here, with y_s the received
// parity rows sorted ascending and e_j the erased data rows ascending:
//   T_y = R_y ^ sum_{present x} C[y][x] D_x          syndromes of ALL m parity rows, with
//                                                    the compile-time coefficients of the
//                                                    preset code (windowed form, one
//                                                    v_bitop3 per (row, sub-row), no
//                                                    scalar dispatch)
//   T_s <- T_{y_s}                                   in place: y_s >= s, ascending
//   Gauss-Jordan on S[s][j] = C[y_s][e_j], replayed on the data in place: for pivot p,
//   T_i ^= g[p][i] * T_p for every slot i (g[p][p] = 1 ^ 1/S'[p][p] normalises the pivot
//   row by linearity), one W/Z expansion of T_p per pivot, r^2 run-time applies per group
//   T_j = E_{e_j}
// For m >= 7 the reference's matrix is C[y][x] = b_x / (b_x + g_y) (cauchy_256.cpp:
// 459-477; row 0, all ones, is g_0 = 0 and b_0 = 1): a column-scaled Cauchy matrix with
// distinct nodes (checked for these codes by tests/test_psyn_prep.py), so every square
// submatrix of it is nonsingular and the elimination needs no pivoting in any row order.
// The recovered bytes are the unique solution, so the result is bit-exact with the
// reference's bit-matrix elimination.  A zero pivot can only come from a malformed receive
// set (a repeated parity row): status -3, group unchanged, as in every other decode here.
//
// Against the run-time decode it replaces (gf_stream_kernel<decode>, k x r run-time applies
// with two scalar nibble dispatches each): (10, 10) at 5 losses goes from 50 run-time
// applies per group to 25, and the other 5 x 10 row contributions are compile-time.
//
// Stream: as gf_bsyn (every wave owns groups g0, g0 + W, ...; a group's k received blocks in
// the prep table's order: present data rows ascending, then the extras in slot order; each
// block's 16-byte aligned envelope DMA'd into a ring of D + 1 block buffers, read at its
// 8-byte skew).  Groups of odd k start 8 bytes off a 16-byte boundary; the block address
// decides the skew.  Loads go through a buffer resource bounded by the end of the input, so
// the envelope of the last block of the buffer reads zeros past it.
//
// vmcnt bookkeeping as in gf_bsyn: a block is NPC DMA instructions; a group's stores
// (8 * SPR per recovered block) sit in the count before the waits for the next group's
// blocks 1 .. D - 1.  tests/test_isa.py checks the compiler adds no VMEM instruction or
// vmcnt wait of its own.
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf256.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

#define QP_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void psyn_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void psyn_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds, uint32_t voff,
                                           int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QP_LPTR(lds), 16, voff, soff, 0, 2);
#else
    (void)rs, (void)lds, (void)voff, (void)soff;
#endif
}

__device__ __forceinline__ uint32_t psyn_cload_u32(const uint8_t* base, int byte_off) {
    return ((const __attribute__((address_space(4))) uint32_t*)(base))[byte_off >> 2];
}

// f(integral_constant<int, v>) for the run-time v in [LO, HI]: a binary tree of uniform
// branches, so register arrays can be indexed by a wave-uniform value
template <int LO, int HI, class F>
__device__ __forceinline__ void psyn_dispatch(int v, F&& f) {
    if constexpr (LO == HI) {
        f(std::integral_constant<int, LO>{});
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (v <= MID) psyn_dispatch<LO, MID>(v, f);
        else psyn_dispatch<MID + 1, HI>(v, f);
    }
}

// s_waitcnt vmcnt(min(63, BASE + PER * n)) for a wave-uniform n >= 0
template <int BASE, int PER, int N = 0>
__device__ __forceinline__ void psyn_wait_stores(int n) {
    constexpr int W = BASE + PER * N > 63 ? 63 : BASE + PER * N;
    if constexpr (W == 63) {
        psyn_wait_vmcnt<63>();
    } else {
        if (n <= N) psyn_wait_vmcnt<W>();
        else psyn_wait_stores<BASE, PER, N + 1>(n);
    }
}

constexpr unsigned kPDrop = 0x80000000u;   // buffer offset past any range: lane dropped

__constant__ GfTables c_gf_psyn = make_gf_tables();   // this code object's copy

template <int S>
struct PsynShape {
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4, NWF = S / 4;
    static constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);   // stores per sub-row
    static constexpr int BUFB = (BB + 8 + 15) / 16 * 16;        // the 16-byte envelope
    static constexpr int NPC = BUFB > 1024 ? 2 : 1;              // DMA instructions per block
    static constexpr int P1L = BUFB > 1024 ? (BUFB - 1024) / 16 : 0;   // lanes of the 2nd
};

constexpr int kPsynWaves = 4;   // waves per workgroup (independent)

// KC, MC: the compiled code (k, m); RC = min(k, m): recovered blocks at most; S: sub-row
// bytes; D: blocks in flight per wave; PF: block b + 1 is read from LDS into registers while
// block b is combined (16 more VGPRs; without, each block is read when its turn comes and
// the other waves of the SIMD cover the LDS latency).  JUMP: the solve's run-time products go
// (1) through one indirect jump into a table of 256 leaves (gf_winjump.h win_mul_rt) into a
// temporary scattered to its slot, or (2) through two nibble jumps straight into the slot's
// accumulator (wz_mul_acc_rt, one call site per slot), instead of (0) a 256-way tree of
// uniform branches.  Bit 2 of JUMP (4): the recovered blocks are stored non-temporal (dec_nt).
// Bits 3 and 4 (8, 16) are timing probes only (psyn_ablate; results wrong): no stores, no
// arithmetic (each block XORed into one accumulator, no solve).
template <int KC, int MC, int RC, int S, int D, bool PF, int JUMP>
__global__ __launch_bounds__(kPsynWaves * 64) void gf_psyn_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
    const uint8_t* __restrict__ cenc, const uint8_t* __restrict__ slots,
    const int32_t* __restrict__ nout, long long groups, int rmax, long long out_gstride) {
    using SH = PsynShape<S>;
    constexpr int BB = SH::BB, NW = SH::NW, NWF = SH::NWF, SPR = SH::SPR;
    constexpr int BUFB = SH::BUFB, NPC = SH::NPC, P1L = SH::P1L;
    constexpr int NB = D + 1;                 // the block being read + D in flight
    constexpr int WAITN = (D - 1) * NPC;      // younger than block b + 1 when it is awaited
    constexpr int WAITNF = D * NPC;           // (no PF) younger than block b when it is awaited
    static_assert(WAITN <= 63 && D >= 2 && KC >= D, "pipeline depth");
    static_assert(KC <= 64 && MC <= 32 && RC <= 16 && RC <= KC && RC <= MC && BB % 8 == 0 &&
                      NB <= 32,
                  "compiled small-block code");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    uint8_t* ring = smem + (size_t)w * NB * BUFB;
    constexpr int SA = (JUMP & 4) ? 2 : 0;    // recovered blocks stored non-temporal (dec_nt)
    const long long W = (long long)gridDim.x * kPsynWaves;
    const long long g0 = (long long)blockIdx.x * kPsynWaves + w;
    if (g0 >= groups) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));
    const int c = lane < NW ? lane : NW - 1;  // idle lanes shadow the last word
    constexpr long long GB = (long long)KC * BB;
    const long long in_bytes = groups * GB;

    // ---- DMA side: stream block b = position iss_x of group g0 + i * W, the slot the table
    // names there, into ring buffer iss_buf; bit iss_buf of `skew` = its 8-byte skew.  Past
    // the stream's end the last block is re-read (every step issues and waits the same way).
    int iss_buf = 0, iss_x = 0;
    int iss_left = cnt * KC;
    long long iss_a = g0 * GB;                              // the group's byte offset
    const uint8_t* iss_t = tab + g0 * (long long)psyn::kBytes;
    const long long gstride = W * GB;
    const long long tstride = W * (long long)psyn::kBytes;
    uint32_t perm_w = 0, skew = 0;
    auto issue_next = [&]() __attribute__((always_inline)) {
        if ((iss_x & 3) == 0) perm_w = psyn_cload_u32(iss_t, psyn::kPerm + iss_x);
        const int slot = min((int)((perm_w >> (8 * (iss_x & 3))) & 0xFFu), KC - 1);
        const long long a = iss_a + (long long)slot * BB;   // the block's byte offset
        const long long a16 = a & ~15LL;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(in + a16), 0, (unsigned)min(in_bytes - a16, 0x7FFFFFF0LL), 0x00020000);
        uint8_t* dst = ring + iss_buf * BUFB;
        psyn_dma16(rs, dst, 16u * (uint32_t)lane, 0);
        if constexpr (NPC == 2)
            if (lane < P1L) psyn_dma16(rs, dst + 1024, 1024u + 16u * (uint32_t)lane, 0);
        skew = (a & 15) ? (skew | (1u << iss_buf)) : (skew & ~(1u << iss_buf));
        if (++iss_buf == NB) iss_buf = 0;
        if (--iss_left > 0 && ++iss_x == KC) {
            iss_x = 0;
            iss_a += gstride;
            iss_t += tstride;
        }
    };
    // column word c of the 8 sub-rows of stream block bi: aligned dwords (the buffer start
    // plus the skew is 8-byte aligned, sub-row t is misaligned by the constant (t*S) & 3)
    auto read_block = [&](int bi, uint32_t (&lo)[8], uint32_t (&hi)[8])
                          __attribute__((always_inline)) {
        const int buf = (int)((unsigned)bi % NB);
        uint32_t a = 4u * (uint32_t)c + (uint32_t)(buf * BUFB) + (((skew >> buf) & 1u) << 3);
        asm volatile("" : "+v"(a));   // no hoisting across blocks
        const uint8_t* L = ring + a;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int o = t * S;
            const uint32_t* q = (const uint32_t*)(L + (o & ~3));
            lo[t] = q[0];
            hi[t] = (o & 3) ? q[1] : 0u;
        }
    };

#pragma unroll 1
    for (int u = 0; u < D; ++u) issue_next();
    uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
    if constexpr (PF) {
        psyn_wait_vmcnt<WAITN>();
        read_block(0, lo0, hi0);
    }

    int b = 0;        // stream index of the block in (lo0, hi0) / the current block
    int prev_n = -1;  // recovered blocks the previous group stored (-1: no previous group)
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = g0 + (long long)i * W;
        const uint8_t* tb = tab + g * (long long)psyn::kBytes;
        const uint32_t mlo = psyn_cload_u32(tb, psyn::kMask), mhi = psyn_cload_u32(tb, psyn::kMask + 4);
        const int n = min(min(nout[g], rmax), RC);
        const int ne = KC - __builtin_popcount(mlo) - __builtin_popcount(mhi);
        int p = 0;    // blocks of this group consumed
        uint32_t acc[MC][8];
#pragma unroll
        for (int y = 0; y < MC; ++y)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[y][r] = 0;

        // consume the block in (lo, hi): prefetch block b + D, pull block b + 1 into
        // (nlo, nhi), return block b's realigned words
        auto advance = [&](const uint32_t (&lo)[8], const uint32_t (&hi)[8], uint32_t (&nlo)[8],
                           uint32_t (&nhi)[8], uint32_t (&wv)[8]) __attribute__((always_inline)) {
            issue_next();
            // block b + 1 is position p + 1 of this group (the next group's position 0 when
            // p + 1 == KC, awaited before this group's stores); positions 1 .. D - 1 were
            // DMA'd before the previous group's stores, which are younger
            if (prev_n >= 0 && p + 1 <= D - 1)
                psyn_wait_stores<WAITN, 8 * SPR>(prev_n);
            else
                psyn_wait_vmcnt<WAITN>();
            read_block(b + 1, nlo, nhi);
            ++b;
            ++p;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                wv[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
        };
        // (no PF) consume block b: prefetch block b + D, wait for block b (positions 0 .. D - 1
        // of a group were DMA'd before the previous group's stores), read and realign it
        auto take = [&](uint32_t (&wv)[8]) __attribute__((always_inline)) {
            issue_next();
            if (prev_n >= 0 && p <= D - 1)
                psyn_wait_stores<WAITNF, 8 * SPR>(prev_n);
            else
                psyn_wait_vmcnt<WAITNF>();
            uint32_t lo[8], hi[8];
            read_block(b, lo, hi);
            ++b;
            ++p;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                wv[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
        };
        // data row x (compile time): its block, if present, into every syndrome row
        auto row_step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                            uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            const uint32_t mw = x < 32 ? mlo : mhi;
            if ((mw >> (x & 31)) & 1u) {
                uint32_t wv[8];
                if constexpr (PF) advance(lo, hi, nlo, nhi, wv);
                else take(wv);
                if constexpr (JUMP & 16) {   // ablation probe: no arithmetic
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[x % MC][r] ^= wv[r];
                } else {
                    Win win;
                    win_build(wv, win);
                    static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                        constexpr int y = decltype(yc)::value;
                        win_apply<cauchy_coef(MC, y, x)>(acc[y], win);
                    });
                }
            } else if constexpr (PF) {
                // row x erased: the block waiting in (lo, hi) is the next present row's
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    nlo[t] = lo[t];
                    nhi[t] = hi[t];
                }
            }
        };
        static_for<KC>([&](auto xc) __attribute__((always_inline)) {
            // accumulators opaque at every block boundary (no cross-block XOR reassociation)
#pragma unroll
            for (int y = 0; y < MC; ++y)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[y][r]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(xc)::value % 2 == 0) row_step(xc, lo0, hi0, lo1, hi1);
            else row_step(xc, lo1, hi1, lo0, hi0);
        });
        // the row loop alternates (lo0, hi0) / (lo1, hi1): after an odd KC the next block is
        // in (lo1, hi1); the extras (and the next group) take it from (lo0, hi0)
        if constexpr (PF && KC % 2 == 1) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                lo0[t] = lo1[t];
                hi0[t] = hi1[t];
            }
        }

        // extras: a received parity row y adds its block to T_y; a repeated data row adds
        // C[y][row] times its block to every T_y (run-time coefficients, cenc = [m][k],
        // one apply into a temporary, then scattered: this path is rare).  One extra per
        // iteration (the next block moves into (lo0, hi0)): the body is emitted once.
#pragma unroll 1
        for (int e = 0; e < ne; ++e) {
            WZ v;
            if constexpr (PF) {
                advance(lo0, hi0, lo1, hi1, v.W8);
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    lo0[t] = lo1[t];
                    hi0[t] = hi1[t];
                }
            } else {
                take(v.W8);
            }
            const int row = (int)((psyn_cload_u32(tb, psyn::kERow + (e & ~3)) >> (8 * (e & 3))) & 0xFFu);
            if (row >= KC) {
                const int y = row - KC;   // >= MC (255: a no-op extra of an unchanged group)
                if (y < MC)
                    psyn_dispatch<0, MC - 1>(y, [&](auto yc) __attribute__((always_inline)) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[decltype(yc)::value][r] ^= v.W[r];
                    });
            } else {
                expand_wz(v);
#pragma unroll 1
                for (int yy = 0; yy < MC; ++yy) {
                    const int ci = yy * KC + row;
                    const uint32_t cf = (psyn_cload_u32(cenc, ci & ~3) >> (8 * (ci & 3))) & 0xFFu;
                    uint32_t tmp[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        tmp[r] = 0;
                        // opaque zero: the dispatch cases must stay in the loop (folded, they
                        // are loop-invariant and ~70 of them would be hoisted into registers)
                        asm volatile("" : "+v"(tmp[r]));
                    }
                    apply_nibble<0>(tmp, cf & 15u, v);
                    apply_nibble<4>(tmp, cf >> 4, v);
                    psyn_dispatch<0, MC - 1>(yy, [&](auto yc) __attribute__((always_inline)) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[decltype(yc)::value][r] ^= tmp[r];
                    });
                }
            }
        }
        if (!(JUMP & 16) && n > 0) {
            // ---- T_s <- T_{y_s}: ascending, y_s >= s, so no source is overwritten early
            const uint32_t ys0 = psyn_cload_u32(tb, psyn::kYs), ys1 = psyn_cload_u32(tb, psyn::kYs + 4);
            const uint32_t ys2 = psyn_cload_u32(tb, psyn::kYs + 8), ys3 = psyn_cload_u32(tb, psyn::kYs + 12);
            static_for<RC>([&](auto sc) __attribute__((always_inline)) {
                constexpr int s = decltype(sc)::value;
                const uint32_t yw = s < 4 ? ys0 : s < 8 ? ys1 : s < 12 ? ys2 : ys3;
                const int y = (int)((yw >> (8 * (s & 3))) & 0xFFu);
                if (s < n && y != s)
                    psyn_dispatch<s, MC - 1>(y, [&](auto yc) __attribute__((always_inline)) {
                        constexpr int yy = decltype(yc)::value;
                        if constexpr (yy != s) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) acc[s][r] = acc[yy][r];
                        }
                    });
            });
            // ---- Gauss-Jordan replay: the pivot row T_p windowed once (gf_bitslice.h), then
            // T_i ^= g[p][i] T_p for every slot, g[p][p] = 1 ^ inverse pivot.  Each product
            // is a 256-way uniform branch tree to the windowed code of that coefficient, a
            // compile-time constant there (at most 8 VALU), into a temporary that is then
            // scattered to slot i: one copy of the tree, not RC
#pragma unroll 1
            for (int pv = 0; pv < n; ++pv) {
                uint32_t pw[8];
                psyn_dispatch<0, RC - 1>(pv, [&](auto pc) __attribute__((always_inline)) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) pw[r] = acc[decltype(pc)::value][r];
                });
                const int cb = psyn::kCoef + 16 * pv;
                uint32_t cw[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) cw[q] = psyn_cload_u32(tb, cb + 4 * q);
                if constexpr ((JUMP & 3) == 2) {
                    // W/Z form, each slot's product by two nibble jumps straight into its
                    // accumulator (one call site per slot, compile-time target)
                    WZ v;
#pragma unroll
                    for (int r = 0; r < 8; ++r) v.W[r] = pw[r];
                    expand_wz(v);
                    static_for<RC>([&](auto ic) __attribute__((always_inline)) {
                        constexpr int i = decltype(ic)::value;
                        if (i < n) wz_mul_acc_rt(acc[i], v, (cw[i >> 2] >> (8 * (i & 3))) & 0xFFu);
                    });
                    continue;
                }
                Win win;
                win_build(pw, win);
#pragma unroll 1
                for (int ii = 0; ii < n; ++ii) {
                    // the window is opaque per product: folded, every leaf's result is
                    // loop-invariant and would be hoisted into registers
#pragma unroll
                    for (int q = 1; q < 16; ++q) asm volatile("" : "+v"(win.lo[q]), "+v"(win.hi[q]));
                    const int cf = (int)((cw[0] >> (8 * (ii & 3))) & 0xFFu);
                    uint32_t tmp[8];
                    if constexpr ((JUMP & 3) == 1) {
                        win_mul_rt(tmp, win, (uint32_t)cf);
                    } else {
                        psyn_dispatch<0, 255>(cf, [&](auto cc) __attribute__((always_inline)) {
                            win_set<decltype(cc)::value>(tmp, win);
                        });
                    }
                    psyn_dispatch<0, RC - 1>(ii, [&](auto ic) __attribute__((always_inline)) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[decltype(ic)::value][r] ^= tmp[r];
                    });
                    // next coefficient byte: shift the 16-byte row down
                    if ((ii & 3) == 3) {
                        cw[0] = cw[1];
                        cw[1] = cw[2];
                        cw[2] = cw[3];
                    }
                }
            }
        }

        // ---- stores: recovered block j (data row e_j) into its output slot, 8 * SPR store
        // instructions each, as soon as the solve is done
        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
        static_for<RC>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            if (!(JUMP & 8) && j < n) {   // (JUMP & 8: ablation probe, no stores)
                const int oslot = slots ? (int)((psyn_cload_u32(slots, (int)((g * rmax + j) & ~3LL)) >>
                                                 (8 * ((g * rmax + j) & 3))) & 0xFFu)
                                        : j;
                uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
                const int ln = (int)__lane_id();
                uint32_t vo = ln < NWF ? 4u * (uint32_t)ln : kPDrop;
                uint32_t vt = (ln == NWF && NWF < NW) ? 4u * (uint32_t)ln : kPDrop;
                asm volatile("" : "+v"(vo), "+v"(vt));
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    __builtin_amdgcn_raw_buffer_store_b32(acc[j][r], rs, vo, r * S, SA);
                    if (S & 2)
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)acc[j][r], rs, vt, r * S, SA);
                    if (S & 1)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(acc[j][r] >> (8 * (S & 2))),
                                                             rs, vt, r * S + (S & 2), SA);
                }
            }
        });
        asm volatile("" ::: "memory");
        prev_n = n;
    }
    psyn_wait_vmcnt<0>();
}

// ------------------------------------------------------------------ prep
// 16 lanes per group: the bookkeeping of cauchy_256_decode (sort_blocks :543-575, the erased
// rows ascending, the recovery blocks in array order receive them, the row rewrite :791, the
// status codes :1287-1294), then Gauss-Jordan without pivoting on S[s][j] = C[y_s][e_j]
// (received parity rows ascending), recording per pivot p the coefficient g[p][i] the kernel
// applies to T_p for slot i, and the psyn:: table.  k <= 64, m <= 32, rmax <= 16.
// Lane s holds row s of S in registers (16 bytes); a pivot row reaches the group's lanes by
// four shuffles, and a row update is n GF(256) products through the LDS log / exp tables.
constexpr int kPsynLanes = 16;

__device__ __forceinline__ void psyn_wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int psyn_byte(const uint32_t (&w)[4], int c) {
    const uint32_t v = c < 4 ? w[0] : c < 8 ? w[1] : c < 12 ? w[2] : w[3];
    return (int)((v >> (8 * (c & 3))) & 0xFFu);
}

__global__ __launch_bounds__(256) void decode_prep_psyn_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ tab, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rmax) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    constexpr int GPB = 256 / kPsynLanes;                       // groups per block
    __shared__ uint8_t lrows[GPB][64];
    __shared__ uint8_t llist[GPB][3][16];                       // recpos, y (array order), era
    __shared__ __attribute__((aligned(16))) uint8_t ltab[GPB][psyn::kBytes];
    extern __shared__ __attribute__((aligned(16))) uint8_t lcenc[];   // m x k
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf_psyn.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf_psyn.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    const long long gfirst = (long long)blockIdx.x * GPB;
    const int ng = (int)min((long long)GPB, groups - gfirst);
    for (int i = threadIdx.x; i < ng * k; i += blockDim.x)
        lrows[i / k][i % k] = rows_in[gfirst * k + i];
    for (int i = threadIdx.x; i < GPB * psyn::kBytes / 4; i += blockDim.x)
        ((uint32_t*)ltab)[i] = 0;
    __syncthreads();
    const int gl = threadIdx.x / kPsynLanes, l = threadIdx.x % kPsynLanes;
    const int seg = (threadIdx.x & 63) / kPsynLanes;            // the group's 16 lanes in the wave
    const int sbase = (threadIdx.x & 63) - l;                   // lane 0 of the group in the wave
    const bool live = gl < ng;
    const long long g = gfirst + gl;
    const uint8_t* rg = lrows[gl];
    uint8_t* lrec = llist[gl][0];
    uint8_t* ly = llist[gl][1];
    uint8_t* lera = llist[gl][2];
    uint8_t* T = ltab[gl];

    // ---- bookkeeping: slot i = 16 q + l.  isrec: slot i holds a recovery block; first: slot
    // i holds the first copy of its data row; present: data row r was received
    uint64_t isrec = 0, isdat = 0, present = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = kPsynLanes * q + l;
        const int r = (live && i < k) ? rg[i] : 0;
        const bool rec = live && i < k && r >= k;
        const bool dat = live && i < k && r < k;
        if (dat) present |= 1ull << r;
        const uint64_t b1 = __ballot(rec), b2 = __ballot(dat);
        isrec |= ((b1 >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
        isdat |= ((b2 >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
    }
#pragma unroll
    for (int o = 1; o < kPsynLanes; o <<= 1) present |= __shfl_xor(present, o, kPsynLanes);
    uint64_t first = isdat;
    if (__popcll(isdat) != __popcll(present)) {   // a repeated data row (rare): find firsts
        first = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = kPsynLanes * q + l;
            bool fst = (isdat >> i) & 1;
            if (fst)
                for (int j = 0; j < i; ++j)
                    if (rg[j] == rg[i]) { fst = false; break; }
            first |= ((__ballot(fst) >> (kPsynLanes * seg)) & 0xFFFFull) << (kPsynLanes * q);
        }
    }
    const int nrec = __popcll(isrec);
    const uint64_t kmask = k == 64 ? ~0ull : ((1ull << k) - 1);
    const uint64_t missing = ~present & kmask;
    const int nera = __popcll(missing);
    // entry l of the lists: the l-th recovery slot, its parity row, the l-th erased row
    int myrec = -1, myera = -1;
    {
        uint64_t a = isrec, e = missing;
        for (int j = 0; j < l && a; ++j) a &= a - 1;
        for (int j = 0; j < l && e; ++j) e &= e - 1;
        if (a) myrec = __ffsll((long long)a) - 1;
        if (e) myera = __ffsll((long long)e) - 1;
    }
    const int myy = myrec >= 0 ? rg[myrec] - k : 0;
    const bool badrow = l < nrec && myy >= m;
    const bool anybad = (__ballot(badrow) >> (kPsynLanes * seg)) & 0xFFFFull;
    int early = 1;
    if (nrec == 0) early = 0;                                               // :1287-1289
    else if (k + m > 256 || (bb & 7)) early = -1;                           // :1292-1294
    else if (nrec > rmax || nera < nrec || anybad) early = -3;              // malformed rows
    int n = early == 1 ? nrec : 0;
    if (l < n) {
        lrec[l] = (uint8_t)myrec;
        ly[l] = (uint8_t)myy;
        lera[l] = (uint8_t)myera;
    }
    psyn_wave_sync();
    // ---- row s of S = C[ys_s][e_j] in lane s (s = the rank of y_l: sorted ascending, ties by
    // array order), packed 4 bytes per dword
    int mys = 0;
    for (int j = 0; j < n; ++j) mys += (ly[j] < myy) || (ly[j] == myy && j < l);
    uint32_t row[4] = {0u, 0u, 0u, 0u};
    if (l < n) {
#pragma unroll
        for (int j = 0; j < 16; ++j)   // compile-time indices: row[] stays in registers
            if (j < n) row[j >> 2] |= (uint32_t)lcenc[myy * k + lera[j]] << (8 * (j & 3));
    }
    // lane l ends up holding row s = mys; the shuffles below address rows by s, so the lane
    // holding row s is found through lsrc (lane of row s)
    __shared__ uint8_t lsrc[GPB][16];
    if (l < n) lsrc[gl][mys] = (uint8_t)l;
    psyn_wave_sync();
    const int ok_n = n;
    // ---- Gauss-Jordan without pivoting (every leading minor of a Cauchy submatrix is
    // nonzero); a zero pivot means a repeated parity row: malformed, status -3
    for (int p = 0; p < ok_n; ++p) {
        const int src = sbase + lsrc[gl][p];
        uint32_t prow[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) prow[q] = (uint32_t)__shfl((int)row[q], src, 64);
        const int piv = psyn_byte(prow, p);
        if (piv == 0) {
            early = -3;
            n = 0;
            break;
        }
        const int linv = 255 - glog[piv];                       // log of the inverse pivot
        const int inv = gexp[linv];
        const bool me = mys == p;
        const int f = psyn_byte(row, p);
        // the coefficient the kernel applies to T_p (before this step) for slot mys
        int lg = 0, gco = 0;
        if (me) {
            gco = 1 ^ inv;
            lg = linv;                                          // new row p = inv * row p
        } else if (f) {
            lg = glog[f] + linv;                                // row ^= (f / piv) * row p
            gco = gexp[lg];
        }
        if (lg >= 255) lg -= 255;                               // lg + log(x) < 512: gexp's range
        if (l < ok_n) T[psyn::kCoef + 16 * p + mys] = (uint8_t)gco;
        if (l < ok_n && (me || f)) {
            uint32_t nrow[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                if (c < ok_n) {
                    const int pc = psyn_byte(prow, c);
                    const int prod = pc ? gexp[lg + glog[pc]] : 0;
                    nrow[c >> 2] |= (uint32_t)prod << (8 * (c & 3));
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) row[q] = me ? nrow[q] : (row[q] ^ nrow[q]);
        }
    }
    // ---- the table: a changed group streams its present rows ascending, then the extras in
    // slot order; an unchanged one streams its slots in order as no-op extras (row tag 255)
    if (n > 0) {
        const int np = __popcll(present);
        const uint64_t extra = ~first & kmask;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = kPsynLanes * q + l;
            if (i < k) {
                const int r = rg[i];
                if ((first >> i) & 1) {
                    T[psyn::kPerm + __popcll(present & ((1ull << r) - 1))] = (uint8_t)i;
                } else {
                    const int e = __popcll(extra & ((1ull << i) - 1));
                    T[psyn::kPerm + np + e] = (uint8_t)i;
                    T[psyn::kERow + e] = (uint8_t)r;
                }
            }
        }
        if (l == 0) {
            *(uint32_t*)(T + psyn::kMask) = (uint32_t)present;
            *(uint32_t*)(T + psyn::kMask + 4) = (uint32_t)(present >> 32);
        }
        if (l < n) T[psyn::kYs + mys] = (uint8_t)myy;
    } else {
        for (int i = l; i < k; i += kPsynLanes) {
            T[psyn::kPerm + i] = (uint8_t)i;
            T[psyn::kERow + i] = 255;
        }
        if (l == 0) {                                            // mask: nothing present
            *(uint32_t*)(T + psyn::kMask) = 0u;
            *(uint32_t*)(T + psyn::kMask + 4) = 0u;
        }
    }
    if (live) {
        const uint8_t* rgg = rows_in + g * k;
        uint8_t* ro = rows_out ? rows_out + g * k : nullptr;
        uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
        if (ro && ro != rgg)
            for (int i = l; i < k; i += kPsynLanes) ro[i] = rg[i];
        psyn_wave_sync();
        if (l < n) {
            slots[g * rmax + l] = lrec[l];
            if (ro) ro[lrec[l]] = lera[l];                                     // :791
        }
        if (rec)
            for (int j = l; j < rmax; j += kPsynLanes) rec[j] = j < n ? lera[j] : 255;
        if (l == 0) {
            nout[g] = n;
            if (status) status[g] = early == 1 ? 0 : early;
        }
    }
    __syncthreads();
    // coalesced copy of the block's tables
    uint32_t* dst = (uint32_t*)(tab + gfirst * (long long)psyn::kBytes);
    const int nd = ng * psyn::kBytes / 4;
    for (int d = threadIdx.x; d < nd; d += blockDim.x) dst[d] = ((const uint32_t*)ltab)[d];
}

// ------------------------------------------------------------------ launchers
namespace {
constexpr int kPsynS = 169;   // bb = 1352: 1350-byte payloads

// Workgroups of `kern` one CU holds at once (the runtime's occupancy answer, computed once
// per kernel and LDS size).
template <class K>
int resident_blocks(K kern, int threads, size_t lds) {
    static int cached[64] = {};
    const int key = (int)(lds / 1024) & 63;
    if (!cached[key]) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, lds) != hipSuccess ||
            n < 1)
            n = 1;
        cached[key] = n;
    }
    return cached[key];
}
}  // namespace

// The codes compiled here: the QuicR presets with m >= 7 (their matrices are column-scaled
// Cauchy matrices: no pivoting needed), at 1352-byte blocks.
bool gf_psyn_supported(int k, int m, int bb, int rmax, const Tune& t) {
    if (!t.psyn || !t.const_enc || bb != 8 * kPsynS || rmax > 16) return false;
    return (k == 10 && (m == 10 || m == 15 || m == 20)) || (k == 15 && m == 15);
}

hipError_t launch_decode_prep_psyn(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                                   const uint8_t* cenc, uint8_t* tab, uint8_t* slots,
                                   int32_t* nout, uint8_t* rec_rows, int k, int m, int bb,
                                   int rmax, long long groups, hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    if (k > 64 || m > 32 || rmax > 16 || (((uintptr_t)tab) & 3))
        return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((groups + 15) / 16);
    note_kernel("decode_prep_psyn_kernel");
    qlaunch((decode_prep_psyn_kernel), dim3(nb), dim3(256), (uint32_t)(((size_t)m * k + 15) & ~(size_t)15),
            st, rows_in, rows_out, status, cenc, tab, slots, nout, rec_rows, groups, k, m, bb, rmax);
    return hipGetLastError();
}

hipError_t launch_gf_psyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* cenc, const uint8_t* slots, const int32_t* nout, int k,
                          int m, int bb, long long groups, int rmax, long long out_gstride,
                          hipStream_t st, const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_psyn_supported(k, m, bb, rmax, t)) return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)cenc | (uintptr_t)slots) & 3))
        return hipErrorInvalidValue;
    using SH = PsynShape<kPsynS>;
    const int D = t.psyn_depth;
    if (D != 5 && D != 7) return hipErrorInvalidValue;
    const bool pf = t.psyn_pf != 0;
    const int jump = t.psyn_jump;
    const size_t lds = (size_t)kPsynWaves * (D + 1) * SH::BUFB;
    const long long want = (groups + kPsynWaves - 1) / kPsynWaves;
    note_kernel("gf_psyn_kernel<decode,preset>");
    // persistent grid: the workgroups the CUs hold at once (registers and LDS decide)
#define QP_GO(KV, MV, DV, PFV, JV)                                                             \
    do {                                                                                       \
        auto kern = gf_psyn_kernel<KV, MV, (KV < MV ? KV : MV), kPsynS, DV, PFV, JV>;          \
        long long cap = (long long)t.cus * resident_blocks(kern, kPsynWaves * 64, lds);        \
        if (t.stream_grid > 0) cap = t.stream_grid;   /* tests: many groups per wave */        \
        const unsigned grid = (unsigned)std::min<long long>(want, cap);                       \
        if ((groups + (long long)grid * kPsynWaves - 1) / ((long long)grid * kPsynWaves) * k >=\
            (1LL << 31))                                                                       \
            return hipErrorInvalidValue;                                                       \
        qlaunch(kern, dim3(grid), dim3(kPsynWaves * 64), lds, st, in, out, tab, cenc, slots,   \
                nout, groups, rmax, out_gstride);                                              \
    } while (0)
#define QP_CODE3(DV, PFV, JV)                                 \
    switch (k * 256 + m) {                                    \
        case 10 * 256 + 10: QP_GO(10, 10, DV, PFV, JV); break;\
        case 10 * 256 + 15: QP_GO(10, 15, DV, PFV, JV); break;\
        case 10 * 256 + 20: QP_GO(10, 20, DV, PFV, JV); break;\
        default: QP_GO(15, 15, DV, PFV, JV); break;           \
    }
#define QP_CODE2(DV, PFV)                    \
    if (jump == 2) {                         \
        if (t.dec_nt) QP_CODE3(DV, PFV, 6)   \
        else QP_CODE3(DV, PFV, 2)            \
    } else if (jump) {                       \
        if (t.dec_nt) QP_CODE3(DV, PFV, 5)   \
        else QP_CODE3(DV, PFV, 1)            \
    } else QP_CODE3(DV, PFV, 0)
#define QP_CODE(DV)                \
    if (pf) QP_CODE2(DV, true)     \
    else QP_CODE2(DV, false)
    if (t.psyn_ablate) {   // timing probes: depth 7, prefetch, nibble jumps, nt stores
        if (D != 7 || !pf) return hipErrorInvalidValue;
        if (t.psyn_ablate == 1) QP_CODE3(7, true, 14)
        else if (t.psyn_ablate == 2) QP_CODE3(7, true, 22)
        else QP_CODE3(7, true, 30)
    } else if (D == 5) QP_CODE(5)
    else QP_CODE(7)
#undef QP_CODE
#undef QP_CODE2
#undef QP_CODE3
#undef QP_GO
    return hipGetLastError();
}

}  // namespace qfec
