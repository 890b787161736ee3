// gf_psyn.h — the gf_psyn_kernel template and its helpers (see gf_psyn.hip for the method).
// Each instantiation object (gf_psyn_<k><m>.hip) includes this header and compiles one
// preset code's variants, so the codes build in parallel.
#pragma once
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf256.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

namespace {


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
constexpr int kPsynStage = 1536;   // per-wave LDS staging buffer of the wide stores (3 x 512 B reads)

// KC, MC: the compiled code (k, m); RC = min(k, m): recovered blocks at most; S: sub-row
// bytes; D: blocks in flight per wave; PF: block b + 1 is read from LDS into registers while
// block b is combined (16 more VGPRs; without, each block is read when its turn comes and
// the other waves of the SIMD cover the LDS latency).  JUMP: the solve's run-time products go
// (2) through two nibble jumps straight into the slot's accumulator (gf_winjump.h
// wz_mul_acc_rt, one call site per slot), or (0) through a 256-way tree of uniform branches
// into a temporary scattered to its slot.  Bit 2 of JUMP (4): the recovered blocks are stored non-temporal (dec_nt).
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
    // WIDE (JUMP & 32): a recovered block is assembled in a per-wave LDS staging buffer
    // (8 unaligned ds_write_b32 per lane, one per sub-row) and written with 3 dwordx2 stores
    // of contiguous bytes (64 lanes x 8 B), instead of 8 x (b32 + b8) stores of 169-byte
    // sub-rows: 3 VMEM instructions per block instead of 16
    constexpr bool WIDE = (JUMP & 32) != 0;
    constexpr int NSB = WIDE ? 3 : 8 * SPR;   // store instructions per recovered block
    uint8_t* stage = smem + (size_t)kPsynWaves * NB * BUFB + (size_t)w * kPsynStage;
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
                psyn_wait_stores<WAITN, NSB>(prev_n);
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
                psyn_wait_stores<WAITNF, NSB>(prev_n);
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
                    psyn_dispatch<0, 255>(cf, [&](auto cc) __attribute__((always_inline)) {
                        win_set<decltype(cc)::value>(tmp, win);
                    });
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
            if (WIDE && !(JUMP & 8) && j < n) {
                const int oslot = slots ? (int)((psyn_cload_u32(slots, (int)((g * rmax + j) & ~3LL)) >>
                                                 (8 * ((g * rmax + j) & 3))) & 0xFFu)
                                        : j;
                uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
                const int ln = (int)__lane_id();
                // The staging accesses are inline asm with explicit lgkmcnt waits: as C++ LDS
                // accesses the compiler would first wait for every LDS-DMA in flight
                // (vmcnt(0)), since it cannot tell the staging buffer from the ring.
                const uint32_t sb =
                    (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)stage;
                static_assert(S == 169, "stage_block_169");
                if (ln < NW) stage_block_169(sb, acc[j], ln);
                static_assert(BB <= 3 * 512 && BB % 8 == 0, "three dwordx2 stores per block");
                const uint32_t ra = sb + 8u * (uint32_t)ln;
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
                for (int h = 0; h < 3; ++h) {
                    const uint32_t o = 512u * h + 8u * (uint32_t)ln;   // past BB: dropped
                    __builtin_amdgcn_raw_buffer_store_b64(
                        qf_u32x2(vv[h]),
                        rs, o, 0, SA);
                }
            } else if (!(JUMP & 8) && j < n) {   // (JUMP & 8: ablation probe, no stores)
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

}  // namespace

constexpr int kPsynS = 169;   // bb = 1352: 1350-byte payloads

// launch arguments of one preset code's variants (gf_psyn_<k><m>.hip)
struct PsynLaunch {
    const uint8_t *in; uint8_t *out; const uint8_t *tab, *cenc, *slots; const int32_t *nout;
    long long groups; int rmax; long long out_gstride; hipStream_t st; const Tune *t;
    int k; bool wide; size_t lds;
};
hipError_t psyn_go_1010(const PsynLaunch& a);
hipError_t psyn_go_1015(const PsynLaunch& a);
hipError_t psyn_go_1020(const PsynLaunch& a);
hipError_t psyn_go_1515(const PsynLaunch& a);

// Workgroups of `kern` one CU holds at once (the runtime's occupancy answer, computed once
// per kernel and LDS size).
template <class K>
int psyn_resident_blocks(K kern, int threads, size_t lds) {
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

// One code's variants: ring depth {5, 7} x register prefetch x products (0: 256-way trees,
// 2: nibble jumps) x non-temporal / wide stores, and the depth-7 timing probes.
#define QP_DEFINE_GO(NAME, KV, MV)                                                             \
    hipError_t NAME(const PsynLaunch& a) {                                                     \
        const Tune& t = *a.t;                                                                  \
        const long long want = (a.groups + kPsynWaves - 1) / kPsynWaves;                       \
        auto go = [&](auto kern) -> hipError_t {                                               \
            long long cap = (long long)t.cus * psyn_resident_blocks(kern, kPsynWaves * 64, a.lds); \
            if (t.stream_grid > 0) cap = t.stream_grid; /* tests: many groups per wave */      \
            const unsigned grid = (unsigned)std::min<long long>(want, cap);                   \
            if ((a.groups + (long long)grid * kPsynWaves - 1) / ((long long)grid * kPsynWaves) *  \
                    a.k >= (1LL << 31))                                                        \
                return hipErrorInvalidValue;                                                   \
            qlaunch(kern, dim3(grid), dim3(kPsynWaves * 64), a.lds, a.st, a.in, a.out, a.tab,  \
                    a.cenc, a.slots, a.nout, a.groups, a.rmax, a.out_gstride);                \
            return hipGetLastError();                                                          \
        };                                                                                     \
        constexpr int RCV = KV < MV ? KV : MV;                                                 \
        const int D = t.psyn_depth, J = t.psyn_jump;                                           \
        const bool pf = t.psyn_pf != 0;                                                        \
        const int var = J == 0 ? 0 : (2 | (t.dec_nt ? 4 : 0) | (a.wide ? 32 : 0));             \
        if (t.psyn_ablate) {                                                                   \
            if (D != 7 || !pf) return hipErrorInvalidValue;                                    \
            if (t.psyn_ablate == 1) return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, 7, true, 14>); \
            if (t.psyn_ablate == 2) return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, 7, true, 22>); \
            return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, 7, true, 30>);                       \
        }                                                                                      \
        auto pick = [&](auto dc, auto pc) -> hipError_t {                                     \
            constexpr int DV = decltype(dc)::value;                                            \
            constexpr bool PV = decltype(pc)::value;                                           \
            switch (var) {                                                                     \
                case 0: return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, DV, PV, 0>);             \
                case 2: return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, DV, PV, 2>);             \
                case 6: return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, DV, PV, 6>);             \
                case 34: return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, DV, PV, 34>);           \
                default: return go(gf_psyn_kernel<KV, MV, RCV, kPsynS, DV, PV, 38>);           \
            }                                                                                  \
        };                                                                                     \
        using I5 = std::integral_constant<int, 5>;                                             \
        using I7 = std::integral_constant<int, 7>;                                             \
        if (D == 5) return pf ? pick(I5{}, std::true_type{}) : pick(I5{}, std::false_type{});  \
        return pf ? pick(I7{}, std::true_type{}) : pick(I7{}, std::false_type{});              \
    }

}  // namespace qfec
