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

// 16 bytes per lane from buffer rs at voff into LDS at lds + 16 * lane (nt).  (Device only:
// in a lambda the builtin would void the kernel's host stub.)
__device__ __forceinline__ void psyn_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QP_LPTR(lds), 16, voff, 0, 0, 2);
#else
    (void)rs, (void)lds, (void)voff;
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

// KC, MC: the compiled code (k, m); RC = min(k, m): recovered blocks at most; S: sub-row
// bytes; D: blocks in flight per wave.  Each block is read from LDS when its turn comes (the
// other waves of the SIMD cover the LDS latency; no register prefetch: fewer VGPRs, more
// waves).  The solve's run-time products go through two nibble jumps straight into the slot's
// accumulator (gf_winjump.h wz_mul_acc_rt, one call site per slot); recovered blocks are
// stored non-temporal.  (Measured variants: DESIGN.md section 3.7.)
//
// Per-block bookkeeping is kept scalar-light: one buffer resource per GROUP (its 16-byte
// aligned start, bounded by the end of the input), a block is its slot's byte offset added to
// the lanes' DMA offsets (one VALU); and every group issues at least NSTMIN stores (empty-range
// ones pad a group with fewer than 4 recovered blocks), so the wait for a block DMA'd before
// the previous group's stores is always vmcnt(63): no wait ladder over the store count.
// WIDE: each recovered block is staged in LDS as its contiguous bytes and written as three
// 512-byte runs of 8-byte lanes (3 store instructions instead of 8 x SPR); every group then
// issues exactly 3 x RC stores (empty-range ones pad it), so all its waits are exact
// immediates below 63 instead of the vmcnt(63) that over-waits behind > 63 stores.
constexpr int kPsynStage = 1360;   // per-wave staging buffer (WIDE), after the rings
template <int KC, int MC, int RC, int S, int D, bool WIDE = false>
__global__ __launch_bounds__(kPsynWaves * 64) void gf_psyn_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
    const uint8_t* __restrict__ cenc, const uint8_t* __restrict__ slots,
    const int32_t* __restrict__ nout, long long groups, int rmax, long long out_gstride) {
    using SH = PsynShape<S>;
    constexpr int BB = SH::BB, NW = SH::NW, NWF = SH::NWF, SPR = SH::SPR;
    constexpr int BUFB = SH::BUFB, NPC = SH::NPC, P1L = SH::P1L;
    constexpr int NB = D + 1;                 // the block being read + D in flight
    constexpr int WAITN = D * NPC;            // younger than block b when it is awaited
    constexpr int NSB = 8 * SPR;              // store instructions per recovered block
    constexpr int NSTMIN = 63 - WAITN;        // stores a group issues at least
    constexpr int NSTW = 3 * RC;              // (WIDE) stores a group issues, exactly
    constexpr int WAIT0 = WIDE ? WAITN + NSTW : 63;   // a block DMA'd before the last stores
    static_assert(WAITN <= 63 && D >= 2 && KC >= D, "pipeline depth");
    static_assert(!WIDE || (S == 169 && WAIT0 <= 63), "wide stores: 1352-byte blocks");
    static_assert(KC <= 64 && MC <= 32 && RC <= 16 && RC <= KC && RC <= MC && BB % 8 == 0 &&
                      NB <= 32 && BUFB <= 2048,
                  "compiled small-block code");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int w = wave_id();
    uint8_t* ring = smem + (size_t)w * NB * BUFB;
    const uint32_t stage =   // (WIDE) this wave's staging buffer (LDS address)
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(
            smem + (size_t)kPsynWaves * NB * BUFB + (size_t)w * kPsynStage);
    const long long W = (long long)gridDim.x * kPsynWaves;
    const long long g0 = (long long)blockIdx.x * kPsynWaves + w;
    if (g0 >= groups) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));
    constexpr long long GB = (long long)KC * BB;
    const long long in_bytes = groups * GB;
    uint32_t v16 = 16u * (uint32_t)__lane_id();   // the lane's 16 bytes of a DMA instruction
    asm volatile("" : "+v"(v16));

    // ---- DMA side: stream block b = position iss_x of group iss_g, the slot the table names
    // there, into ring buffer iss_buf; bit iss_buf of `skew` = its 8-byte skew.  Past the
    // stream's end the last block is re-read (every step issues and waits the same way).
    int iss_buf = 0, iss_x = 0;
    int iss_left = cnt * KC;
    long long iss_g = g0;
    const uint8_t* iss_t = tab + g0 * (long long)psyn::kBytes;
    const long long tstride = W * (long long)psyn::kBytes;
    uint32_t perm_w = 0, skew = 0;
    int iss_sk = 0;                               // the issued group's start mod 16 (0 or 8)
    __amdgpu_buffer_rsrc_t iss_rs;
    auto group_rsrc = [&]() __attribute__((always_inline)) {
        const long long a = iss_g * GB;
        const long long a16 = a & ~15LL;
        iss_sk = (int)(a & 15);
        iss_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(in + a16), 0,
                                                   (unsigned)min(in_bytes - a16, GB + 32), 0x00020000);
    };
    group_rsrc();
    auto issue_next = [&]() __attribute__((always_inline)) {
        if ((iss_x & 3) == 0) perm_w = psyn_cload_u32(iss_t, psyn::kPerm + iss_x);
        const int slot = min((int)((perm_w >> (8 * (iss_x & 3))) & 0xFFu), KC - 1);
        const int off = iss_sk + slot * BB;        // the block's offset from the group's 16-B start
        uint32_t vo = v16 + (uint32_t)(off & ~15);
        uint8_t* dst = ring + iss_buf * BUFB;
        psyn_dma16(iss_rs, dst, vo);
        if constexpr (NPC == 2)
            if (__lane_id() < P1L) psyn_dma16(iss_rs, dst + 1024, vo + 1024u);
        skew = (off & 8) ? (skew | (1u << iss_buf)) : (skew & ~(1u << iss_buf));
        if (++iss_buf == NB) iss_buf = 0;
        if (--iss_left > 0 && ++iss_x == KC) {
            iss_x = 0;
            iss_g += W;
            iss_t += tstride;
            group_rsrc();
        }
    };

#pragma unroll 1
    for (int u = 0; u < D; ++u) issue_next();
    asm volatile("" ::: "memory");
    {
        // the stores a previous group would have issued (empty range): the first group's
        // blocks 0 .. D - 1 are awaited like every other group's
        const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
        for (int q = 0; q < (WIDE ? NSTW : NSTMIN); ++q)
            __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
    }
    asm volatile("" ::: "memory");

    int b = 0;        // stream index of the next block to consume
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = g0 + (long long)i * W;
        const uint8_t* tb = tab + g * (long long)psyn::kBytes;
        const uint32_t mlo = psyn_cload_u32(tb, psyn::kMask), mhi = psyn_cload_u32(tb, psyn::kMask + 4);
        // the syndrome rows the solve uses (the received parity rows); the others are not
        // accumulated (cauchy_256.cpp:712-795: only received recovery rows enter the system)
        const uint32_t need = psyn_cload_u32(tb, psyn::kNeed);
        const int n = min(min(nout[g], rmax), RC);
        const int ne = KC - __builtin_popcount(mlo) - __builtin_popcount(mhi);
        int p = 0;    // blocks of this group consumed
        uint32_t acc[MC][8];
#pragma unroll
        for (int y = 0; y < MC; ++y)
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[y][r] = 0;

        // consume block b: issue block b + D, wait for block b (positions 0 .. D - 1 of a group
        // were DMA'd before the previous group's >= NSTMIN stores), read and realign it
        auto take = [&](uint32_t (&wv)[8]) __attribute__((always_inline)) {
            issue_next();
            if (p < D) psyn_wait_vmcnt<WAIT0>();
            else psyn_wait_vmcnt<WAITN>();
            const int buf = (int)((unsigned)b % NB);
            uint32_t a = 4u * (uint32_t)min((int)__lane_id(), NW - 1) + (uint32_t)(buf * BUFB) +
                         (((skew >> buf) & 1u) << 3);
            asm volatile("" : "+v"(a));   // no hoisting across blocks
            const uint8_t* L = ring + a;
            uint32_t lo[8], hi[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                const uint32_t* q = (const uint32_t*)(L + (o & ~3));
                lo[t] = q[0];
                hi[t] = (o & 3) ? q[1] : 0u;
            }
            ++b;
            ++p;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int o = t * S;
                wv[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
            }
        };
        // data row x (compile time): its block, if present, into every syndrome row
        static_for<KC>([&](auto xc) __attribute__((always_inline)) {
            constexpr int x = decltype(xc)::value;
            // accumulators opaque at every block boundary (no cross-block XOR reassociation)
#pragma unroll
            for (int y = 0; y < MC; ++y)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[y][r]));
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t mw = x < 32 ? mlo : mhi;
            if ((mw >> (x & 31)) & 1u) {
                uint32_t wv[8];
                take(wv);
                Win win;
                win_build(wv, win);
                static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                    constexpr int y = decltype(yc)::value;
                    // a uniform branch per row; the empty asm keeps it a branch (no select)
                    if (__builtin_expect((need >> y) & 1u, 1)) {
                        asm volatile("");
                        win_apply<cauchy_coef(MC, y, x)>(acc[y], win);
                    }
                });
            }
        });

        // extras: a received parity row y adds its block to T_y; a repeated data row adds
        // C[y][row] times its block to every T_y (run-time coefficients, cenc = [m][k],
        // one apply into a temporary, then scattered: this path is rare)
#pragma unroll 1
        for (int e = 0; e < ne; ++e) {
            WZ v;
            take(v.W8);
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
                    if (!((need >> yy) & 1u)) continue;
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
        if (n > 0) {
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
            // ---- Gauss-Jordan replay: the pivot row T_p expanded once (W/Z form), then
            // T_i ^= g[p][i] T_p for every slot by two nibble jumps straight into slot i's
            // accumulator (one call site per slot), g[p][p] = 1 ^ inverse pivot
#pragma unroll 1
            for (int pv = 0; pv < n; ++pv) {
                WZ v;
                psyn_dispatch<0, RC - 1>(pv, [&](auto pc) __attribute__((always_inline)) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v.W[r] = acc[decltype(pc)::value][r];
                });
                const int cb = psyn::kCoef + 16 * pv;
                uint32_t cw[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) cw[q] = psyn_cload_u32(tb, cb + 4 * q);
                expand_wz(v);
                static_for<RC>([&](auto ic) __attribute__((always_inline)) {
                    constexpr int i = decltype(ic)::value;
                    if (i < n) wz_mul_acc_rt(acc[i], v, (cw[i >> 2] >> (8 * (i & 3))) & 0xFFu);
                });
            }
        }

        // ---- stores: recovered block j (data row e_j) into its output slot, NSB store
        // instructions each, non-temporal; a group with fewer than 4 recovered blocks pads to
        // NSTMIN stores with empty-range ones
        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
        if constexpr (WIDE) {
            const int ln = (int)__lane_id();
            const uint32_t ra = stage + 8u * (uint32_t)ln;
            static_for<RC>([&](auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value;
                if (j < n) {
                    const int oslot = slots ? (int)((psyn_cload_u32(slots, (int)((g * rmax + j) & ~3LL)) >>
                                                     (8 * ((g * rmax + j) & 3))) & 0xFFu)
                                            : j;
                    uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
                    if (ln < NW) stage_block_169(stage, acc[j], ln);
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
                                                              512u * h + 8u * (uint32_t)ln, 0, 2);
                }
            });
            // pad to exactly NSTW stores (empty range)
            const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll 1
            for (int q = 3 * n; q < NSTW; ++q) __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 0, 0);
            asm volatile("" ::: "memory");
            continue;
        }
        static_for<RC>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            if (j < n) {
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
                    __builtin_amdgcn_raw_buffer_store_b32(acc[j][r], rs, vo, r * S, 2);
                    if (S & 2)
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)acc[j][r], rs, vt, r * S, 2);
                    if (S & 1)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(acc[j][r] >> (8 * (S & 2))),
                                                             rs, vt, r * S + (S & 2), 2);
                }
            }
        });
        static_assert(4 * NSB >= NSTMIN, "four recovered blocks are enough stores");
        if (n < 4) {
            const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0u, 0x00020000);
#pragma unroll
            for (int q = 0; q < NSTMIN; ++q) __builtin_amdgcn_raw_buffer_store_b32(0u, none, 0u, 4 * q, 0);
        }
        asm volatile("" ::: "memory");
    }
    psyn_wait_vmcnt<0>();
}

}  // namespace

constexpr int kPsynS = 169;   // bb = 1352: 1350-byte payloads

// launch arguments of one preset code's variants (gf_psyn_<k><m>.hip)
struct PsynLaunch {
    const uint8_t *in; uint8_t *out; const uint8_t *tab, *cenc, *slots; const int32_t *nout;
    long long groups; int rmax; long long out_gstride; hipStream_t st; const Tune *t;
    int k; size_t lds; bool wide;
};
hipError_t psyn_go_1010(const PsynLaunch& a);
hipError_t psyn_go_1015(const PsynLaunch& a);
hipError_t psyn_go_1020(const PsynLaunch& a);
hipError_t psyn_go_1515(const PsynLaunch& a);
hipError_t psyn_go_55(const PsynLaunch& a);

// One code's kernel: ring depth 5, no register prefetch, solve products by nibble jumps,
// non-temporal stores (the other variants measured slower, 3.7).
// The grid is the workgroups one CU holds at once (the runtime's occupancy answer for this
// kernel, cached per kernel: the codes differ in VGPRs) times the CUs.
#define QP_DEFINE_GO(NAME, KV, MV)                                                             \
    hipError_t NAME(const PsynLaunch& a) {                                                     \
        const Tune& t = *a.t;                                                                  \
        constexpr int RCV = KV < MV ? KV : MV;                                                 \
        const auto kern = a.wide ? gf_psyn_kernel<KV, MV, RCV, kPsynS, 5, true>               \
                                 : gf_psyn_kernel<KV, MV, RCV, kPsynS, 5, false>;             \
        const long long want = (a.groups + kPsynWaves - 1) / kPsynWaves;                       \
        long long cap = (long long)t.cus * resident_blocks((const void*)kern, kPsynWaves * 64, a.lds); \
        if (t.psyn_wg > 0) /* oversubscribed: about psyn_wg groups per wave */                \
            cap = (a.groups + (long long)kPsynWaves * t.psyn_wg - 1) /                         \
                  ((long long)kPsynWaves * t.psyn_wg);                                         \
        if (t.stream_grid > 0) cap = t.stream_grid; /* tests: many groups per wave */          \
        const unsigned grid = (unsigned)std::min<long long>(want, cap);                       \
        if ((a.groups + (long long)grid * kPsynWaves - 1) / ((long long)grid * kPsynWaves) *   \
                a.k >= (1LL << 31))                                                            \
            return hipErrorInvalidValue;                                                       \
        note_grid("gf_psyn_kernel", grid);                                                     \
        qlaunch(kern, dim3(grid), dim3(kPsynWaves * 64), a.lds, a.st, a.in, a.out, a.tab,      \
                a.cenc, a.slots, a.nout, a.groups, a.rmax, a.out_gstride);                    \
        return hipGetLastError();                                                              \
    }

}  // namespace qfec
