// gf_bsyn.hip — syndrome decode of a compiled small-block code: BASELINE configs B and C,
// (32 data + 4 parity) x 1352 B blocks, r <= 4 erasures.
//
// The reference decodes in two stages (cauchy_256_decode, cauchy_256.cpp:1269-1420): the
// received originals are eliminated from the recovery rows, then the r x r system over the
// erased rows is solved.  With y_i the parity row of received recovery block R_i:
//   T_y = R_y ^ sum_{present data rows x} C[y][x] D_x      (syndromes, y = 0 .. m - 1)
//   E_j = sum_{i < r} Sinv[j][i] T_{y_i}                    (the r x r solve)
// The recovered bytes are the unique solution, so any exact solver is bit-exact.  Here the
// syndromes of ALL m parity rows are formed with the compile-time Cauchy coefficients of
// row x (cauchy_const.h; the windowed form of gf_bitslice.h, one v_bitop3 per (row,
// sub-row)), exactly the work of the compiled encode: no per-(row, block) coefficient
// loads or scalar nibble dispatch, which cost the run-time decode (gf_stream_kernel<decode>)
// more scalar than vector instructions.  Run-time coefficients remain only in the r x r
// solve (r^2 nibble applies per group against k block steps) and for the rare extra block
// that repeats a data row.
//
// Stream: every wave owns groups g0, g0 + W, ... (no barriers, no cross-wave traffic) and
// streams each group's k received blocks in the order the prep's table gives: the present
// data rows ascending, then the extras (recovery blocks, repeated data rows) in slot order.
// A block is read from wherever its slot lies (bb = 1352 is 8 mod 16: the 16-byte aligned
// envelope of the block is DMA'd, buffer_load_dwordx4 ... lds, and the block is read at the
// 8-byte skew), into a ring of D + 1 block buffers per wave.  The unrolled loop over the k
// data rows consumes the next streamed block only where row x is present (a uniform branch
// per row), so every coefficient stays a compile-time constant.
//
// vmcnt bookkeeping as in gf_tile.hip: a block is NPC DMA instructions; a group's stores
// (8 * SPR per recovered block) sit in the count before the waits for the next group's
// blocks 1 .. D - 1.  tests/test_isa.py checks the compiler adds no VMEM instruction or
// vmcnt wait of its own.
#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf256.h"
#include "gf_bitslice.h"
#include "gf_winjump.h"

namespace qfec {

#define QB_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void bsyn_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16 bytes per lane from buffer rs at voff + soff into LDS at lds + 16 * lane (nt).  The
// builtin is device-only: in a lambda the host pass would drop the kernel's host stub.
__device__ __forceinline__ void bsyn_dma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds,
                                           uint32_t voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, QB_LPTR(lds), 16, voff, soff, 0, 2);
#else
    (void)rs, (void)lds, (void)voff, (void)soff;
#endif
}

__device__ __forceinline__ uint32_t bsyn_cload_u32(const uint8_t* base, int byte_off) {
    return ((const __attribute__((address_space(4))) uint32_t*)(base))[byte_off >> 2];
}

// s_waitcnt vmcnt(BASE + 8 * SPR * n) for a wave-uniform n in [0, 4] (the stores of a group
// with n recovered blocks), capped at 63
template <int BASE, int PER>
__device__ __forceinline__ void bsyn_wait_stores(int n) {
    constexpr int W0 = BASE, W1 = BASE + PER > 63 ? 63 : BASE + PER;
    constexpr int W2 = BASE + 2 * PER > 63 ? 63 : BASE + 2 * PER;
    constexpr int W3 = BASE + 3 * PER > 63 ? 63 : BASE + 3 * PER;
    constexpr int W4 = BASE + 4 * PER > 63 ? 63 : BASE + 4 * PER;
    if (n <= 1) {
        if (n <= 0) bsyn_wait_vmcnt<W0>();
        else bsyn_wait_vmcnt<W1>();
    } else if (n <= 2) {
        bsyn_wait_vmcnt<W2>();
    } else {
        if (n == 3) bsyn_wait_vmcnt<W3>();
        else bsyn_wait_vmcnt<W4>();
    }
}

constexpr unsigned kBDrop = 0x80000000u;   // buffer offset past any range: lane dropped

__constant__ GfTables c_gf_bsyn = make_gf_tables();   // this code object's copy

template <int S>
struct BsynShape {
    static constexpr int BB = 8 * S;
    static constexpr int NW = (S + 3) / 4, NWF = S / 4;
    static constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);   // stores per sub-row
    static constexpr int BUFB = (BB + 8 + 15) / 16 * 16;        // the 16-byte envelope
    static constexpr int NPC = BUFB > 1024 ? 2 : 1;              // DMA instructions per block
    static constexpr int P1L = BUFB > 1024 ? (BUFB - 1024) / 16 : 0;   // lanes of the 2nd
};

constexpr int kBsynWaves = 4;   // waves per workgroup (independent)
constexpr int kBsynRC = 4;      // recovered blocks per group (rmax <= 4)

// KC, MC: the compiled code (k, m); S: sub-row bytes; D: blocks in flight per wave.
// NTS: the recovered blocks are stored non-temporal
template <int KC, int MC, int S, int D, bool NTS = false>
__global__ __launch_bounds__(kBsynWaves * 64) void gf_bsyn_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ tab,
    const uint8_t* __restrict__ cenc, const uint8_t* __restrict__ slots,
    const int32_t* __restrict__ nout, long long groups, int rmax, long long out_gstride) {
    using SH = BsynShape<S>;
    constexpr int BB = SH::BB, NW = SH::NW, NWF = SH::NWF, SPR = SH::SPR;
    constexpr int BUFB = SH::BUFB, NPC = SH::NPC, P1L = SH::P1L;
    constexpr int NB = D + 1;                 // the block being read + D in flight
    constexpr int RC = kBsynRC;
    constexpr int WAITN = (D - 1) * NPC;      // younger than block b + 1 when it is awaited
    static_assert(WAITN <= 63 && D >= 2 && KC >= D, "pipeline depth");
    static_assert(KC <= 64 && MC <= 8 && (KC * BB) % 16 == 0 && BB % 8 == 0 && NB <= 32,
                  "compiled small-block code");
    static_assert(KC % 2 == 0, "register double buffer parity");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    uint8_t* ring = smem + (size_t)w * NB * BUFB;
    const long long W = (long long)gridDim.x * kBsynWaves;
    const long long g0 = (long long)blockIdx.x * kBsynWaves + w;
    if (g0 >= groups) return;
    const int cnt = __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));
    const int c = lane < NW ? lane : NW - 1;  // idle lanes shadow the last word

    // ---- DMA side: stream block b = position iss_x of group g0 + i * W, the slot the table
    // names there, into ring buffer iss_buf; bit iss_buf of `skew` = its 8-byte skew.  Past
    // the stream's end the last block is re-read (every step issues and waits the same way).
    int iss_buf = 0, iss_x = 0;
    int iss_left = cnt * KC;
    const uint8_t* iss_g = in + g0 * (long long)(KC * BB);
    const uint8_t* iss_t = tab + g0 * (long long)bsyn::kBytes;
    const long long gstride = W * (long long)(KC * BB);
    const long long tstride = W * (long long)bsyn::kBytes;
    uint32_t perm_w = 0, skew = 0;
    auto issue_next = [&]() __attribute__((always_inline)) {
        if ((iss_x & 3) == 0) perm_w = bsyn_cload_u32(iss_t, bsyn::kPerm + iss_x);
        const int slot = min((int)((perm_w >> (8 * (iss_x & 3))) & 0xFFu), KC - 1);
        const int off = slot * BB;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)iss_g, 0, 0x7FFFFFFF, 0x00020000);
        uint8_t* dst = ring + iss_buf * BUFB;
        bsyn_dma16(rs, dst, 16u * (uint32_t)lane, off & ~15);
        if constexpr (NPC == 2)
            if (lane < P1L) bsyn_dma16(rs, dst + 1024, 1024u + 16u * (uint32_t)lane, off & ~15);
        skew = (off & 15) ? (skew | (1u << iss_buf)) : (skew & ~(1u << iss_buf));
        if (++iss_buf == NB) iss_buf = 0;
        if (--iss_left > 0 && ++iss_x == KC) {
            iss_x = 0;
            iss_g += gstride;
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
    bsyn_wait_vmcnt<WAITN>();
    read_block(0, lo0, hi0);

    int b = 0;        // stream index of the block in (lo0, hi0) / the current block
    int prev_n = -1;  // recovered blocks the previous group stored (-1: no previous group)
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {
        const long long g = g0 + (long long)i * W;
        const uint8_t* tb = tab + g * (long long)bsyn::kBytes;
        const uint32_t mlo = bsyn_cload_u32(tb, bsyn::kMask), mhi = bsyn_cload_u32(tb, bsyn::kMask + 4);
        const uint32_t ymap = bsyn_cload_u32(tb, bsyn::kY);
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
                bsyn_wait_stores<WAITN, 8 * SPR>(prev_n);
            else
                bsyn_wait_vmcnt<WAITN>();
            read_block(b + 1, nlo, nhi);
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
                advance(lo, hi, nlo, nhi, wv);
                Win win;
                win_build(wv, win);
                static_for<MC>([&](auto yc) __attribute__((always_inline)) {
                    constexpr int y = decltype(yc)::value;
                    win_apply<cauchy_coef(MC, y, x)>(acc[y], win);
                });
            } else {
                // row x erased: the block waiting in (lo, hi) is the next present row's
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
            for (int y = 0; y < MC; ++y)
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[y][r]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (decltype(xc)::value % 2 == 0) row_step(xc, lo0, hi0, lo1, hi1);
            else row_step(xc, lo1, hi1, lo0, hi0);
        });

        // extras: a received parity row y adds its block to T_y; a repeated data row adds
        // C[y][row] times its block to every T_y (run-time coefficients, cenc = [m][k])
        auto extra = [&](int e, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                         uint32_t (&nhi)[8]) __attribute__((always_inline)) {
            WZ v;
            advance(lo, hi, nlo, nhi, v.W8);
            const int row = (int)((bsyn_cload_u32(tb, bsyn::kERow + (e & ~3)) >> (8 * (e & 3))) & 0xFFu);
            if (row >= KC) {
                const int y = row - KC;   // >= MC (255: a no-op extra of an unchanged group)
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
                    const uint32_t cf = (bsyn_cload_u32(cenc, yy * KC + (row & ~3)) >> (8 * (row & 3))) & 0xFFu;
                    apply_nibble<0>(acc[yy], cf & 15u, v);
                    apply_nibble<4>(acc[yy], cf >> 4, v);
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

        // ---- E_j = sum_i Sinv[j][i] T_{y_i}, one recovered block at a time, stored as soon
        // as it is formed (8 * SPR store instructions per recovered block)
        asm volatile("" ::: "memory");   // stores stay in issue order among the DMAs
#pragma unroll 1
        for (int j = 0; j < n; ++j) {
            uint32_t o[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) o[r] = 0;
            const uint32_t sw = bsyn_cload_u32(tb, bsyn::kSinv + 4 * j);   // Sinv[j][0..3]
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
                // the product by two nibble jumps (gf_winjump.h), not two branch trees
                wz_mul_acc_rt(o, v, (sw >> (8 * ii)) & 0xFFu);
            }
            const int oslot = slots ? (int)((bsyn_cload_u32(slots, (int)((g * rmax + j) & ~3LL)) >>
                                             (8 * ((g * rmax + j) & 3))) & 0xFFu)
                                    : j;
            uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
            // lane offsets from the lane id (not kept live across the block loop)
            const int ln = (int)__lane_id();
            uint32_t vo = ln < NWF ? 4u * (uint32_t)ln : kBDrop;
            uint32_t vt = (ln == NWF && NWF < NW) ? 4u * (uint32_t)ln : kBDrop;
            asm volatile("" : "+v"(vo), "+v"(vt));
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                constexpr int SA = NTS ? 2 : 0;
                __builtin_amdgcn_raw_buffer_store_b32(o[r], rs, vo, r * S, SA);
                if (S & 2)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)o[r], rs, vt, r * S, SA);
                if (S & 1)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(o[r] >> (8 * (S & 2))), rs, vt,
                                                         r * S + (S & 2), SA);
            }
        }
        asm volatile("" ::: "memory");
        prev_n = n;
    }
    bsyn_wait_vmcnt<0>();
}

// ------------------------------------------------------------------ prep
// One lane per group: the bookkeeping of cauchy_256_decode (sort_blocks :543-575, the
// erased rows ascending, the row rewrite :791, the status codes :1287-1294) and the r x r
// GF(256) Gauss-Jordan inverse, then the bsyn:: table.  k <= 64, rmax <= 4.
__global__ __launch_bounds__(256) void decode_prep_bsyn_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ tab, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rmax) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    extern __shared__ __attribute__((aligned(16))) uint8_t lsm[];
    uint8_t* lcenc = lsm;                                    // m x k (padded to 16)
    uint8_t* lrows = lsm + ((m * k + 15) & ~15);             // 256 x k (k % 4 == 0)
    uint8_t* ltab = lrows + 256 * k;                         // 256 x kBytes
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf_bsyn.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf_bsyn.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    const long long gfirst = (long long)blockIdx.x * 256;
    const int ng = (int)min(256LL, groups - gfirst);
    {
        const uint32_t* src = (const uint32_t*)(rows_in + gfirst * k);
        const int nd = ng * k / 4;
        for (int i = threadIdx.x; i < nd; i += blockDim.x) ((uint32_t*)lrows)[i] = src[i];
    }
    __syncthreads();
    const int gl = threadIdx.x;
    const long long g = gfirst + gl;
    const bool live = gl < ng;
    const uint8_t* rg = lrows + (live ? gl : 0) * k;
    uint8_t* T = ltab + gl * bsyn::kBytes;
    auto B = [](uint32_t v, int j) -> int { return (int)((v >> (8 * j)) & 0xFF); };
    auto mul = [&](int a, int b2) -> int { return (a && b2) ? gexp[glog[a] + glog[b2]] : 0; };

    uint64_t present = 0, first = 0;
    int nrec = 0;
    uint32_t recpos = 0, recrow = 0;
    for (int i = 0; i < k; ++i) {
        const int r = rg[i];
        if (r < k) {
            if (!((present >> r) & 1)) {
                present |= 1ull << r;
                first |= 1ull << i;
            }
        } else {
            if (nrec < 4) {
                recpos |= (uint32_t)i << (8 * nrec);
                recrow |= (uint32_t)(r - k < 255 ? r - k : 255) << (8 * nrec);
            }
            ++nrec;
        }
    }
    const uint64_t kmask = k == 64 ? ~0ull : ((1ull << k) - 1);
    uint64_t missing = ~present & kmask;
    const int nera = __popcll(missing);
    int early = 1;
    if (nrec == 0) early = 0;                                               // :1287-1289
    else if (k + m > 256 || (bb & 7)) early = -1;                           // :1292-1294
    else if (nrec > rmax || nera < nrec) early = -3;                        // malformed rows
    else
        for (int i = 0; i < nrec; ++i)
            if (B(recrow, i) >= m) early = -3;                              // row >= k + m
    int n = early == 1 ? nrec : 0;
    uint32_t era = 0;
    for (int j = 0; j < n; ++j) {
        const int e = __ffsll((long long)missing) - 1;
        missing &= missing - 1;
        era |= (uint32_t)e << (8 * j);
    }
    // [S | I], S[i][j] = C[y_i][e_j]; Gauss-Jordan unrolled over the 4 x 8 maximum
    uint8_t M[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint8_t v = 0;
            if (i < n && j < n) v = lcenc[B(recrow, i) * k + B(era, j)];
            else if (i < n && j >= 4) v = (j - 4 == i) ? 1 : 0;
            M[i][j] = v;
        }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (p < n) {
            int piv = -1;
#pragma unroll
            for (int i = 3; i >= p; --i)
                if (i < n && M[i][p] != 0) piv = i;
            if (piv < 0) {                                                  // singular
                early = -3;
                piv = p;
            }
#pragma unroll
            for (int i = p + 1; i < 4; ++i) {
                if (i == piv) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint8_t t = M[p][j];
                        M[p][j] = M[i][j];
                        M[i][j] = t;
                    }
                }
            }
            const int inv = M[p][p] ? gexp[255 - glog[M[p][p]]] : 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) M[p][j] = (uint8_t)mul(M[p][j], inv);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i != p && i < n) {
                    const int f = M[i][p];
                    if (f) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) M[i][j] ^= (uint8_t)mul(f, M[p][j]);
                    }
                }
            }
        }
    }
    if (early != 1) n = 0;

    // the table: a changed group streams its present rows ascending, then the extras in slot
    // order; an unchanged one streams its slots in order as no-op extras (row tag 255)
    if (n > 0) {
        int ne = 0;
        const int np = __popcll(present);
        for (int i = 0; i < k; ++i) {
            const int r = rg[i];
            if ((first >> i) & 1) {
                T[bsyn::kPerm + __popcll(present & ((1ull << r) - 1))] = (uint8_t)i;
            } else {
                T[bsyn::kPerm + np + ne] = (uint8_t)i;
                T[bsyn::kERow + ne] = (uint8_t)r;
                ++ne;
            }
        }
        *(uint32_t*)(T + bsyn::kMask) = (uint32_t)present;
        *(uint32_t*)(T + bsyn::kMask + 4) = (uint32_t)(present >> 32);
        *(uint32_t*)(T + bsyn::kY) = recrow;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t sw = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (j < n && i < n) sw |= (uint32_t)M[j][4 + i] << (8 * i);
            *(uint32_t*)(T + bsyn::kSinv + 4 * j) = sw;
        }
    } else {
        for (int i = 0; i < k; ++i) {
            T[bsyn::kPerm + i] = (uint8_t)i;
            T[bsyn::kERow + i] = 255;
        }
        *(uint32_t*)(T + bsyn::kMask) = 0;
        *(uint32_t*)(T + bsyn::kMask + 4) = 0;
    }
    if (live) {
        const uint8_t* rgg = rows_in + g * k;
        uint8_t* ro = rows_out ? rows_out + g * k : nullptr;
        uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
        if (ro && ro != rgg)
            for (int i = 0; i < k; ++i) ro[i] = rg[i];
        for (int j = 0; j < n; ++j) {
            slots[g * rmax + j] = (uint8_t)B(recpos, j);
            if (ro) ro[B(recpos, j)] = (uint8_t)B(era, j);                  // :791
        }
        if (rec)
            for (int j = 0; j < rmax; ++j) rec[j] = j < n ? (uint8_t)B(era, j) : 255;
        nout[g] = n;
        if (status) status[g] = early == 1 ? 0 : early;
    }
    __syncthreads();
    // coalesced copy of the block's tables
    uint32_t* dst = (uint32_t*)(tab + gfirst * (long long)bsyn::kBytes);
    const int nd = ng * bsyn::kBytes / 4;
    for (int d = threadIdx.x; d < nd; d += blockDim.x) dst[d] = ((const uint32_t*)ltab)[d];
}

// ------------------------------------------------------------------ launchers
namespace {
constexpr int kBsynS = 169;   // bb = 1352: 1350-byte payloads (BASELINE configs B, C)
}  // namespace

bool gf_bsyn_supported(int k, int m, int bb, int rmax, const Tune& t) {
    return t.bsyn && t.const_enc && k == 32 && m == 4 && bb == 8 * kBsynS && rmax <= kBsynRC;
}

hipError_t launch_decode_prep_bsyn(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                                   const uint8_t* cenc, uint8_t* tab, uint8_t* slots,
                                   int32_t* nout, uint8_t* rec_rows, int k, int m, int bb,
                                   int rmax, long long groups, hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    if (k > 64 || k % 4 != 0 || rmax > 4 || (long long)m * k > 4096 ||
        ((((uintptr_t)tab) | (uintptr_t)rows_in) & 3))
        return hipErrorInvalidValue;
    const unsigned nb = (unsigned)((groups + 255) / 256);
    const size_t lds = (((size_t)m * k + 15) & ~(size_t)15) + 256 * (size_t)k +
                       256 * (size_t)bsyn::kBytes;
    note_kernel("decode_prep_bsyn_kernel");
    qlaunch((decode_prep_bsyn_kernel), dim3(nb), dim3(256), lds, st, rows_in, rows_out, status,
            cenc, tab, slots, nout, rec_rows, groups, k, m, bb, rmax);
    return hipGetLastError();
}

hipError_t launch_gf_bsyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* cenc, const uint8_t* slots, const int32_t* nout, int k,
                          int m, int bb, long long groups, int rmax, long long out_gstride,
                          hipStream_t st, const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (!gf_bsyn_supported(k, m, bb, rmax, t)) return hipErrorInvalidValue;
    if ((((uintptr_t)in) & 15) || ((((uintptr_t)tab) | (uintptr_t)cenc | (uintptr_t)slots) & 3))
        return hipErrorInvalidValue;
    using SH = BsynShape<kBsynS>;
    const int D = t.bsyn_depth;
    if (D != 3 && D != 5 && D != 7) return hipErrorInvalidValue;
    const size_t lds = (size_t)kBsynWaves * (D + 1) * SH::BUFB;
    const int per_cu = std::max(1, std::min((int)((160 * 1024) / lds), 20 / kBsynWaves));
    const long long want = (groups + kBsynWaves - 1) / kBsynWaves;
    long long cap = (long long)t.cus * per_cu;
    // oversubscribed: about bwg groups per wave (B decode 0.60-0.61 -> 0.53-0.60 ms, DESIGN.md
    // section 4.5)
    const int bwg = t.bsyn_wg >= 0 ? t.bsyn_wg : 2;
    if (bwg > 0) cap = (groups + (long long)kBsynWaves * bwg - 1) / ((long long)kBsynWaves * bwg);
    if (t.stream_grid > 0) cap = t.stream_grid;          // tests: many groups per wave
    const unsigned grid = (unsigned)std::min<long long>(want, cap);
    if ((groups + (long long)grid * kBsynWaves - 1) / ((long long)grid * kBsynWaves) * k >=
        (1LL << 31))
        return hipErrorInvalidValue;
    note_kernel("gf_bsyn_kernel<decode,k32m4>");
    // recovered blocks stored non-temporal (B decode 0.655 -> 0.631 ms)
#define QB_GO(DV)                                                                             \
    qlaunch((gf_bsyn_kernel<32, 4, kBsynS, DV, true>), dim3(grid), dim3(kBsynWaves * 64), lds, \
            st, in, out, tab, cenc, slots, nout, groups, rmax, out_gstride)
    switch (D) {
        case 3: QB_GO(3); break;
        case 5: QB_GO(5); break;
        default: QB_GO(7); break;
    }
#undef QB_GO
    return hipGetLastError();
}

}  // namespace qfec
