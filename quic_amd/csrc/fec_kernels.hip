// fec_kernels.hip — gfx950 kernels for QuicR packet-group FEC (encode + erasure recover).
//
// The reference codec (libcat cauchy_256, net/quic/core/libcat/cauchy_256.cpp) is a
// bit-sliced Cauchy Reed-Solomon code over GF(2^8): each block of bb bytes is 8 sub-rows
// of s = bb/8 bytes and a GF(256) coefficient c acts on a block through its transposed
// 8x8 bit expansion
//      out[r][j] ^= XOR_{t : bit t of (c * alpha^r)} in[t][j]          (j = byte column)
// i.e. pure byte XORs between sub-rows at the SAME column j.  No multiplications touch
// the data, so the work is HBM-bound byte streaming (no MFMA: nothing here is a
// floating-point contraction).
//
// Kernel set (all wave64, 256-thread workgroups = 4 independent waves):
//   xor_encode / xor_decode   m = 1 XOR parity (cauchy_256.cpp:1519-1528, :486-540)
//   gf_apply<RC>              bit-sliced GF(256) matrix x blocks, RC outputs per wave;
//                             used for encode (Cauchy rows, :1502-1601) and for decode
//                             (per-group recovery rows from the prep kernel)
//   decode_prep               per-group GF(256) inverse of the erasure submatrix
//                             (replaces sort_blocks/eliminate_original/bitmatrix GE,
//                             :543-1252: same unique solution, one pass over the data)
//
// The coefficient of a (output, input) pair is wave-uniform, so it lives in SGPRs and the
// 8x8 expansion is a scalar branch over its two nibbles; the data lane only ever runs
// v_xor / v_bitop3 (3-input XOR).  See DESIGN.md "Kernels" for the derivation of the
// W/Z recurrences used below.
#include "fec_kernels.h"
#include "gf256.h"
#include "gf_bitslice.h"

namespace qfec {

typedef uint32_t u32ua __attribute__((aligned(1)));   // unaligned dword (gfx950 unaligned mode)
typedef uint64_t u64a __attribute__((aligned(8)));

__constant__ GfTables c_gf = make_gf_tables();

// ------------------------------------------------------------------ m = 1 XOR paths
// Flat mapping: every lane owns one VS-byte unit (g, q) of one group and issues all k of
// its loads back to back, so a wave keeps k * 64 * VS bytes in flight in a single phase.
// The last unit of a block is shifted back to end at bb (loads stay inside the block) and
// stores only the bytes no other unit owns, so no byte is written twice and an in-place
// decode never reads a byte another lane has already rewritten and then uses it.
//   encode: out = parity + g*out_gstride
//   decode: out = blocks' slot eidx[g] (the slot tagged row >= k); the XOR runs over all
//           k slots — the erased slot's own parity included (cauchy_256.cpp:505-531) —
//           so the loads never wait on eidx, only the store does.
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));

template <int VS> struct Unit;
// Loads and stores are non-temporal: every byte is touched exactly once, and on gfx950
// nt streaming measured +17-23% over the default policy with cold caches
// (tools/microbench).
template <> struct Unit<16> {
    typedef u32x4a8 T;
    static __device__ __forceinline__ T ld(const uint8_t* p) {
        return __builtin_nontemporal_load((const T*)p);
    }
    static __device__ __forceinline__ void st(uint8_t* p, T v) {
        __builtin_nontemporal_store(v, (T*)p);
    }
};
template <> struct Unit<4> {
    typedef uint32_t T;
    static __device__ __forceinline__ T ld(const uint8_t* p) {
        return __builtin_nontemporal_load((const u32ua*)p);
    }
    static __device__ __forceinline__ void st(uint8_t* p, T v) {
        __builtin_nontemporal_store(v, (u32ua*)p);
    }
};

template <int VS, int K, bool DECODE>
__global__ __launch_bounds__(256) void xor_flat_kernel(
    const uint8_t* __restrict__ in, uint8_t* out, const uint8_t* __restrict__ eidx, int k,
    int bb, int nu, unsigned total_units, long long in_gstride, long long out_gstride,
    long long e_stride) {
    typedef typename Unit<VS>::T V;
    const unsigned u = blockIdx.x * 256u + threadIdx.x;
    if (u >= total_units) return;
    const unsigned g = u / (unsigned)nu;
    const int q = (int)(u - g * (unsigned)nu);
    const int off = min(q * VS, bb - VS);
    const uint8_t* p = in + (long long)g * in_gstride + off;
    int e = 0;
    if (DECODE) e = eidx[g];   // issued beside the data loads
    V acc = Unit<VS>::ld(p);
    if (K) {
#pragma unroll
        for (int x = 1; x < (K ? K : 1); ++x) acc ^= Unit<VS>::ld(p + (long long)x * bb);
    } else {
#pragma unroll 4
        for (int x = 1; x < k; ++x) acc ^= Unit<VS>::ld(p + (long long)x * bb);
    }
    uint8_t* dst = out + (long long)g * out_gstride;
    if (DECODE) {
        if (e == 255) return;   // nothing erased in this group
        dst += (long long)e * e_stride;   // e_stride 0: recovered-blocks layout
    }
    const int own = q * VS;   // first byte this unit owns
    if (own + VS <= bb) {
        Unit<VS>::st(dst + off, acc);
    } else {
        // tail unit: owns bytes [own, bb) = the top (bb - own) bytes of the shifted vector
        const int skip = own - off;
        const uint8_t* b = (const uint8_t*)&acc;
        if (VS == 16 && skip == 8) {
            *(uint64_t*)(dst + own) = ((const uint64_t*)b)[1];
        } else {
            for (int i = skip; i < VS; ++i) dst[off + i] = b[i];
        }
    }
}

#define QF_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QF_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Tiny blocks (bb < 4): one byte per lane.
template <bool DECODE>
__global__ __launch_bounds__(256) void xor_bytes_kernel(
    const uint8_t* __restrict__ in, uint8_t* out, const uint8_t* __restrict__ eidx, int k,
    int bb, long long total, long long in_gstride, long long out_gstride, long long e_stride) {
    const long long u = (long long)blockIdx.x * 256 + threadIdx.x;
    if (u >= total) return;
    const long long g = u / bb;
    const int i = (int)(u % bb);
    const uint8_t* p = in + g * in_gstride + i;
    uint8_t acc = 0;
    for (int x = 0; x < k; ++x) acc ^= p[(long long)x * bb];
    uint8_t* dst = out + g * out_gstride;
    if (DECODE) {
        const int e = eidx[g];
        if (e == 255) return;
        dst += (long long)e * e_stride;
    }
    dst[i] = acc;
}

// m = 1 decode bookkeeping (cauchy_decode_m1, cauchy_256.cpp:486-540), one thread per
// group: the erased slot is the first with row >= k; its new row is the first data row
// not tagged by any other slot.  eidx[g] = that slot (255 = nothing erased).  compact:
// rows_out is [G] and receives the recovered data row (255 = nothing erased) instead of
// the rewritten tags.
__global__ __launch_bounds__(256) void m1_prep_kernel(const uint8_t* __restrict__ rows_in,
                                                      uint8_t* rows_out,
                                                      int32_t* __restrict__ status,
                                                      uint8_t* __restrict__ eidx, int k,
                                                      long long groups, int compact) {
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g >= groups) return;
    const uint8_t* rg = rows_in + g * k;
    uint8_t* ro = compact ? nullptr : rows_out + g * k;
    uint64_t seen[4] = {0, 0, 0, 0};
    int e = -1;
    for (int i = 0; i < k; ++i) {
        const int r = rg[i];
        if (r >= k) {
            if (e < 0) { e = i; continue; }
        }
        if (r < k) seen[r >> 6] |= 1ull << (r & 63);
        if (ro && ro != rg) ro[i] = (uint8_t)r;
    }
    if (status) status[g] = 0;
    if (e < 0) {
        eidx[g] = 255;
        if (compact) rows_out[g] = 255;
        return;
    }
    int miss = -1;
    for (int w = 0; w < 4 && miss < 0; ++w) {
        const uint64_t free = ~seen[w];
        if (free) {
            const int b = w * 64 + __ffsll((long long)free) - 1;
            if (b < k) miss = b;
            break;
        }
    }
    const uint8_t nr = miss >= 0 ? (uint8_t)miss : rg[e];
    if (compact) rows_out[g] = nr;
    else ro[e] = nr;
    eidx[g] = (uint8_t)e;
}

__global__ void replicate_kernel(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                 int m, int bb, long long groups) {
    const long long total = groups * m * (long long)bb;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long g = i / ((long long)m * bb);
        const long long b = i % bb;
        parity[i] = data[g * bb + b];   // k = 1: the group holds one block
    }
}

// k <= 1, recovered-blocks layout: a block tagged anything but row 0 is a parity copy of
// data row 0 (cauchy_256.cpp:1508-1516), so it is that row's recovered block.
__global__ void rec_k1_kernel(const uint8_t* __restrict__ blocks, const uint8_t* __restrict__ rows_in,
                              uint8_t* __restrict__ rec, uint8_t* __restrict__ rec_rows,
                              int32_t* __restrict__ status, int bb, int rmax, long long groups) {
    const long long total = groups * (long long)bb;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long g = i / bb;
        const long long b = i % bb;
        const bool lost = rows_in[g] != 0;
        if (lost) rec[g * rmax * (long long)bb + b] = blocks[g * (long long)bb + b];
        if (b == 0) {
            rec_rows[g * rmax] = lost ? 0 : 255;
            if (status) status[g] = 0;
        }
    }
}

__global__ void rows_k1_kernel(const uint8_t* __restrict__ rows_in, uint8_t* rows_out,
                               int32_t* __restrict__ status, long long groups) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= groups) return;
    rows_out[g] = 0;
    (void)rows_in;
    if (status) status[g] = 0;
}

// Column-word access.  Word c of sub-row t covers bytes [t*s + 4c, +4); the last word of a
// sub-row may be partial (s % 4 != 0).  Loads of the last word are shifted back inside the
// sub-row (never past the block) and realigned; stores write only the valid bytes.
struct ColAccess {
    int lo;        // byte offset of the dword actually loaded within the sub-row
    int shift;     // right shift (bits) that realigns it
    int nvalid;    // valid bytes of this lane's word (0 = lane idle)
};

template <bool TINY>
__device__ __forceinline__ ColAccess col_access(int c, int nw, int s) {
    ColAccess a;
    const int cc = c < nw ? c : nw - 1;
    const int off = 4 * cc;
    a.nvalid = c < nw ? min(4, s - off) : 0;
    if (!TINY) {
        a.lo = min(off, s - 4);
        a.shift = 8 * (off - a.lo);
    } else {
        a.lo = 0;
        a.shift = 0;
    }
    return a;
}

// TINY = blocks under 32 bytes (s < 4): bytewise, never past the sub-row.  Otherwise the
// raw (unshifted) dword; the caller applies `>> shift`.
template <bool TINY>
__device__ __forceinline__ uint32_t load_raw(const uint8_t* sub, const ColAccess& a, int s) {
    if (!TINY) return *(const u32ua*)(sub + a.lo);
    uint32_t v = 0;
    for (int b = 0; b < 3; ++b)
        if (b < s) v |= (uint32_t)sub[b] << (8 * b);
    return v;
}

__device__ __forceinline__ void store_word(uint8_t* sub, int c, const ColAccess& a, uint32_t v) {
    if (a.nvalid == 4) {
        *(u32ua*)(sub + 4 * c) = v;
    } else if (a.nvalid > 0) {
        for (int b = 0; b < a.nvalid; ++b) sub[4 * c + b] = (uint8_t)(v >> (8 * b));
    }
}

// Workgroup-size bound per output-chunk width: it caps VGPRs at 512 / ceil(waves / 4), so
// the RC x 8 accumulators never spill (RC 4: 128 VGPR, RC 8: 170, RC 16: 256).
template <int RC> struct ApplyBound { static constexpr int T = RC <= 4 ? 1024 : (RC == 8 ? 640 : 320); };

// One wave = one (group, output chunk, 64-word column tile).  RC outputs per wave.
//   coef:  [(g) * coef_gstride + (chunk * k + pos) * RCP + j]  (RCP = max(4, RC))
//   encode: outputs o = chunk*RC + j < m go to out + g*out_gstride + o*bb
//   decode: outputs o < nout[g] go to out + g*out_gstride + slots[g*rmax + o]*bb
//   FLAT (encode only: the coefficients are the same for every group): the lanes of a wave
//   take consecutive (group, column word) pairs across group boundaries, so no lane idles
//   when a sub-row is not a multiple of 64 words (169-byte sub-rows: 43 words, 67 % of a
//   wave); waves are numbered (lane tile, chunk) with the chunk fastest.
template <int RC, bool DECODE, bool TINY, int PD, bool FLAT = false>
__global__ __launch_bounds__(ApplyBound<RC>::T) void gf_apply_kernel(
    const uint8_t* __restrict__ in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, int k, int m, int bb,
    int nw, int ntiles, int nchunk, int rmax, long long coef_gstride, long long out_gstride,
    int total_units, long long flat_lanes = 0) {
    static_assert(!(FLAT && DECODE), "decode coefficients differ per group");
    constexpr int RCP = RC < 4 ? 4 : RC;
    constexpr int NCW = RCP / 4;
    const int lane = threadIdx.x & 63;
    // Units are numbered (group, chunk, tile) with the tile fastest; a workgroup holds 4
    // consecutive units.  The chunks of a group re-read the same input blocks, so the
    // workgroups of one group should share an L2: hardware deals workgroups round-robin
    // to the 8 XCDs (each with its own L2), so logical workgroup l runs as hardware
    // block b with consecutive l on one XCD (a bijection for any grid size).
    const unsigned nbk = gridDim.x, b = blockIdx.x, xcd = b & 7u, q8 = nbk >> 3, r8 = nbk & 7u;
    const unsigned lwg = xcd * q8 + (xcd < r8 ? xcd : r8) + (b >> 3);
    const int unit = (int)lwg * 4 + wave_id();
    if (unit >= total_units) return;
    int g, chunk, c;
    bool live = true;
    if (FLAT) {
        chunk = unit % nchunk;
        long long u = (long long)(unit / nchunk) * 64 + lane;
        live = u < flat_lanes;
        if (!live) u = flat_lanes - 1;
        g = (int)(u / nw);
        c = (int)(u - (long long)g * nw);
    } else {
        const int tile = unit % ntiles;
        const int gc = unit / ntiles;
        chunk = gc % nchunk;
        g = gc / nchunk;
        c = tile * 64 + lane;
    }
    int n = DECODE ? nout[g] : m;
    n = min(n - chunk * RC, RC);
    if (n <= 0) return;
    const int s = bb >> 3;
    const ColAccess ca = col_access<TINY>(c, nw, s);

    const uint8_t* gin = in + (long long)g * k * bb;
    const uint32_t* cw = (const uint32_t*)(coef + (FLAT ? 0 : (long long)g * coef_gstride) +
                                           (long long)chunk * k * RCP);

    uint32_t acc[RC][8];
#pragma unroll
    for (int j = 0; j < RC; ++j)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[j][r] = 0;

    // Software pipeline PD blocks deep: raw words of blocks pos+1 .. pos+PD are in flight
    // while block pos is combined (the realigning shift is applied at use, so the
    // compiler's vmcnt wait lands at the consumer).  The loop is unrolled by PD so every
    // ring slot is a fixed register set.  Loads past the last block are clamped to it.
    uint32_t raw[PD][8];
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        const uint8_t* p = gin + (long long)min(u, k - 1) * bb;
#pragma unroll
        for (int t = 0; t < 8; ++t) raw[u][t] = load_raw<TINY>(p + t * s, ca, s);
    }

#pragma unroll 1
    for (int pos0 = 0; pos0 < k; pos0 += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int pos = pos0 + u;
            if (pos < k) {
                WZ v;
#pragma unroll
                for (int t = 0; t < 8; ++t) v.W[t] = TINY ? raw[u][t] : (raw[u][t] >> ca.shift);
                const uint8_t* p = gin + (long long)min(pos + PD, k - 1) * bb;
#pragma unroll
                for (int t = 0; t < 8; ++t) raw[u][t] = load_raw<TINY>(p + t * s, ca, s);
                uint32_t cwv[NCW];
#pragma unroll
                for (int q = 0; q < NCW; ++q) cwv[q] = cw[pos * NCW + q];
                expand_wz(v);
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (j < n) {
                        const uint32_t a = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                        apply_nibble<0>(acc[j], a & 15u, v);
                        apply_nibble<4>(acc[j], a >> 4, v);
                    }
                }
            }
        }
    }

    if (!live) return;
#pragma unroll
    for (int j = 0; j < RC; ++j) {
        if (j < n) {
            const int o = chunk * RC + j;
            const int slot = (DECODE && slots) ? slots[(long long)g * rmax + o] : o;
            uint8_t* dst = out + (long long)g * out_gstride + (long long)slot * bb;
#pragma unroll
            for (int r = 0; r < 8; ++r) store_word(dst + r * s, c, ca, acc[j][r]);
        }
    }
}

// ------------------------------------------------------------------- decode prep
// One wave per group (persistent: each wave walks groups w, w + W, ...; the GF log/exp
// tables are staged in LDS once per workgroup).  Restates the reference's decode
// bookkeeping (sort_blocks :543-575, erasure list, recovery row rewrite :791) and replaces
// its GF(2) bitmatrix elimination by a GF(256) Gauss-Jordan inverse of the r x r erasure
// submatrix S[i][j] = C[y_i][e_j]: since c -> (8x8 expansion) is a ring homomorphism, the
// inverse bitmatrix is the expansion of S^-1, and the recovered data is unique.  Output:
//   recovered e_j = sum_i Sinv[j][i] * R_i + sum_{x present} (sum_i Sinv[j][i] C[y_i][x]) * D_x
// so one coefficient per (j, input slot) and a single pass over the received blocks.
// Lanes of one wave exchange data through LDS without barriers: a wave's LDS operations
// execute in order, so wave_sync() only has to stop the compiler from reordering them.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

struct PrepScratch {
    uint8_t* rowl;      // 256
    uint8_t* present;   // 256
    uint8_t* recpos;    // 256: slot of recovery i
    uint8_t* era;       // 256: erased row j
    uint8_t* recidx;    // 256: recovery index of slot (255 = original)
    uint8_t* mat;       // rmax x (2 rmax)
};

__device__ __forceinline__ void prep_group(
    long long g, int lane, const uint8_t* gexp, const uint8_t* glog, const PrepScratch& sc,
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* cenc, uint8_t* __restrict__ coef, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, int k, int m, int bb, int rc,
    int rmax, int nchunk, bool syndrome) {
    uint8_t* rowl = sc.rowl;
    uint8_t* present = sc.present;
    uint8_t* recpos = sc.recpos;
    uint8_t* era = sc.era;
    uint8_t* recidx = sc.recidx;
    uint8_t* mat = sc.mat;
    const int rcp = rc < 4 ? 4 : rc;
    for (int i = lane; i < 256; i += 64) {
        present[i] = 0;
        recidx[i] = 255;
    }
    const uint8_t* rg = rows_in + g * k;
    uint8_t* ro = rows_out ? rows_out + g * k : nullptr;   // null: recovered-blocks layout
    uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
    for (int i = lane; i < k; i += 64) rowl[i] = rg[i];
    wave_sync();
    // present[x] != 0: data row x received; syndrome mode keeps one of its slots + 1
    for (int i = lane; i < k; i += 64)
        if (rowl[i] < k) present[rowl[i]] = syndrome ? (uint8_t)(i + 1) : 1;
    wave_sync();
    // recovery blocks in array order (sort_blocks)
    int nrec = 0;
    for (int base = 0; base < k; base += 64) {
        const int i = base + lane;
        const bool isrec = i < k && rowl[i] >= k;
        const unsigned long long msk = __ballot(isrec);
        const int pre = __popcll(msk & ((1ull << lane) - 1));
        if (isrec) {
            recpos[nrec + pre] = (uint8_t)i;
            recidx[i] = (uint8_t)(nrec + pre);
        }
        nrec += __popcll(msk);
    }
    // erasures: the first nrec data rows not present, ascending
    int nera = 0;
    for (int base = 0; base < k && nera < nrec; base += 64) {
        const int x = base + lane;
        const bool miss = x < k && !present[x];
        const unsigned long long msk = __ballot(miss);
        const int pre = __popcll(msk & ((1ull << lane) - 1));
        if (miss && nera + pre < nrec) era[nera + pre] = (uint8_t)x;
        nera += __popcll(msk);
    }
    wave_sync();

    uint8_t* tb = coef + g * (long long)nchunk * k * rcp;   // syndrome table (syn::)
    auto finish_unchanged = [&](int st) {
        if (syndrome) {
            // a stream of k extras in slot order that feeds no syndrome row: the apply
            // kernel still reads every group's k blocks
            for (int i = lane; i < k; i += 64) tb[syn::kPerm + i] = (uint8_t)i;
            if (lane < 5) ((uint32_t*)(tb + syn::kMask))[lane] = 0;   // mask and need
            // gf_dcol: every row position a zero block, no extras
            for (int x = lane; x < 128; x += 64) tb[syn::kRowSlot + x] = 255;
            if (lane == 0) *(uint32_t*)(tb + syn::kNExt) = 0;
        }
        if (ro && ro != rg)
            for (int i = lane; i < k; i += 64) ro[i] = rowl[i];
        if (rec)
            for (int j = lane; j < rmax; j += 64) rec[j] = 255;
        if (lane == 0) {
            nout[g] = 0;
            if (status) status[g] = st;
        }
    };
    if (nrec == 0) { finish_unchanged(0); return; }                       // :1287-1289
    if (k + m > 256 || (bb & 7)) { finish_unchanged(-1); return; }        // :1292-1294
    if (nrec > rmax || nera < nrec) { finish_unchanged(-3); return; }     // malformed rows
    const int n = nrec;
    const int n2 = 2 * n;
    bool bad = false;
    for (int i = 0; i < n; ++i)
        if (rowl[recpos[i]] - k >= m) bad = true;                          // row >= k + m
    if (bad) { finish_unchanged(-3); return; }

    // [S | I]
    for (int idx = lane; idx < n * n2; idx += 64) {
        const int i = idx / n2, j = idx % n2;
        uint8_t v;
        if (j < n) v = cenc[(rowl[recpos[i]] - k) * k + era[j]];
        else v = (j - n == i) ? 1 : 0;
        mat[i * n2 + j] = v;
    }
    wave_sync();
    auto mul = [&](uint8_t a, uint8_t b) -> uint8_t {
        return (a && b) ? gexp[glog[a] + glog[b]] : 0;
    };
    for (int p = 0; p < n; ++p) {
        int piv = -1;
        for (int base = p; base < n && piv < 0; base += 64) {
            const int i = base + lane;
            const unsigned long long msk = __ballot(i < n && mat[i * n2 + p] != 0);
            if (msk) piv = base + __ffsll((long long)msk) - 1;
        }
        if (piv < 0) { finish_unchanged(-3); return; }                     // singular
        if (piv != p) {
            for (int j = lane; j < n2; j += 64) {
                const uint8_t t = mat[p * n2 + j];
                mat[p * n2 + j] = mat[piv * n2 + j];
                mat[piv * n2 + j] = t;
            }
            wave_sync();
        }
        const uint8_t inv = gexp[255 - glog[mat[p * n2 + p]]];
        wave_sync();
        for (int j = lane; j < n2; j += 64) mat[p * n2 + j] = mul(mat[p * n2 + j], inv);
        wave_sync();
        for (int i = 0; i < n; ++i) {
            if (i == p) continue;
            const uint8_t f = mat[i * n2 + p];
            wave_sync();
            if (f)
                for (int j = lane; j < n2; j += 64) mat[i * n2 + j] ^= mul(f, mat[p * n2 + j]);
            wave_sync();
        }
    }

    if (syndrome) {
        // recovered e_j = sum_i Sinv[j][i] T_i with the syndromes
        // T_i = R_i ^ sum_{data slots} C[y_i][row] D_slot (cauchy_256.cpp:1269-1420: the
        // originals are eliminated from the recovery rows, then the r x r system is solved)
        int np = 0;
        for (int base = 0; base < 128; base += 64) {   // present rows ascending, k <= 128
            const int x = base + lane;
            const bool pres = x < k && present[x] != 0;
            const unsigned long long msk = __ballot(pres);
            const int pre = __popcll(msk & ((1ull << lane) - 1));
            if (pres) tb[syn::kPerm + np + pre] = (uint8_t)(present[x] - 1);
            if (lane < 2)
                ((uint32_t*)(tb + syn::kMask))[base / 32 + lane] = (uint32_t)(msk >> (32 * lane));
            np += __popcll(msk);
        }
        int ne = 0;
        for (int base = 0; base < k; base += 64) {    // extras in slot order
            const int i = base + lane;
            const bool ext = i < k && (rowl[i] >= k || present[rowl[i]] != i + 1);
            const unsigned long long msk = __ballot(ext);
            const int pre = __popcll(msk & ((1ull << lane) - 1));
            if (ext) {
                tb[syn::kPerm + np + ne + pre] = (uint8_t)i;
                tb[syn::kERow + ne + pre] = rowl[i];
            }
            ne += __popcll(msk);
        }
        // gf_dcol: the slot of each data row (255: erased), the parity row of each syndrome,
        // the count of extras
        for (int x = lane; x < 128; x += 64)
            tb[syn::kRowSlot + x] = x < k && present[x] ? (uint8_t)(present[x] - 1) : (uint8_t)255;
        if (lane < n) tb[syn::kYmap + lane] = (uint8_t)(rowl[recpos[lane]] - k);
        if (lane == 0) *(uint32_t*)(tb + syn::kNExt) = (uint32_t)ne;
        uint32_t need = 0;
        for (int i = 0; i < n; ++i) need |= 1u << (rowl[recpos[i]] - k);
        if (lane < n) tb[syn::kISlot + rowl[recpos[lane]] - k] = (uint8_t)lane;
        if (lane == 0) *(uint32_t*)(tb + syn::kNeed) = need;
        for (int idx = lane; idx < n * n; idx += 64) {
            const int j = idx / n, i = idx % n;
            tb[syn::kSinv + j * 16 + i] = mat[j * n2 + n + i];
        }
    }
    // recovery coefficients per (output j, input slot pos)
    for (int pos = lane; pos < k && !syndrome; pos += 64) {
        const int ri = recidx[pos];
        for (int j = 0; j < n; ++j) {
            const uint8_t* inv_row = mat + j * n2 + n;   // Sinv[j][*]
            uint8_t cval;
            if (ri != 255) {
                cval = inv_row[ri];
            } else {
                const int x = rowl[pos];
                cval = 0;
                for (int i = 0; i < n; ++i)
                    cval ^= mul(inv_row[i], cenc[(rowl[recpos[i]] - k) * k + x]);
            }
            const int ch = j / rc, jj = j % rc;
            coef[g * (long long)nchunk * k * rcp + ((long long)ch * k + pos) * rcp + jj] = cval;
        }
    }
    if (ro && ro != rg)
        for (int i = lane; i < k; i += 64) ro[i] = rowl[i];
    wave_sync();
    for (int j = lane; j < n; j += 64) {
        slots[g * rmax + j] = recpos[j];
        if (ro) ro[recpos[j]] = era[j];                                    // :791
    }
    if (rec)
        for (int j = lane; j < rmax; j += 64) rec[j] = j < n ? era[j] : 255;
    if (lane == 0) {
        nout[g] = n;
        if (status) status[g] = 0;
    }
}

__global__ __launch_bounds__(256) void decode_prep_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ coef, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rc, int rmax, int nchunk, int scratch_bytes, int syndrome) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* gexp = smem;              // 512
    uint8_t* glog = gexp + 512;        // 256
    uint8_t* lcenc = glog + 256;       // m x k encode matrix (the inner loops read it at random)
    const int cbytes = (m * k + 15) & ~15;
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    __syncthreads();
    const int nwv = blockDim.x >> 6;
    const int w = wave_id(), lane = threadIdx.x & 63;
    uint8_t* base = lcenc + cbytes + (size_t)w * scratch_bytes;
    PrepScratch sc{base, base + 256, base + 512, base + 768, base + 1024, base + 1280};
    for (long long g = (long long)blockIdx.x * nwv + w; g < groups;
         g += (long long)gridDim.x * nwv)
        prep_group(g, lane, gexp, glog, sc, rows_in, rows_out, status, lcenc, coef, slots, nout,
                   rec_rows, k, m, bb, rc, rmax, nchunk, syndrome != 0);
}

// Decode prep with SIXTEEN lanes per group for small groups with up to 16 erasures (k <= 64:
// the QuicR presets (5, 5) .. (15, 15) at 1350-byte payloads).  Same bookkeeping, status
// codes and outputs as prep_group (cauchy_256.cpp:543-575, :791, :1287-1294).  The 16 lanes
// split the slots (bookkeeping by ballots), then the columns of [S | I] (lane l owns columns
// l and l + 16 of the group's n x 2n matrix in LDS) for the Gauss-Jordan inverse, then the
// slots again for the per-slot coefficients.  A wave holds four groups and the lanes of a
// group exchange data through LDS in program order (one wave: no barrier).  prep_group runs
// one group per wave through a chain of wave-wide LDS round trips: 270 us for 65,536
// (10, 10) groups with 5 losses.
constexpr int kWideLanes = 16;
__global__ __launch_bounds__(256) void decode_prep_wide_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ coef, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rc, int rmax, int nchunk) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    constexpr int GPB = 256 / kWideLanes;                       // groups per block
    __shared__ uint8_t lrows[GPB][64];
    __shared__ uint8_t lmat[GPB][16][32];                       // [S | I], row-major
    __shared__ uint8_t llist[GPB][3][16];                       // recpos, y, era
    extern __shared__ __attribute__((aligned(16))) uint8_t lcenc[];   // m x k
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    const long long gfirst = (long long)blockIdx.x * GPB;
    const int ng = (int)min((long long)GPB, groups - gfirst);
    for (int i = threadIdx.x; i < ng * k; i += blockDim.x)
        lrows[i / k][i % k] = rows_in[gfirst * k + i];
    __syncthreads();
    const int gl = threadIdx.x / kWideLanes, l = threadIdx.x % kWideLanes;
    const int seg = (threadIdx.x & 63) / kWideLanes;            // the group's 16 lanes in the wave
    if (gl >= ng) return;                                       // whole groups: no barrier below
    const long long g = gfirst + gl;
    const uint8_t* rg = lrows[gl];
    uint8_t (*M)[32] = lmat[gl];
    uint8_t* lrec = llist[gl][0];
    uint8_t* ly = llist[gl][1];
    uint8_t* lera = llist[gl][2];
    auto mul = [&](int a, int b) -> int { return (a && b) ? gexp[glog[a] + glog[b]] : 0; };

    // ---- bookkeeping: slot i = 16 q + l.  isrec: bit i = slot i holds a recovery block;
    // present: bit r = data row r was received (OR over the group's lanes)
    uint64_t isrec = 0, present = 0;
    bool badrow = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = kWideLanes * q + l;
        const int r = i < k ? rg[i] : 0;
        const bool rec = i < k && r >= k;
        if (i < k && r < k) present |= 1ull << r;
        const uint64_t b = __ballot(rec);
        isrec |= ((b >> (kWideLanes * seg)) & 0xFFFFull) << (kWideLanes * q);
    }
#pragma unroll
    for (int o = 1; o < kWideLanes; o <<= 1) present |= __shfl_xor(present, o, kWideLanes);
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
    if (l < nrec && l < 16) badrow = myy >= m;
    const bool anybad = (__ballot(badrow) >> (kWideLanes * seg)) & 0xFFFFull;
    uint8_t* ro = rows_out ? rows_out + g * k : nullptr;        // null: recovered-blocks layout
    const uint8_t* rgg = rows_in + g * k;
    uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
    auto finish_unchanged = [&](int st) {
        if (ro && ro != rgg)
            for (int i = l; i < k; i += kWideLanes) ro[i] = rg[i];
        if (rec)
            for (int j = l; j < rmax; j += kWideLanes) rec[j] = 255;
        if (l == 0) {
            nout[g] = 0;
            if (status) status[g] = st;
        }
    };
    if (nrec == 0) { finish_unchanged(0); return; }                       // :1287-1289
    if (k + m > 256 || (bb & 7)) { finish_unchanged(-1); return; }        // :1292-1294
    if (nrec > rmax || nera < nrec || anybad) { finish_unchanged(-3); return; }   // malformed
    const int n = nrec;                                                   // <= rmax <= 16
    if (l < n) {
        lrec[l] = (uint8_t)myrec;
        ly[l] = (uint8_t)myy;
        lera[l] = (uint8_t)myera;
    }
    wave_sync();
    // ---- [S | I], S[i][j] = C[y_i][e_j]: lane l fills columns l and l + 16
    for (int i = 0; i < n; ++i) {
        const int yi = ly[i];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = l + kWideLanes * h;
            if (c < 2 * n) M[i][c] = c < n ? lcenc[yi * k + lera[c]] : (uint8_t)(c - n == i);
        }
    }
    wave_sync();
    // ---- Gauss-Jordan (the lanes own columns; rows through LDS)
    for (int p = 0; p < n; ++p) {
        int piv = -1;
        for (int i = p; i < n && piv < 0; ++i)
            if (M[i][p]) piv = i;                                 // the same for every lane
        if (piv < 0) { finish_unchanged(-3); return; }             // singular
        if (piv != p) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = l + kWideLanes * h;
                if (c < 2 * n) {
                    const uint8_t t = M[p][c];
                    M[p][c] = M[piv][c];
                    M[piv][c] = t;
                }
            }
            wave_sync();
        }
        const int inv = gexp[255 - glog[M[p][p]]];
        wave_sync();                                              // every lane read M[p][p]
        int rowp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = l + kWideLanes * h;
            rowp[h] = c < 2 * n ? mul(M[p][c], inv) : 0;
            if (c < 2 * n) M[p][c] = (uint8_t)rowp[h];
        }
        for (int i = 0; i < n; ++i) {
            if (i == p) continue;
            const int f = M[i][p];                               // before column p changes
            wave_sync();
            if (f) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = l + kWideLanes * h;
                    if (c < 2 * n) M[i][c] ^= (uint8_t)mul(f, rowp[h]);
                }
            }
            wave_sync();
        }
    }
    // ---- coefficients per (output j, input slot pos): recovery slot ri: Sinv[j][ri]; data
    // row x: sum_i Sinv[j][i] C[y_i][x]
    for (int pos = l; pos < k; pos += kWideLanes) {
        const bool isr = (isrec >> pos) & 1;
        const int ri = isr ? __popcll(isrec & ((1ull << pos) - 1)) : -1;
        const int x = rg[pos];
        for (int j = 0; j < n; ++j) {
            int cval;
            if (isr) {
                cval = M[j][n + ri];
            } else {
                cval = 0;
                for (int i = 0; i < n; ++i) cval ^= mul(M[j][n + i], lcenc[ly[i] * k + x]);
            }
            const int ch = j / rc, jj = j % rc;
            coef[g * (long long)nchunk * k * (rc < 4 ? 4 : rc) + ((long long)ch * k + pos) *
                 (rc < 4 ? 4 : rc) + jj] = (uint8_t)cval;
        }
    }
    if (ro && ro != rgg)
        for (int i = l; i < k; i += kWideLanes) ro[i] = rg[i];
    wave_sync();
    if (l < n) {
        slots[g * rmax + l] = lrec[l];
        if (ro) ro[lrec[l]] = lera[l];                                     // :791
    }
    if (rec)
        for (int j = l; j < rmax; j += kWideLanes) rec[j] = j < n ? lera[j] : 255;
    if (l == 0) {
        nout[g] = n;
        if (status) status[g] = 0;
    }
}

// Decode prep with four LANES per group, for small erasure counts (rmax <= 4, k <= 64: the
// 1350-byte configs).  Same bookkeeping, status codes and outputs as prep_group above
// (cauchy_256.cpp:543-575, :791, :1287-1294); the r x r inverse and the per-slot
// coefficients are computed in registers with the GF(256) log/exp tables in LDS, so a
// group costs a few hundred independent LDS reads instead of a chain of wave-wide LDS
// round trips (prep_group: ~90 us for 65,536 (32, 4) groups, most of it latency).
// Packed small lists: byte j of recpos/recrow/era = entry j (j < 4).
__global__ __launch_bounds__(256) void decode_prep_lane_kernel(
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    const uint8_t* __restrict__ cenc, uint8_t* __restrict__ coef, uint8_t* __restrict__ slots,
    int32_t* __restrict__ nout, uint8_t* __restrict__ rec_rows, long long groups, int k, int m,
    int bb, int rmax) {
    // LDS: exp/log tables, the m x k encode matrix, the block's row tags [256][k] (loaded
    // coalesced) and its coefficient dwords [256][k + 1] (stored coalesced at the end)
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    extern __shared__ __attribute__((aligned(16))) uint8_t lsm[];
    uint8_t* lcenc = lsm;                                       // m x k (padded to 16)
    constexpr int LPG = 4;                                      // lanes per group
    constexpr int GPB = 256 / LPG;                              // groups per block
    uint8_t* lrows = lsm + ((m * k + 15) & ~15);                // GPB x k
    uint32_t* lcoef = (uint32_t*)(lrows + GPB * k);             // GPB x (k + 1), k % 4 == 0
    for (int i = threadIdx.x; i < 512; i += blockDim.x) gexp[i] = c_gf.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) glog[i] = c_gf.log[i];
    for (int i = threadIdx.x; i < m * k; i += blockDim.x) lcenc[i] = cenc[i];
    const long long gfirst = (long long)blockIdx.x * GPB;
    const int ng = (int)min((long long)GPB, groups - gfirst);
    {
        const uint32_t* src = (const uint32_t*)(rows_in + gfirst * k);   // 4-byte aligned
        const int nd = ng * k / 4;
#pragma unroll 4
        for (int i = threadIdx.x; i < nd; i += blockDim.x) ((uint32_t*)lrows)[i] = src[i];
    }
    __syncthreads();
    // LPG lanes per group: each runs the bookkeeping and the r x r inverse (cheap) and
    // computes the coefficients of every LPG-th input slot; lane q == 0 writes the rest
    const int gl = threadIdx.x / LPG, q = threadIdx.x % LPG;
    const long long g = gfirst + gl;
    const bool live = gl < ng;
    const bool lead = live && q == 0;
    const uint8_t* rg = lrows + gl * k;                         // this group's tags (LDS)
    const uint8_t* rgg = rows_in + g * k;
    uint8_t* ro = rows_out ? rows_out + g * k : nullptr;
    uint8_t* rec = rec_rows ? rec_rows + g * rmax : nullptr;
    uint32_t* mycoef = lcoef + gl * (k + 1);
    // every lane runs the body (dead lanes on a copy of lane 0's tags, no global writes)
    // so that the block reaches the coalesced coefficient store together
    if (!live) rg = lrows;

    // tags four at a time (k % 4 == 0, rows 4-byte aligned in LDS)
    const uint32_t* rg4 = (const uint32_t*)rg;
    uint64_t present = 0;
    int nrec = 0;
    uint32_t recpos = 0, recrow = 0;
    for (int i4 = 0; i4 < k; i4 += 4) {
        const uint32_t t4 = rg4[i4 >> 2];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i4 + u;
            const int r = (int)((t4 >> (8 * u)) & 0xFF);
            if (r < k) {
                present |= 1ull << r;
            } else {
                if (nrec < 4) {
                    recpos |= (uint32_t)i << (8 * nrec);
                    recrow |= (uint32_t)(r - k < 255 ? r - k : 255) << (8 * nrec);
                }
                ++nrec;
            }
        }
    }
    const uint64_t kmask = k == 64 ? ~0ull : ((1ull << k) - 1);
    uint64_t missing = ~present & kmask;
    const int nera = __popcll(missing);

    // a group left unchanged writes no coefficients (nout = 0: the apply skips it)
    auto finish_unchanged = [&](int st) {
        if (!lead) return;
        if (ro && ro != rgg)
            for (int i = 0; i < k; ++i) ro[i] = rg[i];
        if (rec)
            for (int j = 0; j < rmax; ++j) rec[j] = 255;
        nout[g] = 0;
        if (status) status[g] = st;
    };
    int early = 1;   // status of a group that needs no coefficients; 1 = go on
    if (nrec == 0) early = 0;                                               // :1287-1289
    else if (k + m > 256 || (bb & 7)) early = -1;                           // :1292-1294
    else if (nrec > rmax || nera < nrec) early = -3;                        // malformed rows
    else
        for (int i = 0; i < nrec; ++i)
            if ((int)((recrow >> (8 * i)) & 0xFF) >= m) early = -3;         // row >= k + m
    const int n = early == 1 ? nrec : 0;
    uint32_t era = 0;
    for (int j = 0; j < n; ++j) {
        const int e = __ffsll((long long)missing) - 1;
        missing &= missing - 1;
        era |= (uint32_t)e << (8 * j);
    }
    auto B = [](uint32_t v, int j) -> int { return (int)((v >> (8 * j)) & 0xFF); };
    auto mul = [&](int a, int b) -> int { return (a && b) ? gexp[glog[a] + glog[b]] : 0; };

    // [S | I], S[i][j] = C[y_i][e_j]; Gauss-Jordan fully unrolled over the 4 x 8 maximum
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
    // log of S^-1 (256 = zero)
    int lsi[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int v = (j < n && i < n) ? M[j][4 + i] : 0;
            lsi[j][i] = v ? glog[v] : 256;
        }
    // coefficient dword per input slot: byte j = recovered row j's coefficient
    for (int pos4 = 4 * q; pos4 < k; pos4 += 4 * LPG) {
      const uint32_t t4 = rg4[pos4 >> 2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {   // four independent lookup chains
        const int pos = pos4 + u;
        int ri = -1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < n && B(recpos, i) == pos) ri = i;
        uint32_t cw = 0;
        if (ri >= 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < n) {
                    int v = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (i == ri) v = M[j][4 + i];
                    cw |= (uint32_t)v << (8 * j);
                }
        } else if (n > 0) {
            const int x = (int)((t4 >> (8 * u)) & 0xFF);
            int acc[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i < n) {
                    const int cv = lcenc[B(recrow, i) * k + x];
                    if (cv) {
                        const int lc = glog[cv];
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (j < n && lsi[j][i] != 256) acc[j] ^= gexp[lsi[j][i] + lc];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) cw |= (uint32_t)acc[j] << (8 * j);
        }
        mycoef[pos] = cw;
      }
    }
    if (early != 1) {
        finish_unchanged(early);
    } else if (lead) {
        if (ro && ro != rgg)
            for (int i = 0; i < k; ++i) ro[i] = rg[i];
        for (int j = 0; j < n; ++j) {
            slots[g * rmax + j] = (uint8_t)B(recpos, j);
            if (ro) ro[B(recpos, j)] = (uint8_t)B(era, j);                // :791
        }
        if (rec)
            for (int j = 0; j < rmax; ++j) rec[j] = j < n ? (uint8_t)B(era, j) : 255;
        nout[g] = n;
        if (status) status[g] = 0;
    }
    __syncthreads();
    // coalesced store of the block's coefficient rows [ng][k] dwords
    uint32_t* cdst = (uint32_t*)(coef + gfirst * (long long)k * 4);
    const int nd = ng * k;
#pragma unroll 4
    for (int d = threadIdx.x; d < nd; d += blockDim.x) {
        const int gg = d / k;
        cdst[d] = lcoef[gg * (k + 1) + (d - gg * k)];
    }
}

// In-place decode with more recovered blocks than one wave holds: the chunks write to a
// [G][rmax][bb] scratch, then this copies each recovered block into its slot.
__global__ __launch_bounds__(256) void scatter_recovered_kernel(
    const uint8_t* __restrict__ scratch, uint8_t* __restrict__ out,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, int k, int bb,
    int rmax, long long units) {
    const long long u = (long long)blockIdx.x * 4 + wave_id();
    if (u >= units) return;
    const long long g = u / rmax;
    const int o = (int)(u % rmax);
    if (o >= nout[g]) return;
    const int lane = threadIdx.x & 63;
    const uint8_t* from = scratch + u * (long long)bb;
    uint8_t* to = out + (g * k + slots[g * rmax + o]) * (long long)bb;
    for (int q = lane; q < bb; q += 64) to[q] = from[q];
}

// ----------------------------------------------------------------------- synth
__device__ __forceinline__ uint64_t splitmix64_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ void synth_fill_kernel(uint8_t* __restrict__ dst, unsigned long long bytes,
                                  unsigned long long seed, unsigned long long off) {
    // requires off % 8 == 0; word i of dst = stream word off/8 + i
    const unsigned long long nwords = bytes / 8;
    const unsigned long long w0 = off / 8;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
         i < nwords; i += (unsigned long long)gridDim.x * blockDim.x)
        ((uint64_t*)dst)[i] = splitmix64_mix(seed + (w0 + i + 1) * 0x9E3779B97F4A7C15ULL);
    const unsigned long long tail = bytes - nwords * 8;
    if (blockIdx.x == 0 && threadIdx.x < tail) {
        const uint64_t w = splitmix64_mix(seed + (w0 + nwords + 1) * 0x9E3779B97F4A7C15ULL);
        dst[nwords * 8 + threadIdx.x] = (uint8_t)(w >> (8 * threadIdx.x));
    }
}

__global__ __launch_bounds__(256) void synth_gather_kernel(
    const uint8_t* __restrict__ data, const uint8_t* __restrict__ parity,
    const int16_t* __restrict__ src, uint8_t* __restrict__ blocks, int k, int m, int bb,
    long long units) {
    const long long u = (long long)blockIdx.x * 4 + wave_id();
    if (u >= units) return;
    const int lane = threadIdx.x & 63;
    const long long g = u / k;
    const int sidx = src[u];
    const uint8_t* from = sidx < k ? data + (g * k + sidx) * (long long)bb
                                   : parity + (g * m + (sidx - k)) * (long long)bb;
    uint8_t* to = blocks + u * (long long)bb;
    if ((bb & 7) == 0) {
        for (int q = lane; q < bb / 8; q += 64) ((u64a*)to)[q] = ((const u64a*)from)[q];
    } else {
        for (int q = lane; q < bb; q += 64) to[q] = from[q];
    }
}

// ---------------------------------------------------------------------- launchers
static inline unsigned blocks_for_waves(long long waves) { return (unsigned)((waves + 3) / 4); }

// 16-byte units need 8-byte alignment of both buffers and of every block; otherwise
// unaligned 4-byte units; blocks under 4 bytes go bytewise.
static int xor_unit(const void* a, const void* b, long long s1, long long s2, int bb) {
    const uintptr_t al = (uintptr_t)a | (uintptr_t)b | (uintptr_t)s1 | (uintptr_t)s2 |
                         (uintptr_t)bb;
    if (bb >= 16 && (al & 7) == 0) return 16;
    return bb >= 4 ? 4 : 1;
}

template <int VS, bool DECODE>
static void xor_flat_launch(const uint8_t* in, uint8_t* out, const uint8_t* eidx, int k, int bb,
                            long long G, long long igs, long long ogs, hipStream_t st,
                            long long es) {
    const int nu = (bb + VS - 1) / VS;
    const unsigned total = (unsigned)(G * nu);
    const unsigned nb = (total + 255) / 256;
    switch (k) {
        case 10: qlaunch((xor_flat_kernel<VS, 10, DECODE>), dim3(nb), dim3(256), 0, st, in, out, eidx, k, bb, nu, total, igs, ogs, es); break;
        case 32: qlaunch((xor_flat_kernel<VS, 32, DECODE>), dim3(nb), dim3(256), 0, st, in, out, eidx, k, bb, nu, total, igs, ogs, es); break;
        default: qlaunch((xor_flat_kernel<VS, 0, DECODE>), dim3(nb), dim3(256), 0, st, in, out, eidx, k, bb, nu, total, igs, ogs, es); break;
    }
}

template <bool DECODE>
static hipError_t xor_any(const uint8_t* in, uint8_t* out, const uint8_t* eidx, int k, int bb,
                          long long G, long long igs, long long ogs, hipStream_t st,
                          const Tune& t, long long es = -1) {
    if (es < 0) es = bb;
    if (G <= 0) return hipSuccess;
    if (es == bb && igs == (long long)k * bb && xor_dma_ok(in, out, k, bb, ogs, t))
        return launch_xor_dma(in, out, eidx, nullptr, nullptr, nullptr, k, bb, G, ogs, DECODE, st,
                              t);
    note_kernel(DECODE ? "xor_flat_kernel<decode>" : "xor_flat_kernel<encode>");
    const int vs = xor_unit(in, out, igs, ogs, bb);
    const long long units = G * ((bb + vs - 1) / vs);
    if (units > 0xffffffffLL) return hipErrorInvalidValue;
    if (vs == 16) xor_flat_launch<16, DECODE>(in, out, eidx, k, bb, G, igs, ogs, st, es);
    else if (vs == 4) xor_flat_launch<4, DECODE>(in, out, eidx, k, bb, G, igs, ogs, st, es);
    else qlaunch((xor_bytes_kernel<DECODE>), dim3((unsigned)((units + 255) / 256)), dim3(256), 0, st, in, out, eidx, k, bb, units, igs, ogs, es);
    return hipGetLastError();
}

hipError_t launch_xor_encode(const uint8_t* data, uint8_t* parity, int k, int bb,
                             long long groups, long long out_gstride, hipStream_t st,
                             const Tune& t) {
    return xor_any<false>(data, parity, nullptr, k, bb, groups, (long long)k * bb, out_gstride,
                          st, t);
}

hipError_t launch_xor_decode(const uint8_t* blocks, uint8_t* out, const uint8_t* rows_in,
                             uint8_t* rows_out, int32_t* status, uint8_t* eidx, int k, int bb,
                             long long groups, hipStream_t st, const Tune& t, bool compact) {
    if (groups <= 0) return hipSuccess;
    const long long gb = (long long)k * bb;
    const long long ogs = compact ? bb : gb;
    if (k <= 64 && xor_dma_ok(blocks, out, k, bb, ogs, t))
        // single launch: the DMA kernel also does the erased-slot / missing-row bookkeeping
        return launch_xor_dma(blocks, out, nullptr, rows_in, rows_out, status, k, bb, groups, ogs,
                              true, st, t, compact);
    note_kernel("m1_prep_kernel");
    qlaunch((m1_prep_kernel), dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, rows_in, rows_out, status,
                                                                     eidx, k, groups,
                                                                     compact ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return xor_any<true>(blocks, out, eidx, k, bb, groups, gb, ogs, st, t, compact ? 0 : bb);
}

hipError_t launch_replicate(const uint8_t* data, uint8_t* parity, int m, int bb,
                            long long groups, hipStream_t st) {
    if (groups <= 0 || m <= 0) return hipSuccess;
    const long long total = groups * m * (long long)bb;
    const unsigned nb = (unsigned)std::min<long long>((total + 255) / 256, 65536);
    note_kernel("replicate_kernel");
    qlaunch((replicate_kernel), dim3(nb), dim3(256), 0, st, data, parity, m, bb, groups);
    return hipGetLastError();
}

hipError_t launch_rec_k1(const uint8_t* blocks, const uint8_t* rows_in, uint8_t* rec,
                        uint8_t* rec_rows, int32_t* status, int bb, int rmax, long long groups,
                        hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    const long long total = groups * (long long)bb;
    const unsigned nb = (unsigned)std::min<long long>((total + 255) / 256, 65536);
    note_kernel("rec_k1_kernel");
    qlaunch((rec_k1_kernel), dim3(nb), dim3(256), 0, st, blocks, rows_in, rec, rec_rows, status, bb, rmax, groups);
    return hipGetLastError();
}

hipError_t launch_rows_k1(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                          long long groups, hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    note_kernel("rows_k1_kernel");
    qlaunch((rows_k1_kernel), dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, rows_in, rows_out, status,
                                                                     groups);
    return hipGetLastError();
}

template <bool DECODE>
static hipError_t gf_apply_dispatch(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                                    const uint8_t* slots, const int32_t* nout, int k, int m,
                                    int bb, long long groups, int rc, int nchunk, int rmax,
                                    long long coef_gstride, long long out_gstride,
                                    hipStream_t st, const Tune& t) {
    const int s = bb / 8;
    const int nw = (s + 3) / 4;
    const int ntiles = (nw + 63) / 64;
    const bool flat = !DECODE && s >= 4 && t.flat && (nw & 63) != 0;
    const long long flat_lanes = groups * nw;
    const long long units = flat ? nchunk * ((flat_lanes + 63) / 64) : groups * nchunk * ntiles;
    if (units <= 0) return hipSuccess;
    if (units > 0x7fffffffLL) return hipErrorInvalidValue;
    const unsigned nb = blocks_for_waves(units);
    const unsigned nthr = 256;
    const int tu = (int)units;
    const int pd = t.pd;
    if (pd < 1 || pd > 3) return hipErrorInvalidValue;
    note_kernel(DECODE ? "gf_apply_kernel<decode>"
                       : (flat ? "gf_apply_kernel<encode,flat>" : "gf_apply_kernel<encode>"));
#define QF_ARGS in, out, coef, slots, nout, k, m, bb, nw, ntiles, nchunk, rmax, coef_gstride, \
                out_gstride, tu, flat_lanes
#define QF_LAUNCH(RCV)                                                                        \
    do {                                                                                      \
        if (flat) {                                                                           \
            if constexpr (!DECODE)                                                            \
                qlaunch((gf_apply_kernel<RCV, false, false, 2, true>), dim3(nb), dim3(nthr), 0, st, QF_ARGS);    \
        } else if (s >= 4 && pd == 3)                                                         \
            qlaunch((gf_apply_kernel<RCV, DECODE, false, 3>), dim3(nb), dim3(nthr), 0, st, QF_ARGS);             \
        else if (s >= 4 && pd == 1)                                                           \
            qlaunch((gf_apply_kernel<RCV, DECODE, false, 1>), dim3(nb), dim3(nthr), 0, st, QF_ARGS);             \
        else if (s >= 4)                                                                      \
            qlaunch((gf_apply_kernel<RCV, DECODE, false, 2>), dim3(nb), dim3(nthr), 0, st, QF_ARGS);             \
        else                                                                                  \
            qlaunch((gf_apply_kernel<RCV, DECODE, true, 1>), dim3(nb), dim3(nthr), 0, st, QF_ARGS);              \
    } while (0)
    switch (rc) {
        case 1: QF_LAUNCH(1); break;
        case 2: QF_LAUNCH(2); break;
        case 4: QF_LAUNCH(4); break;
        case 8: QF_LAUNCH(8); break;
        case 16: QF_LAUNCH(16); break;
        default: return hipErrorInvalidValue;
    }
#undef QF_LAUNCH
#undef QF_ARGS
    return hipGetLastError();
}

hipError_t launch_gf_encode(const uint8_t* data, uint8_t* parity, const uint8_t* coef, int k,
                            int m, int bb, long long groups, int rc, hipStream_t st,
                            const Tune& t) {
    const int nchunk = (m + rc - 1) / rc;
    return gf_apply_dispatch<false>(data, parity, coef, nullptr, nullptr, k, m, bb, groups, rc,
                                    nchunk, 0, 0, (long long)m * bb, st, t);
}

hipError_t launch_decode_prep(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                              const uint8_t* cenc, DecodeWork w, int k, int m, int bb, int rc,
                              int rmax, long long groups, hipStream_t st, const Tune& t,
                              uint8_t* rec_rows, bool syndrome) {
    if (groups <= 0) return hipSuccess;
    if (syndrome && (k > 128 || m > 16 || (long long)((rmax + rc - 1) / rc) * k * std::max(rc, 4) <
                                                 syn::kBytes))
        return hipErrorInvalidValue;
    if (!syndrome && t.prep_lane && rmax <= 4 && k <= 64 && k % 4 == 0 && (long long)m * k <= 4096 && rc <= 4 &&
        ((((uintptr_t)w.coef) | (uintptr_t)rows_in) & 3) == 0) {
        const unsigned nb = (unsigned)((groups + 63) / 64);     // 64 groups x 4 lanes
        const size_t lds = (((size_t)m * k + 15) & ~(size_t)15) + 64 * (size_t)k +
                           64 * (size_t)(k + 1) * 4;
        note_kernel("decode_prep_lane_kernel");
        qlaunch((decode_prep_lane_kernel), dim3(nb), dim3(256), lds, st, 
            rows_in, rows_out, status, cenc, w.coef, w.slots, w.nout, rec_rows, groups, k, m, bb,
            rmax);
        return hipGetLastError();
    }
    const int nchunk = (rmax + rc - 1) / rc;
    if (!syndrome && t.prep_lane && k <= 64 && rmax <= 16 && (long long)m * k <= 16384) {
        note_kernel("decode_prep_wide_kernel");
        qlaunch((decode_prep_wide_kernel), dim3((unsigned)((groups + 15) / 16)), dim3(256),
                (uint32_t)(((size_t)m * k + 15) & ~(size_t)15), st, rows_in, rows_out, status,
                cenc, w.coef, w.slots, w.nout, rec_rows, groups, k, m, bb, rc, rmax, nchunk);
        return hipGetLastError();
    }
    const int scratch = (int)((1280 + (size_t)rmax * 2 * rmax + 15) & ~(size_t)15);
    const size_t fixed = 768 + (((size_t)m * k + 15) & ~(size_t)15);
    int nwv = 4;
    while (nwv > 1 && fixed + (size_t)nwv * scratch > 64 * 1024) nwv >>= 1;
    const size_t lds = fixed + (size_t)nwv * scratch;
    const long long want = (groups + nwv - 1) / nwv;
    const unsigned nb = (unsigned)std::min<long long>(want, (long long)t.cus * 16);
    note_kernel(syndrome ? "decode_prep_kernel<syndrome>" : "decode_prep_kernel");
    qlaunch((decode_prep_kernel), dim3(nb), dim3(nwv * 64), lds, st, rows_in, rows_out, status, cenc, w.coef,
                                                   w.slots, w.nout, rec_rows, groups, k, m, bb,
                                                   rc, rmax, nchunk, scratch, syndrome ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_gf_decode(const uint8_t* blocks, uint8_t* out, DecodeWork w, int k, int m,
                            int bb, long long groups, int rc, int rmax, hipStream_t st,
                            const Tune& t) {
    const int nchunk = (rmax + rc - 1) / rc;
    const int rcp = rc < 4 ? 4 : rc;
    return gf_apply_dispatch<true>(blocks, out, w.coef, w.slots, w.nout, k, m, bb, groups, rc,
                                   nchunk, rmax, (long long)nchunk * k * rcp,
                                   (long long)k * bb, st, t);
}

hipError_t launch_scatter_recovered(const uint8_t* scratch, uint8_t* out, DecodeWork w, int k,
                                   int bb, int rmax, long long groups, hipStream_t st) {
    const long long units = groups * rmax;
    if (units <= 0) return hipSuccess;
    note_kernel("scatter_recovered_kernel");
    qlaunch((scatter_recovered_kernel), dim3(blocks_for_waves(units)), dim3(256), 0, st, scratch, out, w.slots,
                                                                      w.nout, k, bb, rmax,
                                                                      units);
    return hipGetLastError();
}

hipError_t launch_gf_decode_scratch(const uint8_t* blocks, uint8_t* scratch, DecodeWork w,
                                   int k, int m, int bb, long long groups, int rc, int rmax,
                                   hipStream_t st, const Tune& t) {
    const int nchunk = (rmax + rc - 1) / rc;
    const int rcp = rc < 4 ? 4 : rc;
    return gf_apply_dispatch<true>(blocks, scratch, w.coef, nullptr, w.nout, k, m, bb, groups,
                                   rc, nchunk, rmax, (long long)nchunk * k * rcp,
                                   (long long)rmax * bb, st, t);
}

hipError_t launch_synth_fill(uint8_t* dst, unsigned long long bytes, unsigned long long seed,
                             unsigned long long byte_offset, hipStream_t st) {
    if (bytes == 0) return hipSuccess;
    if (byte_offset % 8) return hipErrorInvalidValue;
    const unsigned long long words = bytes / 8 + 1;
    const unsigned nb = (unsigned)std::min<unsigned long long>((words + 255) / 256, 1u << 16);
    qlaunch((synth_fill_kernel), dim3(nb), dim3(256), 0, st, dst, bytes, seed, byte_offset);
    return hipGetLastError();
}

hipError_t launch_synth_gather(const uint8_t* data, const uint8_t* parity, const int16_t* src,
                               uint8_t* blocks, int k, int m, int bb, long long groups,
                               hipStream_t st) {
    const long long units = groups * k;
    if (units <= 0) return hipSuccess;
    qlaunch((synth_gather_kernel), dim3(blocks_for_waves(units)), dim3(256), 0, st, data, parity, src, blocks, k,
                                                                 m, bb, units);
    return hipGetLastError();
}

}  // namespace qfec
