// xor_dma.hip — m = 1 XOR parity encode and 1-erasure decode (gfx950), the headline path.
//
// Reference: cauchy_256_encode with m = 1 writes P0 = XOR of the k data blocks
// (net/quic/core/libcat/cauchy_256.cpp:1519-1528); cauchy_decode_m1 (:486-540) XORs the
// k - 1 received blocks into the parity block and retags it with the missing data row.
//
// Shape: each wave owns groups g0, g0 + W, g0 + 2W, ... (persistent grid, W = waves in the
// grid) and streams whole groups (k * bb contiguous bytes) into a ring of NSLOT LDS slots
// with global_load_lds_dwordx4 nt, 1 KiB per wave instruction.  NSLOT - 1 groups are in
// flight while the wave XORs the oldest one out of LDS and writes the result with 8-byte
// non-temporal stores.  The whole group is in LDS before anything is stored, so an in-place
// decode has no read-after-write hazard.  Decode also does the cauchy_decode_m1 row
// bookkeeping with a ballot over the group's k <= 64 row tags, so m = 1 decode is one
// launch.
//
// Counted waits: every group costs NDMA DMA instructions plus, for decode, one row-tag
// load issued right AFTER its DMA; `s_waitcnt vmcnt((NSLOT - 1) * (NDMA + R))` then
// retires the oldest group and its tags while the younger groups stay in flight.  The
// stores of a finished group sit between two younger groups in the counter and only make
// that wait slightly conservative.
#include "fec_kernels.h"
#include "gf_bitslice.h"

namespace qfec {

#define QX_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QX_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int N>
__device__ __forceinline__ void xor_wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx9");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// m = 1 decode bookkeeping for one group, done by the wave that decodes it (k <= 64, one
// row tag per lane; cauchy_decode_m1, cauchy_256.cpp:486-540).  `r` is this lane's row
// tag (lanes >= k hold 255).  Returns the erased slot (-1 if none) and writes status and
// either the rewritten row tags (ro, slot layout) or the recovered data row (rec,
// recovered-blocks layout; 255 when nothing was erased).
__device__ __forceinline__ int m1_rows_wave(int r, int k, uint8_t* flags, uint8_t* ro,
                                            uint8_t* rec, int32_t* status, long long g) {
    const int lane = threadIdx.x & 63;
    const unsigned long long er = __ballot(lane < k && r >= k);
    const int e = er ? __ffsll((long long)er) - 1 : -1;
    flags[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    if (lane < k && lane != e && r < k) flags[r] = 1;
    __builtin_amdgcn_wave_barrier();
    const unsigned long long miss = __ballot(lane < k && !flags[lane]);
    if (lane < k) {
        int v = r;
        if (lane == e && miss) v = __ffsll((long long)miss) - 1;
        if (ro) ro[lane] = (uint8_t)v;
        if (rec && lane == e) rec[0] = (uint8_t)v;
    }
    if (rec && e < 0 && lane == 0) rec[0] = 255;
    if (status && lane == 0) status[g] = 0;
    return e;
}

// FUSED (decode only): rows_in/rows_out are handled here; otherwise eidx[g] names the
// erased slot (255 = none), prepared by m1_prep_kernel.
// PROBE (tools/microbench/xor_dec_mb.hip only; the library instantiates 0), decode
// timing probes: bit 0 = skip the row bookkeeping (slot 0 is taken as the erased one),
// bit 1 = write the result densely at out + g * bb, bit 2 = no tag DMA, bit 3 = plain
// (write-back) stores for the encode too.
// COMPACT (decode): recovered-blocks layout, the result of group g goes to out + g * bb and
// its data row to rows_out[g] (see qfec_decode_batch_recovered).
template <int NDMA, int NSLOT, bool DECODE, bool FUSED, int PROBE = 0, bool COMPACT = false>
__global__ __launch_bounds__(256) void xor_dma_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ eidx,
    const uint8_t* __restrict__ rows_in, uint8_t* rows_out, int32_t* __restrict__ status,
    int k, int bb, long long groups, long long out_gstride) {
    constexpr int SLOT = NDMA * 1024;
    constexpr int R = (DECODE && !(PROBE & 4)) ? 1 : 0;   // row-tag loads per group
    constexpr int WAIT = (NSLOT - 1) * (NDMA + R);
    constexpr int kTagBytes = 80;                     // 16-byte multiple >= 64 + 6
    static_assert(WAIT <= 63, "too many DMA instructions in flight for vmcnt");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int nwv = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
    const int w = wave_id(), lane = threadIdx.x & 63;
    uint8_t* myl = smem + (size_t)w * NSLOT * SLOT;
    uint8_t* flags = smem + (size_t)nwv * NSLOT * SLOT + w * 64;
    const long long W = (long long)gridDim.x * nwv;
    const long long g0 = (long long)blockIdx.x * nwv + w;
    if (g0 >= groups) return;
    const long long cnt =   // wave-uniform, kept in SGPRs (the division runs on the VALU)
        __builtin_amdgcn_readfirstlane((int)((groups - 1 - g0) / W + 1));   // groups of this wave
    const int gb = k * bb;
    constexpr bool fused = DECODE && FUSED;            // rows handled here (k <= 64)

    // Row tags (FUSED) or the erased-slot byte (eidx) of a group ride the same LDS-DMA
    // stream as its data: one dword-granular DMA instruction right after the group's
    // pieces, into a small per-slot tag window, so the counted wait covers them and no
    // loaded value is carried in registers across iterations (the compiler would wait for
    // such a value at every copy it makes of it).
    uint8_t* tagl = smem + (size_t)nwv * (NSLOT * SLOT + 64) + (size_t)w * NSLOT * kTagBytes;
    auto tag_addr = [&](long long gg) -> uintptr_t {
        return fused ? (uintptr_t)(rows_in + gg * k) : (uintptr_t)(eidx + gg);
    };
    auto issue = [&](long long i, int slot) {
        const long long gg = g0 + i * W;
        const uint8_t* src = in + gg * gb;
#pragma unroll
        for (int p = 0; p < NDMA; ++p) {
            const int off = min(p * 1024 + lane * 16, gb - 16);   // last piece: clamp inside
            __builtin_amdgcn_global_load_lds(QX_GPTR(src + off),
                                             QX_LPTR(myl + slot * SLOT + p * 1024), 16, 0, 2);
        }
        if (DECODE && !(PROBE & 4)) {
            const uintptr_t t = tag_addr(gg);
            const uintptr_t t0 = t & ~(uintptr_t)3;
            const int nd = (int)((t + (fused ? k : 1) + 3 - t0) >> 2);   // dwords, <= 18
            if (lane < nd)
                __builtin_amdgcn_global_load_lds(QX_GPTR(t0 + lane * 4),
                                                 QX_LPTR(tagl + slot * kTagBytes), 4, 0, 0);
        }
    };

#pragma unroll
    for (int u = 0; u < NSLOT - 1; ++u)
        if (u < cnt) issue(u, u);
    const int nq = bb >> 3;
#pragma unroll 1
    for (long long i0 = 0; i0 < cnt; i0 += NSLOT) {
#pragma unroll
        for (int u = 0; u < NSLOT; ++u) {
            const long long i = i0 + u;
            if (i >= cnt) break;
            const int ua = (u + NSLOT - 1) % NSLOT;
            if (i + NSLOT - 1 < cnt) {
                issue(i + NSLOT - 1, ua);
                xor_wait_vmcnt<WAIT>();   // group i and its tags landed
            } else {
                xor_wait_vmcnt<0>();
            }
            const long long g = g0 + i * W;
            int e = 0;
            if (DECODE && (PROBE & 1)) {
                e = 0;
            } else if (DECODE) {
                const uint8_t* tg = tagl + u * kTagBytes + (tag_addr(g) & 3);
                if (fused) {
                    const int r = lane < k ? tg[lane] : 255;
                    e = COMPACT ? m1_rows_wave(r, k, flags, nullptr, rows_out + g, status, g)
                                : m1_rows_wave(r, k, flags, rows_out + g * k, nullptr, status, g);
                } else {
                    e = tg[0];
                    if (e == 255) e = -1;
                }
            }
            if (!DECODE || e >= 0) {
                const uint8_t* L = myl + u * SLOT;
                uint8_t* o = (COMPACT || (PROBE & 2)) ? out + g * (long long)bb
                                                      : out + g * out_gstride + (long long)e * bb;
                for (int q = lane; q < nq; q += 64) {
                    uint64_t acc = *(const uint64_t*)(L + q * 8);
                    int x = 1;
                    for (; x + 1 < k; x += 2)
                        acc ^= *(const uint64_t*)(L + x * bb + q * 8) ^
                               *(const uint64_t*)(L + (x + 1) * bb + q * 8);
                    if (x < k) acc ^= *(const uint64_t*)(L + x * bb + q * 8);
                    // Decode writes one block per group, 13.5 KB apart in [G][k][bb]: plain
                    // write-back stores measured 3 % faster there than nt (6 % in place,
                    // where the slot's lines were just read); encode's dense parity
                    // stream is faster with nt (tools/microbench/xor_dec_mb.hip).
                    if ((DECODE && !COMPACT) || (PROBE & 8)) *(uint64_t*)(o + q * 8) = acc;
                    else __builtin_nontemporal_store(acc, (uint64_t*)(o + q * 8));
                }
            }
        }
    }
}

// ------------------------------------------------------------------------- launcher
namespace {

struct XorPlan {
    int ndma = 0, nslot = 2, waves = 3;
    size_t lds = 0;
};

// Ring shape: t.xor_slots x t.xor_waves (default 2 slots x 3 waves, the best of the
// 2-4 x 1-4 sweep in profiles/r01/A_*.txt).
bool xor_plan(int k, int bb, const Tune& t, XorPlan* p) {
    const long long gb = (long long)k * bb;
    if (bb % 8 != 0 || gb % 16 != 0 || gb < 16) return false;
    p->ndma = (int)((gb + 1023) / 1024);
    p->nslot = t.xor_slots;
    p->waves = t.xor_waves;
    if (p->nslot < 2 || p->nslot > 4 || p->waves < 1 || p->waves > 4) return false;
    p->lds = (size_t)p->waves * p->nslot * (p->ndma * 1024 + 80) + (size_t)p->waves * 64;
    if (p->lds > 160 * 1024) return false;
    if ((p->nslot - 1) * (p->ndma + 1) > 63) return false;
    return p->ndma <= 20;
}

template <bool DECODE, bool FUSED, bool COMPACT, int NSLOT, int N>
hipError_t xor_go(const XorPlan& p, const uint8_t* in, uint8_t* out, const uint8_t* eidx,
                  const uint8_t* rows_in, uint8_t* rows_out, int32_t* status, int k, int bb,
                  long long G, long long ogs, hipStream_t st, int cus) {
    if constexpr (N > 20 || (NSLOT - 1) * (N + (DECODE ? 1 : 0)) > 63) {
        return hipErrorInvalidValue;
    } else {
        if (p.ndma != N)
            return xor_go<DECODE, FUSED, COMPACT, NSLOT, N + 1>(p, in, out, eidx, rows_in, rows_out,
                                                                status, k, bb, G, ogs, st, cus);
        const long long want = (G + p.waves - 1) / p.waves;
        const unsigned nb = (unsigned)std::min<long long>(want, (long long)cus);
        // the wave's group count is a 32-bit SGPR value
        if ((G + (long long)nb * p.waves - 1) / ((long long)nb * p.waves) >= (1LL << 31))
            return hipErrorInvalidValue;
        note_kernel(DECODE ? (COMPACT ? "xor_dma_kernel<decode,recovered>"
                                      : "xor_dma_kernel<decode>")
                           : "xor_dma_kernel<encode>");
        qlaunch((xor_dma_kernel<N, NSLOT, DECODE, FUSED, 0, COMPACT>), dim3(nb), dim3(p.waves * 64), p.lds, st, 
            in, out, eidx, rows_in, rows_out, status, k, bb, G, ogs);
        return hipGetLastError();
    }
}

template <bool DECODE, bool FUSED, bool COMPACT = false>
hipError_t xor_dispatch(const XorPlan& p, const uint8_t* in, uint8_t* out, const uint8_t* eidx,
                        const uint8_t* rows_in, uint8_t* rows_out, int32_t* status, int k,
                        int bb, long long G, long long ogs, hipStream_t st, int cus) {
    switch (p.nslot) {
        case 2: return xor_go<DECODE, FUSED, COMPACT, 2, 1>(p, in, out, eidx, rows_in, rows_out, status, k, bb, G, ogs, st, cus);
        case 3: return xor_go<DECODE, FUSED, COMPACT, 3, 1>(p, in, out, eidx, rows_in, rows_out, status, k, bb, G, ogs, st, cus);
        case 4: return xor_go<DECODE, FUSED, COMPACT, 4, 1>(p, in, out, eidx, rows_in, rows_out, status, k, bb, G, ogs, st, cus);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool xor_dma_ok(const void* in, const void* out, int k, int bb, long long ogs, const Tune& t) {
    if (!t.dma) return false;
    XorPlan p;
    return xor_plan(k, bb, t, &p) && ((uintptr_t)in & 15) == 0 &&
           (((uintptr_t)out | (uintptr_t)ogs) & 7) == 0;
}

hipError_t launch_xor_dma(const uint8_t* in, uint8_t* out, const uint8_t* eidx,
                          const uint8_t* rows_in, uint8_t* rows_out, int32_t* status, int k,
                          int bb, long long groups, long long out_gstride, bool decode,
                          hipStream_t st, const Tune& t, bool compact) {
    if (groups <= 0) return hipSuccess;
    XorPlan p;
    if (!xor_plan(k, bb, t, &p)) return hipErrorInvalidValue;
    // the grid cap: one workgroup per CU, or (xor_wg) about xor_wg groups per wave
    const int cap = t.xor_wg > 0
                        ? (int)std::min<long long>((groups + (long long)p.waves * t.xor_wg - 1) /
                                                       ((long long)p.waves * t.xor_wg),
                                                   0x7fffffffLL)
                        : t.cus;
    if (!decode)
        return xor_dispatch<false, false>(p, in, out, eidx, rows_in, rows_out, status, k, bb,
                                          groups, out_gstride, st, cap);
    if (rows_in && compact)
        return xor_dispatch<true, true, true>(p, in, out, eidx, rows_in, rows_out, status, k,
                                              bb, groups, out_gstride, st, cap);
    if (rows_in)
        return xor_dispatch<true, true>(p, in, out, eidx, rows_in, rows_out, status, k, bb,
                                        groups, out_gstride, st, cap);
    return xor_dispatch<true, false>(p, in, out, eidx, rows_in, rows_out, status, k, bb, groups,
                                     out_gstride, st, cap);
}

}  // namespace qfec
