// gf_stream.hip — m > 1 encode / decode for groups of small blocks (bb <= 2 KiB, one column
// word of each sub-row per lane), the shape of BASELINE config B ((32 + 4) x 1352 B).
//
// Same arithmetic as gf_apply_kernel (bit-sliced Cauchy code, cauchy_256.cpp:90-125,
// :1502-1601, W/Z nibble expansion of gf_bitslice.h).  What differs is the memory path.
// Reading 169-byte sub-rows with per-lane dword loads tops out at ~4.5 TB/s on MI355X
// (tools/microbench/b_mem_mb.hip, variants a/e), while 1 KiB global_load_lds_dwordx4 pieces
// of whole groups stream at ~5.3 TB/s (variant d).  Earlier whole-group-in-LDS designs
// (gf_group.hip) lost that again: a group is 43 KB, so a CU holds three, and the waves
// that share one need barriers and an LDS reduction.
//
// Here every wave owns whole groups (g0, g0 + W, ...) and streams them through a private
// LDS ring of R one-KiB slots (a block that wraps round the ring end is read with wrapped
// per-lane addresses).  The wave consumes the blocks of a
// group in order; before block x it tops the ring up with the next pieces of its stream
// (crossing into its next group) and waits, with a counted `s_waitcnt vmcnt`, only for the
// pieces block x covers.  No barriers, no cross-wave traffic, about R - 4 pieces in flight
// per wave (R = 10: 10 KiB of LDS per wave, 16 waves per CU).  Lane c takes column word c of the 8 sub-rows of block x with
// unaligned ds_read_b32 (gfx950 unaligned LDS access), expands W/Z and applies the RC
// outputs, exactly like gf_apply.  The group's outputs are stored when its last block is
// done, through buffer stores whose out-of-range lanes are dropped, so the number of VMEM
// instructions per group is fixed and the vmcnt bookkeeping is exact.
//
// vmcnt bookkeeping: `vm` counts every VMEM instruction the wave issued (DMA pieces and
// stores); lane s of `vmv` holds the value of `vm` at the last instruction of the
// piece now in slot s.  VMEM instructions retire in issue order, so waiting for
// vmcnt <= vm - 1 - vmv[slot] retires that piece.  No other VMEM instruction may be
// emitted in the loop (coefficients, nout and slots come through s_load); the ISA check
// in tests/test_isa.py guards that.
//
// Decode: per-group coefficients from decode_prep_kernel ([G][1][k][RCP]), outputs go to
// slots[g][j] (or j, recovered-blocks layout) and groups with nout == 0 are skipped.  All of
// a group's blocks are in LDS before any of its stores, so in place is safe.
#include <utility>

#include "cauchy_const.h"
#include "fec_kernels.h"
#include "gf_bitslice.h"

namespace qfec {

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): a loop whose index is
// a compile-time constant in every iteration (the encode coefficients of a fixed (k, m)).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

#define QS_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define QS_LPTR(p) ((__attribute__((address_space(3))) void*)(p))
typedef uint32_t u32ua_s __attribute__((aligned(1)));

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

// Byte i of a 4-byte-aligned kernel-argument array through s_load_dword: a byte load
// (global_load_ubyte, or flat_load after an integer-to-pointer cast) would be a VMEM
// instruction outside the vmcnt bookkeeping, and its use would drain the ring.
__device__ __forceinline__ int sload_u8(const uint8_t* __restrict__ base, long long i) {
    const uint32_t wv = ((const uint32_t*)base)[i >> 2];
    return (int)((wv >> (8 * (i & 3))) & 0xFFu);
}

constexpr unsigned kSDrop = 0x80000000u;   // buffer offset past any range: lane dropped
constexpr int kStreamWaves = 4;            // waves per workgroup (independent)

// S = sub-row bytes (bb / 8), compile-time so the 8 sub-row reads are one address + ds
// offsets.  RC = outputs per group (one chunk: m <= RC for encode, rmax <= RC for decode).
// RCPT = byte stride of a coefficient row in the table (max(4, table rc)).  Encode is
// instantiated with RC = m exactly, so the per-output `j < n` test folds away (at run time
// the compiler turned it into a lane mask: 2 VALU + 2 SALU per output and block).
// KC > 0 (encode only): the code is fixed, k = KC and m = RC <= 6, and the coefficients come
// from cauchy_const.h at compile time.  The block loop is then fully unrolled and every
// 8x8 bit expansion folds into its straight-line XORs: no coefficient loads and no scalar
// nibble dispatch (about 9 scalar instructions per nibble in the run-time form).
template <int RC, int S, bool DECODE, int RCPT = (RC < 4 ? 4 : RC), int KC = 0>
__global__ __launch_bounds__(kStreamWaves * 64) void gf_stream_kernel(
    const uint8_t* in, uint8_t* out, const uint8_t* __restrict__ coef,
    const uint8_t* __restrict__ slots, const int32_t* __restrict__ nout, long long groups,
    int k, int m, int rmax, long long coef_gstride, long long out_gstride, int R) {
    constexpr int BB = 8 * S;
    constexpr int NW = (S + 3) / 4;                 // column words per sub-row
    constexpr int NWF = S / 4;                      // full words
    constexpr int NCW = RCPT / 4;
    static_assert(RCPT % 4 == 0 && RCPT >= RC, "coefficient row stride");
    constexpr int SPR = 1 + ((S >> 1) & 1) + (S & 1);   // store instructions per sub-row
    constexpr int SAUX = DECODE ? 0 : 2;   // encode's dense parity stream: nt stores
    static_assert(NW <= 64, "one column word per lane");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int w = wave_id();
    const int RB = R * 1024;
    uint8_t* ring = smem + (size_t)w * RB;
    const long long W = (long long)gridDim.x * kStreamWaves;
    const long long g0 = (long long)blockIdx.x * kStreamWaves + w;
    if (g0 >= groups) return;
    const long long cnt = (groups - 1 - g0) / W + 1;   // groups of this wave
    static_assert(KC == 0 || (!DECODE && RC >= 2 && RC <= 6), "compile-time codes: encode, m <= 6");
    if constexpr (KC > 0) k = KC;
    const int gb = k * BB;
    const int NP = (gb + 1023) >> 10;                  // pieces per group
    const int c = lane < NW ? lane : NW - 1;           // idle lanes shadow the last word

    // ---- issue side (wave-uniform): next piece iss_p of the stream, into slot iss_slot
    int iss_p = 0, iss_slot = 0;
    int issued = 0;                                    // pieces issued
    const int total = (int)cnt * NP;
    int vm = 0;                                        // VMEM instructions issued
    uint32_t vmv = 0;                                  // lane s: vm index of slot s's piece
    const uint8_t* isrc = in + g0 * gb;
    const long long istride = W * gb;

    auto issue_one = [&]() {
        const int off = min(iss_p * 1024 + lane * 16, gb - 16);   // last piece: clamp inside
        __builtin_amdgcn_global_load_lds(QS_GPTR(isrc + off), QS_LPTR(ring + iss_slot * 1024),
                                         16, 0, 2);
        ++vm;
        vmv = lane == iss_slot ? (uint32_t)(vm - 1) : vmv;
        ++issued;
        if (++iss_slot == R) iss_slot = 0;
        if (++iss_p == NP) {
            iss_p = 0;
            isrc += istride;
        }
    };
    // top the ring up: every piece from `head` on stays, the rest of the R slots refill
    auto fill = [&](int head) {
        while (issued < total && issued - head < R) issue_one();
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
    // column word c of the 8 sub-rows as aligned dword pairs (the block start is 4-byte
    // aligned: slots are 1 KiB and BB % 8 == 0, so sub-row t is misaligned by the
    // constant (t * S) & 3; v_alignbyte at use).  A block that ends at least 4 bytes
    // before the ring end is read as it lies (ds_read2 pairs; the highest byte read is
    // bp + BB + 3).  A block that wraps round the ring end (once per ring cycle) takes
    // per-lane wrapped addresses, min(a, a - RB) in unsigned arithmetic, one dword at a
    // time.  No mirror of the first slots is kept, so all R * 1 KiB of the wave's LDS are
    // ring slots (R = 10 at 16 waves per CU, against 8 slots + 2 KiB mirror before).
    auto read_block = [&](uint32_t bp, uint32_t (&lo)[8], uint32_t (&hi)[8]) {
        // the lane's byte offset, opaque to the optimiser: in the fully unrolled (KC > 0)
        // form it would otherwise precompute every block's addresses up front
        uint32_t c4 = 4u * (uint32_t)c;
        if constexpr (KC > 0) asm volatile("" : "+v"(c4));
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
                const uint32_t w0 = min(a0, a0 - (uint32_t)RB);
                lo[t] = *(const uint32_t*)(ring + w0);
                if (o & 3) {
                    const uint32_t a1 = a0 + 4u;
                    const uint32_t w1 = min(a1, a1 - (uint32_t)RB);
                    hi[t] = *(const uint32_t*)(ring + w1);
                } else {
                    hi[t] = 0u;
                }
            }
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
        const long long g = g0 + i * W;
        int n = DECODE ? nout[g] : RC;   // encode: RC == m
        n = n > RC ? RC : n;
        if (n > 0) {
            const uint32_t* cw = (const uint32_t*)(coef + (DECODE ? g * coef_gstride : 0));
            uint32_t acc[RC][8];
#pragma unroll
            for (int j = 0; j < RC; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[j][r] = 0;
            // Block x + 1's LDS reads are issued before block x is combined (software
            // pipeline); the ring keeps every piece from block x's first on, so block x's
            // pieces are not refilled while its reads may still be in flight.
            uint32_t bpos = (uint32_t)gslot0 * 1024u;          // ring position of block x
            uint32_t lo0[8], hi0[8], lo1[8], hi1[8];
            fill(gbase);
            wait_block(bpos);
            read_block(bpos, lo0, hi0);
            // xc: the block index, an int or (KC > 0) an integral_constant
            auto step = [&](auto xc, uint32_t (&lo)[8], uint32_t (&hi)[8], uint32_t (&nlo)[8],
                            uint32_t (&nhi)[8]) {
                const int x = xc;
                const uint32_t bn = next_pos(bpos);
                if (x + 1 < k) {
                    fill(gbase + ((x * BB) >> 10));
                    wait_block(bn);
                    read_block(bn, nlo, nhi);
                }
                bpos = bn;
                WZ v;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int o = t * S;
                    v.W[t] = (o & 3) ? __builtin_amdgcn_alignbyte(hi[t], lo[t], o & 3) : lo[t];
                }
                uint32_t cwv[NCW];
                if constexpr (KC == 0) {
#pragma unroll
                    for (int q = 0; q < NCW; ++q) cwv[q] = cw[x * NCW + q];
                }
                expand_wz(v);
                if constexpr (KC > 0) {
                    // row 0 is P0 (all ones); rows 1..m-1 with their compile-time coefficient
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                    static_for<RC - 1>([&](auto jc) {
                        constexpr int j = decltype(jc)::value + 1;
                        constexpr uint32_t cf = cauchy_coef_small(RC, j, decltype(xc)::value);
                        apply_nibble<0>(acc[j], cf & 15u, v);
                        apply_nibble<4>(acc[j], cf >> 4, v);
                    });
                    return;
                }
#pragma unroll
                for (int j = 0; j < RC; ++j) {
                    if (!DECODE && j == 0) {
                        // encode row 0 is P0, all coefficients 1 (cauchy_256.cpp:1519-1523):
                        // a plain XOR, no scalar nibble dispatch
#pragma unroll
                        for (int r = 0; r < 8; ++r) acc[0][r] ^= v.W[r];
                    } else if (!DECODE || j < n) {
                        const uint32_t cf = (cwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                        apply_nibble<0>(acc[j], cf & 15u, v);
                        apply_nibble<4>(acc[j], cf >> 4, v);
                    }
                }
            };
            if constexpr (KC > 0) {
                static_for<KC>([&](auto xc) {
                    // keep each block's work in its own region: unscheduled, the compiler
                    // hoists every LDS read of the group and needs ~490 VGPRs
                    // and make the accumulators opaque at every block boundary: with all
                    // coefficients constant, the XOR reassociation otherwise flattens the
                    // 32 blocks' sums into one tree and keeps every block's W/Z live
#pragma unroll
                    for (int j = 0; j < RC; ++j)
#pragma unroll
                        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(acc[j][r]));
                    if constexpr (decltype(xc)::value % 2 == 0) step(xc, lo0, hi0, lo1, hi1);
                    else step(xc, lo1, hi1, lo0, hi0);
                });
            } else {
#pragma unroll 1
                for (int x = 0; x < k; x += 2) {
                    step(x, lo0, hi0, lo1, hi1);
                    if (x + 1 < k) step(x + 1, lo1, hi1, lo0, hi0);
                }
            }
            // ---- outputs: fixed instruction count per output (dropped lanes, no branches)
#pragma unroll
            for (int j = 0; j < RC; ++j) {
                if (j < n) {
                    const int oslot = (DECODE && slots) ? sload_u8(slots, g * rmax + j) : j;
                    uint8_t* dst = out + g * out_gstride + (long long)oslot * BB;
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc(dst, 0, (unsigned)BB, 0x00020000);
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const uint32_t vsum = acc[j][r];
                        const unsigned at = (unsigned)(r * S + 4 * c);
                        const bool tail = lane == NWF && NWF < NW;
                        __builtin_amdgcn_raw_buffer_store_b32(vsum, rs, lane < NWF ? at : kSDrop,
                                                              0, SAUX);
                        if (S & 2)
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)vsum, rs,
                                                                  tail ? at : kSDrop, 0, SAUX);
                        if (S & 1)
                            __builtin_amdgcn_raw_buffer_store_b8(
                                (uint8_t)(vsum >> (8 * (S & 2))), rs,
                                tail ? at + (S & 2) : kSDrop, 0, SAUX);
                    }
                    vm += 8 * SPR;
                }
            }
        }
        gbase += NP;
        gslot0 = (gslot0 + NP) % R;
    }
    stream_wait_vmcnt<0>();
}

bool gf_stream_supported(int k, int m, int bb, int rc, bool decode, const Tune& t) {
    (void)m;
    (void)decode;
    if (!t.stream) return false;
    if (bb != 1352) return false;                        // S = 169 instantiated
    if (rc != 2 && rc != 4 && rc != 8) return false;
    if (((long long)k * bb) % 16 != 0) return false;     // 16-byte aligned group starts
    return true;
}

hipError_t launch_gf_stream(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                            const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                            long long groups, int rc, int rmax, long long coef_gstride,
                            long long out_gstride, bool decode, hipStream_t st,
                            const Tune& t) {
    if (groups <= 0) return hipSuccess;
    if (((uintptr_t)in & 15) != 0 || ((uintptr_t)slots & 3) != 0) return hipErrorInvalidValue;
    const int R = t.stream_ring;
    if (R < 4 || R > 36) return hipErrorInvalidValue;
    const size_t lds = (size_t)kStreamWaves * R * 1024;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int per_cu = (int)((160 * 1024) / lds);
    const long long want = (groups + kStreamWaves - 1) / kStreamWaves;
    long long cap = (long long)t.cus * per_cu;
    if (t.stream_grid > 0) cap = t.stream_grid;          // tests: many groups per wave
    const unsigned grid = (unsigned)std::min<long long>(want, cap);
    const unsigned threads = kStreamWaves * 64;
#define QS_GO(RCV, DEC, RCPV)                                                                \
    hipLaunchKernelGGL((gf_stream_kernel<RCV, 169, DEC, RCPV>), dim3(grid), dim3(threads), lds, \
                       st, in, out, coef, slots, nout, groups, k, m, rmax, coef_gstride,       \
                       out_gstride, R)
    if (bb != 1352) return hipErrorInvalidValue;
    if (decode) {
        note_kernel("gf_stream_kernel<decode>");
        switch (rc) {
            case 2: QS_GO(2, true, 4); break;
            case 4: QS_GO(4, true, 4); break;
            case 8: QS_GO(8, true, 8); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        // one output per register set: RC = m; the table row stride is max(4, rc)
        if ((rc < 4 ? 4 : rc) != (m <= 4 ? 4 : 8)) return hipErrorInvalidValue;
        if (t.const_enc && k == 32 && m == 4) {
            // BASELINE configs B/C: the code is fixed at compile time
            note_kernel("gf_stream_kernel<encode,k32m4>");
            hipLaunchKernelGGL((gf_stream_kernel<4, 169, false, 4, 32>), dim3(grid), dim3(threads),
                               lds, st, in, out, coef, slots, nout, groups, k, m, rmax,
                               coef_gstride, out_gstride, R);
            return hipGetLastError();
        }
        note_kernel("gf_stream_kernel<encode>");
        switch (m) {
            case 2: QS_GO(2, false, 4); break;
            case 3: QS_GO(3, false, 4); break;
            case 4: QS_GO(4, false, 4); break;
            case 5: QS_GO(5, false, 8); break;
            case 6: QS_GO(6, false, 8); break;
            case 7: QS_GO(7, false, 8); break;
            case 8: QS_GO(8, false, 8); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef QS_GO
    return hipGetLastError();
}

}  // namespace qfec
