// gf_winjump.h — run-time GF(2^8) coefficient times a windowed block by one indirect jump.
//
// (Not used by the product kernels: the microbenchmark's "jump" mode, measured slower than
// the nibble jumps below with the scatter a caller needs; kept with its CPU table test.)
// win_mul_rt(t, w, c): t[r] = (c * alpha^r) applied to the block whose window is w
// (gf_bitslice.h Win), r = 0..7 — the same bytes as win_set<c>(t, w), for a wave-uniform c
// known only at run time.  The table of 256 straight-line leaves (build/gen/win_jump.h,
// tools/gen_win_jump.py) lies inline after the dispatch: leaf c starts QF_WIN_LEAF_BYTES * c
// bytes past it, is 8 four-byte VOP1/VOP2 instructions and an s_branch past the table.  The
// dispatch is s_getpc_b64, s_mul_i32, s_add_u32, s_add_u32, s_addc_u32, s_setpc_b64: against
// the 256-way tree of uniform branches (8 levels of s_cmp + s_cbranch, ~16 scalar
// instructions and 4 taken branches per product), six scalar instructions and two jumps.
//
// Every call site emits its own 9 KB table (code size), so the callers keep one call site
// per kernel (a loop with `#pragma unroll 1` around it) and scatter the product from t.
// The leaves only read the window and write t; the scratch SGPR pair s[88:89] and s90 are
// declared clobbered.
#pragma once
#include "gf_bitslice.h"
#include "win_jump.h"

namespace qfec {

__device__ __forceinline__ void win_mul_rt(uint32_t (&t)[8], const Win& w, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile(
        "s_getpc_b64 s[88:89]\n\t"
        "1:\n\t"
        "s_mul_i32 s90, %[c], " QF_WIN_LEAF_BYTES_S "\n\t"
        "s_add_u32 s90, s90, 2f-1b\n\t"
        "s_add_u32 s88, s88, s90\n\t"
        "s_addc_u32 s89, s89, 0\n\t"
        "s_setpc_b64 s[88:89]\n\t"
        "2:\n\t" QF_WIN_JUMP_LEAVES
        : [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3]),
          [t4] "=&v"(t[4]), [t5] "=&v"(t[5]), [t6] "=&v"(t[6]), [t7] "=&v"(t[7])
        : [c] "s"(c), [l1] "v"(w.lo[1]), [l2] "v"(w.lo[2]), [l3] "v"(w.lo[3]),
          [l4] "v"(w.lo[4]), [l5] "v"(w.lo[5]), [l6] "v"(w.lo[6]), [l7] "v"(w.lo[7]),
          [l8] "v"(w.lo[8]), [l9] "v"(w.lo[9]), [l10] "v"(w.lo[10]), [l11] "v"(w.lo[11]),
          [l12] "v"(w.lo[12]), [l13] "v"(w.lo[13]), [l14] "v"(w.lo[14]), [l15] "v"(w.lo[15]),
          [h1] "v"(w.hi[1]), [h2] "v"(w.hi[2]), [h3] "v"(w.hi[3]), [h4] "v"(w.hi[4]),
          [h5] "v"(w.hi[5]), [h6] "v"(w.hi[6]), [h7] "v"(w.hi[7]), [h8] "v"(w.hi[8]),
          [h9] "v"(w.hi[9]), [h10] "v"(w.hi[10]), [h11] "v"(w.hi[11]), [h12] "v"(w.hi[12]),
          [h13] "v"(w.hi[13]), [h14] "v"(w.hi[14]), [h15] "v"(w.hi[15])
        : "s88", "s89", "s90", "scc");
#else
    (void)w, (void)c;
    for (int r = 0; r < 8; ++r) t[r] = 0;
#endif
}

}  // namespace qfec

namespace qfec {

// wz_mul_acc_rt(acc, v, c): acc[r] ^= (c * alpha^r) applied to the block whose W/Z expansion
// is v (gf_bitslice.h expand_wz), r = 0..7 — apply_nibble<0>(acc, c & 15, v) then
// apply_nibble<4>(acc, c >> 4, v) with each nibble's 16-way uniform branch tree replaced by
// an indirect jump into a table of 16 leaves (QF_NIB_LEAVES_LO / _HI: 8 eight-byte VALU and
// an s_branch each).  Its tables are 2.2 KB per call site, so the target accumulator can be
// a compile-time choice (one call site per target).
__device__ __forceinline__ void wz_mul_acc_rt(uint32_t (&acc)[8], const WZ& v, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile(
        "s_getpc_b64 s[88:89]\n\t"
        "1:\n\t"
        "s_and_b32 s90, %[c], 15\n\t"
        "s_mul_i32 s90, s90, " QF_NIB_LEAF_BYTES_S "\n\t"
        "s_add_u32 s90, s90, 2f-1b\n\t"
        "s_add_u32 s88, s88, s90\n\t"
        "s_addc_u32 s89, s89, 0\n\t"
        "s_setpc_b64 s[88:89]\n\t"
        "2:\n\t" QF_NIB_LEAVES_LO
        "5:\n\t"
        "s_getpc_b64 s[88:89]\n\t"
        "4:\n\t"
        "s_bfe_u32 s90, %[c], 0x40004\n\t"
        "s_mul_i32 s90, s90, " QF_NIB_LEAF_BYTES_S "\n\t"
        "s_add_u32 s90, s90, 6f-4b\n\t"
        "s_add_u32 s88, s88, s90\n\t"
        "s_addc_u32 s89, s89, 0\n\t"
        "s_setpc_b64 s[88:89]\n\t"
        "6:\n\t" QF_NIB_LEAVES_HI
        "7:\n\t"
        : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]),
          [a4] "+v"(acc[4]), [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7])
        : [c] "s"(c), [w0] "v"(v.W[0]), [w1] "v"(v.W[1]), [w2] "v"(v.W[2]), [w3] "v"(v.W[3]),
          [w4] "v"(v.W[4]), [w5] "v"(v.W[5]), [w6] "v"(v.W[6]), [w7] "v"(v.W[7]),
          [w8] "v"(v.W[8]), [w9] "v"(v.W[9]), [w10] "v"(v.W[10]), [w11] "v"(v.W[11]),
          [w12] "v"(v.W[12]), [w13] "v"(v.W[13]), [w14] "v"(v.W[14]), [z0] "v"(v.Z[0]),
          [z1] "v"(v.Z[1]), [z2] "v"(v.Z[2]), [z3] "v"(v.Z[3]), [z4] "v"(v.Z[4]),
          [z5] "v"(v.Z[5]), [z6] "v"(v.Z[6]), [z7] "v"(v.Z[7]), [z8] "v"(v.Z[8]),
          [z9] "v"(v.Z[9]), [z10] "v"(v.Z[10]), [z11] "v"(v.Z[11]), [z12] "v"(v.Z[12]),
          [z13] "v"(v.Z[13])
        : "s88", "s89", "s90", "scc");
#else
    (void)acc, (void)v, (void)c;
#endif
}

}  // namespace qfec

namespace qfec {

// a 64-bit value as the two-dword vector the 8-byte buffer store takes (low dword first)
typedef unsigned qf_u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ qf_u32x2_t qf_u32x2(uint64_t v) {
    qf_u32x2_t r = {(unsigned)v, (unsigned)(v >> 32)};
    return r;
}

// stage_block_169(lds, w, lane): writes one 1352-byte block (8 sub-rows of 169 B) that the wave
// holds bit-sliced (lane c < 43: column word c of each sub-row, bytes 169 t + 4 c ..) to LDS at
// byte address `lds` (8-byte aligned) as its contiguous bytes, with ALIGNED ds_write_b32 only
// (an unaligned one is replayed slowly and measured wrong).  Sub-row t starts a = (t * 169) & 3
// bytes into a dword: lane c writes the dword at 169 t - a + 4 c, built from its own word and
// lane c - 1's (ds_bpermute); lane 0 takes the bytes before the
// sub-row (the previous sub-row's last four, read from its lane 42 into an SGPR).  Sub-rows are
// written in order, so where lane 42's dword runs into the next sub-row, that sub-row's lane 0
// overwrites it with the merged bytes.  Lanes >= 43 must be inactive (exec).  Inline asm with
// its own lgkmcnt waits (as C++ LDS accesses the compiler would first wait for every LDS-DMA in
// flight).
__device__ __forceinline__ void stage_block_169(uint32_t lds, const uint32_t (&w)[8], int lane) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int S = 169;
    const uint32_t qa = lds + 4u * (uint32_t)lane;
    const uint32_t pa = 4u * (uint32_t)(lane - 1);   // lane 0's is replaced below
    uint32_t p[8];   // lane c - 1's word of each sub-row
    asm volatile(
        "ds_bpermute_b32 %0, %8, %9\n\t"
        "ds_bpermute_b32 %1, %8, %10\n\t"
        "ds_bpermute_b32 %2, %8, %11\n\t"
        "ds_bpermute_b32 %3, %8, %12\n\t"
        "ds_bpermute_b32 %4, %8, %13\n\t"
        "ds_bpermute_b32 %5, %8, %14\n\t"
        "ds_bpermute_b32 %6, %8, %15\n\t"
        "ds_bpermute_b32 %7, %8, %16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(p[0]), "=&v"(p[1]), "=&v"(p[2]), "=&v"(p[3]), "=&v"(p[4]), "=&v"(p[5]),
          "=&v"(p[6]), "=&v"(p[7])
        : "v"(pa), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]),
          "v"(w[7]));
    uint32_t X = 0;   // previous sub-row's bytes 165..168 (wave-uniform)
    const bool l0 = lane == 0;
#define QF_STAGE_T(T)                                                                         \
    {                                                                                         \
        constexpr int a = ((T) * S) & 3;                                                      \
        const uint32_t prev = l0 ? X : p[T];                                                  \
        const uint32_t v = a ? __builtin_amdgcn_alignbyte(w[T], prev, (4 - a) & 3) : w[T];    \
        asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(qa), "v"(v), "n"((T) * S - a)      \
                     : "memory");                                                             \
        if ((T) < 7)                                                                          \
            X = (uint32_t)__builtin_amdgcn_readlane(                                          \
                (int)__builtin_amdgcn_alignbyte(w[T], p[T], 1), 42);                          \
    }
    QF_STAGE_T(0) QF_STAGE_T(1) QF_STAGE_T(2) QF_STAGE_T(3)
    QF_STAGE_T(4) QF_STAGE_T(5) QF_STAGE_T(6) QF_STAGE_T(7)
#undef QF_STAGE_T
#else
    (void)lds, (void)w, (void)lane;
#endif
}

}  // namespace qfec
