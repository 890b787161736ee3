// gf_bitslice.h — bit-sliced GF(2^8) helpers shared by the gfx950 FEC kernels.
//
// A block of bb bytes is 8 sub-rows of s = bb/8 bytes; byte column j of the 8 sub-rows
// is one bit-sliced vector (cauchy_256.cpp:90-125).  A lane holds one 4-byte column word
// of each sub-row, W[0..7]; everything below is v_xor / v_bitop3 on those words.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "gf256.h"

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

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // v_bitop3_b32 ... bitop3:0x96
}

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// ------------------------------------------------------------- bit-sliced GF apply
// For one input block, the lane holds its column word of the 8 sub-rows, W[0..7].
// Extend to W[n] = <alpha^n, in> for n = 0..14 (linear in the input):
//   alpha^(n) = alpha^(n-1) + alpha^(n-6) + alpha^(n-7) + alpha^(n-8)   (from 0x187)
// and keep the pair sums Z[n] = W[n] ^ W[n+1].  A coefficient a = sum_b a_b alpha^b then
// contributes  out[r] ^= XOR_{b : a_b} W[b + r]   (r = 0..7), i.e. per nibble p of a at
// bit offset B a fixed XOR of at most two W/Z terms per output sub-row.
struct WZ {
    union {
        uint32_t W[15];
        uint32_t W8[8];   // the block's own 8 sub-row words (W[0..7])
    };
    uint32_t Z[14];
};

__device__ __forceinline__ void expand_wz(WZ& v) {
#pragma unroll
    for (int i = 0; i < 7; ++i) v.Z[i] = v.W[i] ^ v.W[i + 1];
#pragma unroll
    for (int n = 8; n < 15; ++n) v.W[n] = xor3(v.W[n - 1], v.W[n - 6], v.Z[n - 8]);
#pragma unroll
    for (int i = 7; i < 14; ++i) v.Z[i] = v.W[i] ^ v.W[i + 1];
}

template <int B>
__device__ __forceinline__ void apply_nibble(uint32_t (&acc)[8], uint32_t p, const WZ& v) {
#define QF_CASE(P, EXPR)                                   \
    case P:                                                \
        _Pragma("unroll") for (int r = 0; r < 8; ++r) { acc[r] = EXPR; } \
        break;
    switch (p) {
        QF_CASE(1, acc[r] ^ v.W[B + r])
        QF_CASE(2, acc[r] ^ v.W[B + 1 + r])
        QF_CASE(3, acc[r] ^ v.Z[B + r])
        QF_CASE(4, acc[r] ^ v.W[B + 2 + r])
        QF_CASE(5, xor3(acc[r], v.W[B + r], v.W[B + 2 + r]))
        QF_CASE(6, acc[r] ^ v.Z[B + 1 + r])
        QF_CASE(7, xor3(acc[r], v.Z[B + r], v.W[B + 2 + r]))
        QF_CASE(8, acc[r] ^ v.W[B + 3 + r])
        QF_CASE(9, xor3(acc[r], v.W[B + r], v.W[B + 3 + r]))
        QF_CASE(10, xor3(acc[r], v.W[B + 1 + r], v.W[B + 3 + r]))
        QF_CASE(11, xor3(acc[r], v.Z[B + r], v.W[B + 3 + r]))
        QF_CASE(12, acc[r] ^ v.Z[B + 2 + r])
        QF_CASE(13, xor3(acc[r], v.W[B + r], v.Z[B + 2 + r]))
        QF_CASE(14, xor3(acc[r], v.Z[B + 1 + r], v.W[B + 3 + r]))
        QF_CASE(15, xor3(acc[r], v.Z[B + r], v.Z[B + 2 + r]))
        default: break;
    }
#undef QF_CASE
}

// ------------------------------------------------ windowed form, compile-time coefficients
// The reference's windowed encoder (cauchy_256.cpp:1419-1500, win_encode) splits a block's
// 8 sub-rows into two groups of 4 and precomputes every XOR combination of each group; an
// output sub-row r of coefficient c then needs the combination selected by the low nibble
// of c * alpha^r plus the one selected by its high nibble.  With the coefficient known at
// compile time that is ONE v_bitop3 per (output, sub-row) (acc ^ lo[M & 15] ^ hi[M >> 4]),
// against two in the W/Z nibble form above; the compiler drops every combination no output
// of the block uses.  Bit-exact with the W/Z form: both compute XOR_{t in bits(c alpha^r)}.
struct Win {
    uint32_t lo[16];   // lo[i] = XOR of in[t] for the set bits t of i      (t = 0..3)
    uint32_t hi[16];   // hi[i] = XOR of in[4 + t] for the set bits t of i  (t = 0..3)
};

__device__ __forceinline__ void win_group(const uint32_t* in, uint32_t (&o)[16]) {
    o[0] = 0;
    o[1] = in[0];
    o[2] = in[1];
    o[3] = in[0] ^ in[1];
    o[4] = in[2];
    o[5] = in[0] ^ in[2];
    o[6] = in[1] ^ in[2];
    o[7] = xor3(in[0], in[1], in[2]);
    o[8] = in[3];
    o[9] = in[0] ^ in[3];
    o[10] = in[1] ^ in[3];
    o[11] = xor3(in[0], in[1], in[3]);
    o[12] = in[2] ^ in[3];
    o[13] = xor3(in[0], in[2], in[3]);
    o[14] = xor3(in[1], in[2], in[3]);
    o[15] = o[3] ^ o[12];
}

__device__ __forceinline__ void win_build(const uint32_t (&in)[8], Win& w) {
    win_group(in, w.lo);
    win_group(in + 4, w.hi);
}

constexpr uint8_t gf_alpha_pow(int r) {
    uint8_t v = 1;
    for (int i = 0; i < r; ++i) v = gf_xtime(v);
    return v;
}

// o[r] = (c * alpha^r) applied to the block, r = 0..7, for a compile-time coefficient C
// (the product itself, no accumulator: one v_bitop3 or v_xor per sub-row, or a copy)
template <unsigned C>
__device__ __forceinline__ void win_set(uint32_t (&o)[8], const Win& w) {
    static_for<8>([&](auto rc) __attribute__((always_inline)) {
        constexpr int r = decltype(rc)::value;
        constexpr unsigned M = gf_mul((uint8_t)C, gf_alpha_pow(r));
        constexpr unsigned a = M & 15u, b = M >> 4;
        if constexpr (a && b) o[r] = w.lo[a] ^ w.hi[b];
        else if constexpr (a) o[r] = w.lo[a];
        else if constexpr (b) o[r] = w.hi[b];
        else o[r] = 0;
    });
}

// acc[r] ^= (c * alpha^r) applied to the block, r = 0..7, for a compile-time coefficient C
template <unsigned C>
__device__ __forceinline__ void win_apply(uint32_t (&acc)[8], const Win& w) {
    static_for<8>([&](auto rc) __attribute__((always_inline)) {
        constexpr int r = decltype(rc)::value;
        constexpr unsigned M = gf_mul((uint8_t)C, gf_alpha_pow(r));
        constexpr unsigned a = M & 15u, b = M >> 4;
        if constexpr (a && b) acc[r] = xor3(acc[r], w.lo[a], w.hi[b]);
        else if constexpr (a) acc[r] ^= w.lo[a];
        else if constexpr (b) acc[r] ^= w.hi[b];
    });
}

}  // namespace qfec
