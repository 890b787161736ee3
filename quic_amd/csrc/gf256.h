// gf256.h — GF(2^8) arithmetic of the QuicR FEC codec (host + device, constexpr).
//
// Field: polynomial x^8 + x^7 + x^2 + x + 1 (0x187), generator alpha = 2, exactly as the
// reference codec (net/quic/core/libcat/cauchy_256.cpp:272).  The reference ships literal
// LOG/EXP/INV tables (:274-343); here they are generated at compile time from the
// polynomial.  NOTE: libcat's unrelated Galois256.hpp uses 0x15F — never mix them.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define QFEC_HD __host__ __device__
#else
#define QFEC_HD
#endif

namespace qfec {

constexpr unsigned kGfPoly = 0x187;

QFEC_HD constexpr uint8_t gf_xtime(uint8_t v) {
    return (uint8_t)((v & 0x80) ? ((v << 1) ^ kGfPoly) : (v << 1));
}

struct GfTables {
    uint8_t exp[512];   // exp[i] = alpha^(i mod 255), doubled so exp[log a + log b] needs no mod
    uint8_t log[256];   // log[0] unused (0)
    uint8_t inv[256];   // inv[0] = 0
};

constexpr GfTables make_gf_tables() {
    GfTables t{};
    uint8_t v = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = v;
        t.log[v] = (uint8_t)i;
        v = gf_xtime(v);
    }
    for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
    t.inv[0] = 0;
    for (int a = 1; a < 256; ++a) t.inv[a] = t.exp[255 - t.log[a]];
    return t;
}

inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    return (a && b) ? kGf.exp[kGf.log[a] + kGf.log[b]] : 0;
}
constexpr uint8_t gf_div(uint8_t a, uint8_t b) {  // a / b; the reference's b = 0 row is zeros
    return (a && b) ? kGf.exp[kGf.log[a] + 255 - kGf.log[b]] : 0;
}
constexpr uint8_t gf_inv(uint8_t a) { return kGf.inv[a]; }

// alpha^n for n = 0..14: the 8x8 "transposed" expansion of a coefficient c maps input
// sub-row t into output sub-row r when bit t of c * alpha^r is set (cauchy_256.cpp:90-125).
static_assert(gf_mul(2, 0x80) == 0x87, "alpha^8 must be 0x87 for poly 0x187");

}  // namespace qfec
