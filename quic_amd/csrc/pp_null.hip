// pp_null.hip — packet protection next to the FEC path (SURVEY.md §8 f, rank 4): the
// reference's NullEncrypter / NullDecrypter over batches of packets on the device.
//
// The fork's QuicEncrypter::Create maps kNULL to NullEncrypter and every negotiated AEAD
// (kAESG, kCC20) to MyEncrypter, an identity copy (crypto/quic_encrypter.cc:18-29,
// crypto/none_encrypter.cc EncryptPacket).  NullEncrypter is therefore the only packet
// protection of this reference with arithmetic in it:
//   seal (null_encrypter.cc:23-43):  wire = AD || tag12 || PT,  tag12 = the low 12 bytes
//        (little-endian, quic_utils.cc:175-181) of FNV-1a-128(AD || PT);
//   open (null_decrypter.cc DecryptPacket / ReadHash / ComputeHash): reject short input or
//        a tag that differs from FNV-1a-128(AD || CT[12..]) with its top 32 bits cleared;
//        the output holds a copy of the ciphertext before the check and the plaintext after.
//   FNV-1a-128 (quic_utils.cc:38-56,110-125): h = (h ^ byte) * (2^88 + 315) mod 2^128.
//
// The hash is a serial chain over the bytes of one packet, so one lane owns one packet:
// h * (2^88 + 315) = h * 315 + (h << 88), i.e. lo' = lo * 315 and
// hi' = hi * 315 + mulhi(lo, 315) + (lo << 24) (a handful of VALU ops per byte).  Lanes read
// their packets as 16-byte loads, 256 bytes in flight per lane.  The packet bytes are written by the
// whole wave, packet by packet, as coalesced dwords (the 64 tags are handed over in LDS).
// Bound: the dependent per-byte chain (VALU latency), not HBM; DESIGN.md §6.2.
#include "fec_kernels.h"

namespace qfec {

namespace {

constexpr int kPPWaves = 4;   // waves per workgroup (64 packets per wave)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void fnv_byte(uint64_t& lo, uint64_t& hi, uint32_t b) {
    lo ^= b;
    const uint64_t nhi = hi * 315u + __umul64hi(lo, 315u) + (lo << 24);
    lo *= 315u;
    hi = nhi;
}

__device__ __forceinline__ void fnv_word(uint64_t& lo, uint64_t& hi, uint32_t w) {
    fnv_byte(lo, hi, w & 0xFFu);
    fnv_byte(lo, hi, (w >> 8) & 0xFFu);
    fnv_byte(lo, hi, (w >> 16) & 0xFFu);
    fnv_byte(lo, hi, w >> 24);
}

// FNV-1a-128 over p[0 .. len): bytes up to 16-byte alignment, then 256-byte chunks as 16
// dwordx4 loads issued together (one lane streams its own packet: the loads of a chunk are
// in flight at once, so a packet costs a few memory round trips, not one per dword), aligned
// dwords, tail bytes
__device__ void fnv_span(uint64_t& lo, uint64_t& hi, const uint8_t* p, int len) {
    if (len <= 0) return;
    const int head = min(len, (int)((16u - ((uintptr_t)p & 15u)) & 15u));
    for (int i = 0; i < head; ++i) fnv_byte(lo, hi, p[i]);
    const u32x4* q4 = (const u32x4*)(p + head);
    const int rest = len - head;
    const int nc = rest >> 8;   // 256-byte chunks
    for (int j = 0; j < nc; ++j) {
        u32x4 w[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = __builtin_nontemporal_load(q4 + 16 * j + u);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            fnv_word(lo, hi, w[u].x);
            fnv_word(lo, hi, w[u].y);
            fnv_word(lo, hi, w[u].z);
            fnv_word(lo, hi, w[u].w);
        }
    }
    // the last < 256 bytes: up to 15 dwordx4 loads, again issued together
    const u32x4* r4 = q4 + 16 * nc;
    const int nr = (rest & 255) >> 4;
    {
        u32x4 w[15];
#pragma unroll
        for (int u = 0; u < 15; ++u)
            if (u < nr) w[u] = __builtin_nontemporal_load(r4 + u);
#pragma unroll
        for (int u = 0; u < 15; ++u)
            if (u < nr) {
                fnv_word(lo, hi, w[u].x);
                fnv_word(lo, hi, w[u].y);
                fnv_word(lo, hi, w[u].z);
                fnv_word(lo, hi, w[u].w);
            }
    }
    const uint8_t* t = (const uint8_t*)(r4 + nr);
    for (int i = 0; i < (rest & 15); ++i) fnv_byte(lo, hi, t[i]);
}

__device__ __forceinline__ void fnv_init(uint64_t& lo, uint64_t& hi) {
    // kOffset = 144066263297769815596495629667062367629 (quic_utils.cc:116-118)
    hi = 7809847782465536322ull;
    lo = 7113472399480571277ull;
}

__device__ __forceinline__ int len_of(const int32_t* a, int all, long long i) {
    return a ? a[i] : all;
}

// Packet bytes written by the whole wave: out dword u of packet j = bytes 4u .. 4u + 3 of
// the concatenation seg0 (n0 bytes at p0) || seg1 (nt bytes at tag: LDS or global) ||
// seg2 (the rest, at p1)
__device__ void wave_write(uint8_t* out, int total, const uint8_t* p0, int n0,
                           const uint8_t* tag, int nt, const uint8_t* p1, int lane) {
    const int nfull = total >> 2;
    auto byte_at = [&](int o) -> uint32_t {
        if (o < n0) return p0[o];
        if (o < n0 + nt) return tag[o - n0];
        return p1[o - n0 - nt];
    };
#pragma unroll 4
    for (int u = lane; u < nfull; u += 64) {
        const int o = 4 * u;
        const uint32_t v = byte_at(o) | (byte_at(o + 1) << 8) | (byte_at(o + 2) << 16) |
                           (byte_at(o + 3) << 24);
        ((uint32_t*)out)[u] = v;
    }
    if (lane < (total & 3)) out[4 * nfull + lane] = (uint8_t)byte_at(4 * nfull + lane);
}

__global__ __launch_bounds__(kPPWaves * 64) void null_seal_kernel(
    long long n, const uint8_t* __restrict__ ad, long long ad_stride,
    const int32_t* __restrict__ ad_len, int ad_all, const uint8_t* __restrict__ pt,
    long long pt_stride, const int32_t* __restrict__ pt_len, int pt_all, uint8_t* out,
    long long out_stride, int32_t* out_len) {
    __shared__ uint32_t tags[kPPWaves][64][3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long base = ((long long)blockIdx.x * kPPWaves + w) * 64;
    if (base >= n) return;   // uniform over the wave; no workgroup barrier below
    const long long i = base + lane;
    const bool mine = i < n;
    int al = 0, pl = 0;
    bool ok = false;
    if (mine) {
        al = len_of(ad_len, ad_all, i);
        pl = len_of(pt_len, pt_all, i);
        // a row longer than its stride would read the next packet's bytes (or past the
        // buffer for the last one): rejected like a packet that does not fit
        ok = al >= 0 && pl >= 0 && (ad_stride == 0 || al <= ad_stride) &&
             (pt_stride == 0 || pl <= pt_stride) && (long long)al + 12 + pl <= out_stride;
        uint64_t lo, hi;
        fnv_init(lo, hi);
        if (ok) {
            fnv_span(lo, hi, ad + i * ad_stride, al);
            fnv_span(lo, hi, pt + i * pt_stride, pl);
        }
        tags[w][lane][0] = (uint32_t)lo;
        tags[w][lane][1] = (uint32_t)(lo >> 32);
        tags[w][lane][2] = (uint32_t)hi;   // SerializeUint128Short: low 4 bytes of the high half
        out_len[i] = ok ? al + 12 + pl : -1;
    }
    // a wave's LDS operations complete in order: the tags are visible to the wave's lanes
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const int cnt = (int)min(64ll, n - base);
    for (int j = 0; j < cnt; ++j) {
        const int jal = __shfl(al, j), jpl = __shfl(pl, j);
        if (!__shfl((int)ok, j)) continue;
        const long long pj = base + j;
        wave_write(out + pj * out_stride, jal + 12 + jpl, ad + pj * ad_stride, jal,
                   (const uint8_t*)tags[w][j], 12, pt + pj * pt_stride, lane);
    }
}

__global__ __launch_bounds__(kPPWaves * 64) void null_open_kernel(
    long long n, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ pkt_len, int pkt_all, const int32_t* __restrict__ ad_len,
    int ad_all, uint8_t* out, long long out_stride, int32_t* out_len) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long base = ((long long)blockIdx.x * kPPWaves + w) * 64;
    if (base >= n) return;
    const long long i = base + lane;
    const bool mine = i < n;
    int al = 0, cl = 0, res = -1;
    bool copy = false;   // the output receives the ciphertext (reference: before any check)
    if (mine) {
        const uint8_t* p = pkt + i * pkt_stride;
        al = len_of(ad_len, ad_all, i);
        const int tl = len_of(pkt_len, pkt_all, i);
        cl = tl - al;   // ciphertext bytes
        copy = al >= 0 && cl >= 0 && cl <= out_stride && (pkt_stride == 0 || tl <= pkt_stride);
        if (copy && cl >= 12) {
            const uint8_t* c = p + al;
            uint32_t t[3];
#pragma unroll
            for (int q = 0; q < 3; ++q)
                t[q] = c[4 * q] | (c[4 * q + 1] << 8) | (c[4 * q + 2] << 16) |
                       ((uint32_t)c[4 * q + 3] << 24);
            uint64_t lo, hi;
            fnv_init(lo, hi);
            fnv_span(lo, hi, p, al);
            fnv_span(lo, hi, c + 12, cl - 12);
            const bool match = (uint32_t)lo == t[0] && (uint32_t)(lo >> 32) == t[1] &&
                               (uint32_t)hi == t[2];
            res = match ? cl - 12 : -1;
        }
        out_len[i] = res;
    }
    const int cnt = (int)min(64ll, n - base);
    for (int j = 0; j < cnt; ++j) {
        if (!__shfl((int)copy, j)) continue;
        const int jal = __shfl(al, j), jcl = __shfl(cl, j), jres = __shfl(res, j);
        const long long pj = base + j;
        const uint8_t* c = pkt + pj * pkt_stride + jal;
        // accepted: the plaintext, then the last 12 bytes of the ciphertext copy the
        // reference made first (its output buffer holds them past the plaintext); rejected:
        // that copy alone
        if (jres >= 0)
            wave_write(out + pj * out_stride, jcl, c + 12, jres, c + jres, 12, nullptr, lane);
        else
            wave_write(out + pj * out_stride, jcl, c, jcl, nullptr, 0, nullptr, lane);
    }
}

unsigned pp_grid(long long n) {
    return (unsigned)((n + kPPWaves * 64 - 1) / (kPPWaves * 64));
}

}  // namespace

hipError_t launch_null_seal(long long n, const uint8_t* ad, long long ad_stride,
                            const int32_t* ad_len, int ad_all, const uint8_t* pt,
                            long long pt_stride, const int32_t* pt_len, int pt_all, uint8_t* out,
                            long long out_stride, int32_t* out_len, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if ((((uintptr_t)out) | (uintptr_t)out_stride) & 3) return hipErrorInvalidValue;
    if (pp_grid(n) > 0x7fffffffu) return hipErrorInvalidValue;
    note_kernel("null_seal_kernel");
    qlaunch(null_seal_kernel, dim3(pp_grid(n)), dim3(kPPWaves * 64), 0, st, n, ad,
                       ad_stride, ad_len, ad_all, pt, pt_stride, pt_len, pt_all, out, out_stride,
                       out_len);
    return hipGetLastError();
}

hipError_t launch_null_open(long long n, const uint8_t* pkt, long long pkt_stride,
                            const int32_t* pkt_len, int pkt_all, const int32_t* ad_len,
                            int ad_all, uint8_t* out, long long out_stride, int32_t* out_len,
                            hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if ((((uintptr_t)out) | (uintptr_t)out_stride) & 3) return hipErrorInvalidValue;
    if (pp_grid(n) > 0x7fffffffu) return hipErrorInvalidValue;
    note_kernel("null_open_kernel");
    qlaunch(null_open_kernel, dim3(pp_grid(n)), dim3(kPPWaves * 64), 0, st, n, pkt,
                       pkt_stride, pkt_len, pkt_all, ad_len, ad_all, out, out_stride, out_len);
    return hipGetLastError();
}

}  // namespace qfec
