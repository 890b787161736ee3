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
// The hash is a serial chain over the bytes of one packet, so one lane owns one packet and
// does everything for it: it streams the packet's bytes once (16-byte loads, two 64-byte
// chunks in flight), hashes them and writes them to the output as they pass (a per-lane
// dword writer that realigns with one 64-bit shift), then writes the tag.
//
// The chain: h is kept as six 22-bit limbs in carry-save form.  h * 315 is six full-rate
// 24-bit multiplies (v_mul_u32_u24; a limb stays below 2^24, its product below 2^32), each
// limb keeps its low 22 bits and passes the rest up one limb, and h << 88 is two limb adds
// (88 = 4 * 22): about 25 full-rate VALU operations per byte, with six independent lanes of
// work, against seven quarter-rate 32-bit multiplies for the plain 64-bit-halves form.  The
// low limb is always exact (nothing carries into it), so the byte XOR is exact too; the
// limbs are normalised once, for the tag.  Bound: the VALU.
//
// Grouped forms (the FEC group's view of its packets): every data and FEC packet of G groups
// sealed in one launch, and the receiver's open that writes each data packet's plaintext
// straight into its block slot, followed by one wave per group that fills the holes with the
// opened FEC packets and writes the row tags the decode reads.
#include "fec_kernels.h"
#include "pp_null.h"

namespace qfec {

namespace {

constexpr int kPPThreads = 256;   // one packet per lane
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// FNV-1a-128, six 22-bit limbs (limb j = bits 22j ..), carry-save: limbs 1..5 may exceed
// 22 bits by the carry they received (< 2^24 always).
struct Fnv {
    uint32_t l0, l1, l2, l3, l4, l5;
    // kOffset = 144066263297769815596495629667062367629 (quic_utils.cc:116-118)
    __device__ __forceinline__ void init() {
        l0 = 0x15c58du;
        l1 = 0x05d58au;
        l2 = 0x262b82u;
        l3 = 0x2ec050u;
        l4 = 0x272e07u;
        l5 = 0x01b188u;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        constexpr uint32_t M = (1u << 22) - 1u;
        const uint32_t x0 = l0 ^ b;   // l0 < 2^22 is exact: the XOR is the reference's
        const uint32_t p0 = __umul24(x0, 315u), p1 = __umul24(l1, 315u);
        const uint32_t p2 = __umul24(l2, 315u), p3 = __umul24(l3, 315u);
        const uint32_t p4 = __umul24(l4, 315u), p5 = __umul24(l5, 315u);
        const uint32_t n4 = (p4 & M) + (p3 >> 22) + x0;   // + (h << 88), limbs 0, 1 -> 4, 5
        const uint32_t n5 = (p5 & M) + (p4 >> 22) + l1;   // bits >= 128 fall off the top
        l1 = (p1 & M) + (p0 >> 22);
        l2 = (p2 & M) + (p1 >> 22);
        l3 = (p3 & M) + (p2 >> 22);
        l0 = p0 & M;
        l4 = n4;
        l5 = n5;
    }
    __device__ __forceinline__ void word(uint32_t w) {
        byte(w & 0xFFu);
        byte((w >> 8) & 0xFFu);
        byte((w >> 16) & 0xFFu);
        byte(w >> 24);
    }
    // the low 96 bits of h, little-endian dwords (SerializeUint128Short, quic_utils.cc:175-181)
    __device__ __forceinline__ void tag(uint32_t& t0, uint32_t& t1, uint32_t& t2) const {
        constexpr uint32_t M = (1u << 22) - 1u;
        uint32_t c = 0, n[6];
        const uint32_t l[6] = {l0, l1, l2, l3, l4, l5};
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const uint32_t v = l[j] + c;
            n[j] = v & M;
            c = v >> 22;
        }
        const uint64_t lo = (uint64_t)n[0] | ((uint64_t)n[1] << 22) | ((uint64_t)n[2] << 44);
        const uint64_t hi = ((uint64_t)n[2] >> 20) | ((uint64_t)n[3] << 2) |
                            ((uint64_t)n[4] << 24) | ((uint64_t)n[5] << 46);
        t0 = (uint32_t)lo;
        t1 = (uint32_t)(lo >> 32);
        t2 = (uint32_t)hi;
    }
};

// The plain form (pp_hash = 1): 64-bit halves, h * (2^88 + 315) = h * 315 + (h << 88), i.e.
// lo' = lo * 315, hi' = hi * 315 + mulhi(lo, 315) + (lo << 24) (64-bit multiply-adds).
struct Fnv64 {
    uint64_t lo, hi;
    __device__ __forceinline__ void init() {
        hi = 7809847782465536322ull;
        lo = 7113472399480571277ull;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        lo ^= b;
        const uint64_t nhi = hi * 315u + __umul64hi(lo, 315u) + (lo << 24);
        lo *= 315u;
        hi = nhi;
    }
    __device__ __forceinline__ void word(uint32_t w) {
        byte(w & 0xFFu);
        byte((w >> 8) & 0xFFu);
        byte((w >> 16) & 0xFFu);
        byte(w >> 24);
    }
    __device__ __forceinline__ void tag(uint32_t& t0, uint32_t& t1, uint32_t& t2) const {
        t0 = (uint32_t)lo;
        t1 = (uint32_t)(lo >> 32);
        t2 = (uint32_t)hi;
    }
};

// Per-lane byte-stream writer: bytes go out as aligned dword stores; `carry` holds the bytes
// of the current dword not yet stored.  Bytes before `start` are not the writer's: a dword
// that holds some of them is written byte by byte.
struct Sink {
    uint8_t* ptr;
    uint8_t* start;
    uint32_t carry;
    __device__ __forceinline__ void begin(uint8_t* p) {
        ptr = start = p;
        carry = 0;
    }
    __device__ __forceinline__ void store_dw(uint8_t* a, uint32_t v) {   // a 4-byte aligned
        if (a >= start) {
            *(uint32_t*)a = v;
        } else {
            for (int q = (int)(start - a); q < 4; ++q) a[q] = (uint8_t)(v >> (8 * q));
        }
    }
    __device__ __forceinline__ void word(uint32_t w) {
        const uint32_t pb = (uint32_t)(uintptr_t)ptr & 3u;
        const uint64_t v = ((uint64_t)w << (8 * pb)) | carry;
        store_dw(ptr - pb, (uint32_t)v);
        carry = (uint32_t)(v >> 32);
        ptr += 4;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        const uint32_t pb = (uint32_t)(uintptr_t)ptr & 3u;
        carry |= b << (8 * pb);
        ++ptr;
        if (pb == 3) {
            store_dw(ptr - 4, carry);
            carry = 0;
        }
    }
    __device__ __forceinline__ void flush() {
        const uint32_t pb = (uint32_t)(uintptr_t)ptr & 3u;
        uint8_t* a = ptr - pb;
        for (uint32_t q = 0; q < pb; ++q)
            if (a + q >= start) a[q] = (uint8_t)(carry >> (8 * q));
    }
    // zero bytes up to `end`, then flush
    __device__ __forceinline__ void zeros_to(const uint8_t* end) {
        while (ptr < end && ((uintptr_t)ptr & 3u)) byte(0);
        while (ptr + 4 <= end) word(0);
        while (ptr < end) byte(0);
        flush();
    }
};

// One lane streams p[0 .. len): bytes up to 16-byte alignment, then 64-byte chunks of four
// 16-byte loads with the next chunk in flight while this one is consumed, then the last
// < 64 bytes.  HASH: into h; WRITE: through s.
constexpr int CH = 4;
template <bool HASH, bool WRITE, class H>
__device__ __forceinline__ void span(H& h, Sink& s, const uint8_t* p, int len) {
    if (len <= 0) return;
    auto dw = [&](uint32_t w) {
        if constexpr (HASH) h.word(w);
        if constexpr (WRITE) s.word(w);
    };
    auto by = [&](uint32_t b) {
        if constexpr (HASH) h.byte(b);
        if constexpr (WRITE) s.byte(b);
    };
    auto eat = [&](const u32x4& v) {
        dw(v.x);
        dw(v.y);
        dw(v.z);
        dw(v.w);
    };
    const int head = min(len, (int)((16u - ((uintptr_t)p & 15u)) & 15u));
    for (int i = 0; i < head; ++i) by(p[i]);
    const u32x4* q = (const u32x4*)(p + head);
    const int rest = len - head;
    const int nc = rest >> 6;   // 64-byte chunks
    // Line writer for the chunks: 16 source bytes make 4 output dwords d0..d3 (realigned by
    // pb = ptr % 4 bytes with the carry), which land at dword positions di..di+3 of the
    // output's 16-byte lines (di = the dword index of ptr - pb in its line, fixed for the
    // span).  Rotated right by di they fill line L's positions di..3 and line L+1's 0..di-1:
    // line L = (positions < di ? the previous rotation : this one), one 16-byte store; the
    // first line is stored dword by dword from position di (the bytes before it are stored
    // already or are not this writer's), the last partial line by flush_line.
    const uint32_t pb = (uint32_t)(uintptr_t)s.ptr & 3u;
    const uint32_t di = ((uint32_t)((uintptr_t)s.ptr - pb) >> 2) & 3u;
    const uint32_t sh = 4u - pb;
    uint32_t P0 = 0, P1 = 0, P2 = 0, P3 = 0;
    auto eat4 = [&](const u32x4& v, bool first) {
        if constexpr (HASH) {
            h.word(v.x);
            h.word(v.y);
            h.word(v.z);
            h.word(v.w);
        }
        if constexpr (WRITE) {
            uint32_t d0 = v.x, d1 = v.y, d2 = v.z, d3 = v.w, nc4 = 0;
            if (pb) {
                d0 = (v.x << (8 * pb)) | s.carry;
                d1 = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
                d2 = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
                d3 = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
                nc4 = v.w >> (8 * sh);
            }
            // rotate right by di: R[j] = d[(j - di) & 3]
            if (di & 1u) {
                const uint32_t t = d3;
                d3 = d2, d2 = d1, d1 = d0, d0 = t;
            }
            if (di & 2u) {
                uint32_t t = d0;
                d0 = d2, d2 = t;
                t = d1, d1 = d3, d3 = t;
            }
            uint8_t* line = s.ptr - pb - 4 * di;
            if (first) {
                if (di <= 0) s.store_dw(line, d0);
                if (di <= 1) s.store_dw(line + 4, d1);
                if (di <= 2) s.store_dw(line + 8, d2);
                s.store_dw(line + 12, d3);
            } else {
                u32x4 o;
                o.x = di > 0 ? P0 : d0;
                o.y = di > 1 ? P1 : d1;
                o.z = di > 2 ? P2 : d2;
                o.w = d3;
                *(u32x4*)line = o;
            }
            P0 = d0, P1 = d1, P2 = d2, P3 = d3;
            s.carry = nc4;
            s.ptr += 16;
        }
    };
    u32x4 a[CH], b[CH];
    if (nc > 0) {
#pragma unroll
        for (int u = 0; u < CH; ++u) a[u] = __builtin_nontemporal_load(q + u);
    }
    for (int j = 0; j < nc; j += 2) {
        if (j + 1 < nc) {
#pragma unroll
            for (int u = 0; u < CH; ++u) b[u] = __builtin_nontemporal_load(q + CH * (j + 1) + u);
        }
        eat4(a[0], j == 0);
#pragma unroll
        for (int u = 1; u < CH; ++u) eat4(a[u], false);
        if (j + 1 < nc) {
            if (j + 2 < nc) {
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    a[u] = __builtin_nontemporal_load(q + CH * (j + 2) + u);
            }
#pragma unroll
            for (int u = 0; u < CH; ++u) eat4(b[u], false);
        }
    }
    if constexpr (WRITE) {
        // the line the chunks left open: positions 0 .. di - 1 hold P0 .. P(di - 1)
        if (nc > 0) {
            uint8_t* line = s.ptr - pb - 4 * di;
            if (di > 0) s.store_dw(line, P0);
            if (di > 1) s.store_dw(line + 4, P1);
            if (di > 2) s.store_dw(line + 8, P2);
        }
    }
    (void)P3;
    const u32x4* r = q + CH * nc;
    const int nr = (rest & 63) >> 4;
#pragma unroll 1
    for (int u = 0; u < nr; ++u) eat(__builtin_nontemporal_load(r + u));
    const uint8_t* tb = (const uint8_t*)(r + nr);
    for (int i = 0; i < (rest & 15); ++i) by(tb[i]);
}

__device__ __forceinline__ int len_of(const int32_t* a, int all, long long i) {
    return a ? a[i] : all;
}

// the 12 tag bytes at c against (t0, t1, t2)
__device__ __forceinline__ bool tag_matches(const uint8_t* c, uint32_t t0, uint32_t t1,
                                            uint32_t t2) {
    uint32_t w[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
        w[q] = c[4 * q] | (c[4 * q + 1] << 8) | (c[4 * q + 2] << 16) |
               ((uint32_t)c[4 * q + 3] << 24);
    return w[0] == t0 && w[1] == t1 && w[2] == t2;
}

// Plaintext rows: packet p reads b + p * stride (ka == 0), or, grouped, packet
// p = g * (ka + kb) + i reads row (g, i) of a ([G][ka]) for i < ka and row (g, i - ka) of
// b ([G][kb]) otherwise.
struct PtRows {
    const uint8_t* a;
    const uint8_t* b;
    long long stride;
    int ka, kb;
};

__device__ __forceinline__ const uint8_t* pt_row(const PtRows& r, long long p) {
    if (r.ka == 0) return r.b + p * r.stride;
    const int per = r.ka + r.kb;
    const long long g = p / per;
    const int i = (int)(p - g * per);
    return i < r.ka ? r.a + (g * r.ka + i) * r.stride : r.b + (g * r.kb + (i - r.ka)) * r.stride;
}

template <class H>
__global__ __launch_bounds__(kPPThreads) void null_seal_kernel(
    long long n, const uint8_t* __restrict__ ad, long long ad_stride,
    const int32_t* __restrict__ ad_len, int ad_all, PtRows pr, const int32_t* __restrict__ pt_len,
    int pt_all, uint8_t* out, long long out_stride, int32_t* out_len) {
    const long long i = (long long)blockIdx.x * kPPThreads + threadIdx.x;
    if (i >= n) return;
    const int al = len_of(ad_len, ad_all, i), pl = len_of(pt_len, pt_all, i);
    // a row longer than its stride would read the next packet's bytes (or past the buffer for
    // the last one): rejected like a packet that does not fit
    const bool ok = al >= 0 && pl >= 0 && (ad_stride == 0 || al <= ad_stride) &&
                    (pr.stride == 0 || pl <= pr.stride) && (long long)al + 12 + pl <= out_stride;
    out_len[i] = ok ? al + 12 + pl : -1;
    if (!ok) return;
    uint8_t* o = out + i * out_stride;
    H h;
    h.init();
    Sink s;
    s.begin(o);
    span<true, true>(h, s, ad + i * ad_stride, al);
    Sink t = s;   // AD's unstored tail bytes; the tag follows them once it is known
    s.begin(o + al + 12);
    span<true, true>(h, s, pt_row(pr, i), pl);
    s.flush();
    uint32_t t0, t1, t2;
    h.tag(t0, t1, t2);
    t.word(t0);
    t.word(t1);
    t.word(t2);
    t.flush();
}

template <class H>
__global__ __launch_bounds__(kPPThreads) void null_open_kernel(
    long long n, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ pkt_len, int pkt_all, const int32_t* __restrict__ ad_len,
    int ad_all, uint8_t* out, long long out_stride, int32_t* out_len) {
    const long long i = (long long)blockIdx.x * kPPThreads + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = pkt + i * pkt_stride;
    const int al = len_of(ad_len, ad_all, i);
    const int tl = len_of(pkt_len, pkt_all, i);
    const int cl = tl - al;   // ciphertext bytes
    // the output receives the ciphertext (reference: before any check)
    const bool copy = al >= 0 && cl >= 0 && cl <= out_stride && (pkt_stride == 0 || tl <= pkt_stride);
    if (!copy) {
        out_len[i] = -1;
        return;
    }
    uint8_t* o = out + i * out_stride;
    const uint8_t* c = p + al;
    int res = -1;
    if (cl >= 12) {
        H h;
        h.init();
        Sink s;
        s.begin(o);
        span<true, false>(h, s, p, al);
        span<true, true>(h, s, c + 12, cl - 12);
        uint32_t t0, t1, t2;
        h.tag(t0, t1, t2);
        if (tag_matches(c, t0, t1, t2)) {
            // accepted: the plaintext, then the last 12 bytes of the ciphertext copy the
            // reference made first (its output buffer holds them past the plaintext)
            for (int q = 0; q < 12; ++q) s.byte(c[cl - 12 + q]);
            s.flush();
            res = cl - 12;
        }
    }
    if (res < 0) {
        // rejected: the ciphertext copy alone, over the plaintext stores of this lane
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        H h;
        Sink s;
        s.begin(o);
        span<false, true>(h, s, c, cl);
        s.flush();
    }
    out_len[i] = res;
}

// Receiver, grouped: packet p = g * (k + m) + i; a data packet's plaintext goes to its block
// slot, zero-padded to bb.
template <class H>
__global__ __launch_bounds__(kPPThreads) void open_group_kernel(
    int k, int m, int bb, long long n, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ pkt_len, const int32_t* __restrict__ ad_len, int ad_all,
    uint8_t* blocks, int32_t* open_len) {
    const long long p = (long long)blockIdx.x * kPPThreads + threadIdx.x;
    if (p >= n) return;
    const int per = k + m;
    const long long g = p / per;
    const int i = (int)(p - g * per);
    const int tl = pkt_len[p], al = len_of(ad_len, ad_all, p);
    const int cl = tl - al;
    if (!(tl >= 0 && al >= 0 && cl >= 12 && cl - 12 <= bb && tl <= pkt_stride)) {
        open_len[p] = -1;
        return;
    }
    const uint8_t* pp = pkt + p * pkt_stride;
    const uint8_t* c = pp + al;
    H h;
    h.init();
    Sink s;
    span<true, false>(h, s, pp, al);
    if (i < k) {
        s.begin(blocks + (g * k + i) * (long long)bb);
        span<true, true>(h, s, c + 12, cl - 12);
        s.zeros_to(s.start + bb);
    } else {
        span<true, false>(h, s, c + 12, cl - 12);
    }
    uint32_t t0, t1, t2;
    h.tag(t0, t1, t2);
    open_len[p] = tag_matches(c, t0, t1, t2) ? cl - 12 : -1;
}

// dst[0 .. bb) = src[0 .. pl) zero-padded, by the whole wave
__device__ void wave_copy_pad(uint8_t* dst, const uint8_t* src, int pl, int bb, int lane) {
    if ((((uintptr_t)dst) | (uint32_t)bb) & 3u) {
        for (int o = lane; o < bb; o += 64) dst[o] = o < pl ? src[o] : 0;
        return;
    }
    const uint32_t sh = (uint32_t)(uintptr_t)src & 3u;
    const uint32_t* s4 = (const uint32_t*)(src - sh);
    const uint8_t* send = src + pl;
    for (int u = lane; u < (bb >> 2); u += 64) {
        const int o = 4 * u;
        uint32_t v = 0;
        if (o < pl) {
            // only dwords holding a plaintext byte are read
            const uint32_t w0 = s4[u];
            const uint32_t w1 = (sh && (const uint8_t*)(s4 + u + 1) < send) ? s4[u + 1] : 0u;
            v = sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
            if (pl - o < 4) v &= (1u << (8 * (pl - o))) - 1u;
        }
        ((uint32_t*)dst)[u] = v;
    }
}

constexpr int kAsmWaves = 4;

// One wave per group: rows[g][i] = i where data packet i opened; the holes, ascending, take
// the opened FEC packets, ascending (row k + j, plaintext copied into the slot); 255 where
// none is left (the decode then reports the group as malformed, status -3).
__global__ __launch_bounds__(kAsmWaves * 64) void open_assemble_kernel(
    int k, int m, int bb, long long groups, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ ad_len, int ad_all, const int32_t* __restrict__ open_len,
    uint8_t* blocks, uint8_t* rows) {
    __shared__ uint8_t lavail[kAsmWaves][256], lhole[kAsmWaves][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long g = (long long)blockIdx.x * kAsmWaves + w;
    if (g >= groups) return;   // uniform over the wave; no workgroup barrier below
    const int per = k + m;
    const int32_t* ol = open_len + g * per;
    const unsigned long long below = (1ull << lane) - 1ull;
    int na = 0;
    for (int b0 = 0; b0 < m; b0 += 64) {
        const int j = b0 + lane;
        const bool v = j < m && ol[k + j] >= 0;
        const unsigned long long bal = __ballot(v);
        if (v) lavail[w][na + __popcll(bal & below)] = (uint8_t)j;
        na += __popcll(bal);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's LDS writes are visible
    __builtin_amdgcn_wave_barrier();
    int nh = 0;
    for (int b0 = 0; b0 < k; b0 += 64) {
        const int i = b0 + lane;
        const bool miss = i < k && ol[i] < 0;
        const unsigned long long bal = __ballot(miss);
        const int r = nh + __popcll(bal & below);
        if (i < k) {
            int row = i;
            if (miss) {
                row = r < na ? k + lavail[w][r] : 255;
                if (r < na) lhole[w][r] = (uint8_t)i;
            }
            rows[g * k + i] = (uint8_t)row;
        }
        nh += __popcll(bal);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int nfill = min(nh, na);
    for (int h = 0; h < nfill; ++h) {
        const int j = lavail[w][h], i = lhole[w][h];
        const long long p = g * per + k + j;
        const uint8_t* src = pkt + p * pkt_stride + len_of(ad_len, ad_all, p) + 12;
        wave_copy_pad(blocks + (g * k + i) * (long long)bb, src, ol[k + j], bb, lane);
    }
}

// After the decode: a group with an unfilled slot (row 255) is malformed whatever path
// decoded it (the m = 1 XOR decode takes any row >= k as its parity block): status -3 and no
// recovered rows.
__global__ __launch_bounds__(kPPThreads) void open_status_kernel(long long groups, int k,
                                                                 int rmax,
                                                                 const uint8_t* __restrict__ rows,
                                                                 uint8_t* rec_rows,
                                                                 int32_t* status) {
    const long long g = (long long)blockIdx.x * kPPThreads + threadIdx.x;
    if (g >= groups) return;
    const uint8_t* r = rows + g * k;
    bool unfilled = false;
    for (int i = 0; i < k; ++i) unfilled |= r[i] == 255;
    if (!unfilled) return;
    if (status) status[g] = -3;
    for (int j = 0; j < rmax; ++j) rec_rows[g * rmax + j] = 255;
}

unsigned pp_grid(long long n) {
    return (unsigned)((n + kPPThreads - 1) / kPPThreads);
}

bool pp_grid_ok(long long n) {
    return (n + kPPThreads - 1) / kPPThreads <= 0x7fffffffLL;
}

}  // namespace

// pp_hash: 0 = the six-limb chain (Fnv), 1 = 64-bit halves (Fnv64)
#define QPP_GO(KERNEL, ...)                                                                 \
    do {                                                                                   \
        if (form == 1) qlaunch(KERNEL<Fnv64>, __VA_ARGS__);                                \
        else qlaunch(KERNEL<Fnv>, __VA_ARGS__);                                            \
    } while (0)

hipError_t launch_null_seal_h(int form, long long n, const uint8_t* ad, long long ad_stride,
                              const int32_t* ad_len, int ad_all, const uint8_t* pt,
                              long long pt_stride, const int32_t* pt_len, int pt_all,
                              uint8_t* out, long long out_stride, int32_t* out_len,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (!pp_grid_ok(n)) return hipErrorInvalidValue;
    const PtRows pr{nullptr, pt, pt_stride, 0, 1};
    note_kernel("null_seal_kernel");
    QPP_GO(null_seal_kernel, dim3(pp_grid(n)), dim3(kPPThreads), 0, st, n, ad, ad_stride, ad_len,
           ad_all, pr, pt_len, pt_all, out, out_stride, out_len);
    return hipGetLastError();
}

hipError_t launch_null_seal(long long n, const uint8_t* ad, long long ad_stride,
                            const int32_t* ad_len, int ad_all, const uint8_t* pt,
                            long long pt_stride, const int32_t* pt_len, int pt_all, uint8_t* out,
                            long long out_stride, int32_t* out_len, hipStream_t st) {
    return launch_null_seal_h(0, n, ad, ad_stride, ad_len, ad_all, pt, pt_stride, pt_len, pt_all,
                              out, out_stride, out_len, st);
}

hipError_t launch_null_seal_groups(int form, int k, int m, int bb, long long groups,
                                   const uint8_t* data, const uint8_t* parity, const uint8_t* hdr,
                                   long long hdr_stride, const int32_t* hdr_len, int hdr_all,
                                   const int32_t* pt_len, int pt_all, uint8_t* out,
                                   long long out_stride, int32_t* out_len, hipStream_t st) {
    const long long n = groups * (k + m);
    if (n <= 0) return hipSuccess;
    if (!pp_grid_ok(n)) return hipErrorInvalidValue;
    const PtRows pr{data, parity, bb, k, m};
    note_kernel("null_seal_kernel<groups>");
    QPP_GO(null_seal_kernel, dim3(pp_grid(n)), dim3(kPPThreads), 0, st, n, hdr, hdr_stride,
           hdr_len, hdr_all, pr, pt_len, pt_all, out, out_stride, out_len);
    return hipGetLastError();
}

hipError_t launch_null_open_h(int form, long long n, const uint8_t* pkt, long long pkt_stride,
                              const int32_t* pkt_len, int pkt_all, const int32_t* ad_len,
                              int ad_all, uint8_t* out, long long out_stride, int32_t* out_len,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (!pp_grid_ok(n)) return hipErrorInvalidValue;
    note_kernel("null_open_kernel");
    QPP_GO(null_open_kernel, dim3(pp_grid(n)), dim3(kPPThreads), 0, st, n, pkt, pkt_stride,
           pkt_len, pkt_all, ad_len, ad_all, out, out_stride, out_len);
    return hipGetLastError();
}

hipError_t launch_null_open(long long n, const uint8_t* pkt, long long pkt_stride,
                            const int32_t* pkt_len, int pkt_all, const int32_t* ad_len,
                            int ad_all, uint8_t* out, long long out_stride, int32_t* out_len,
                            hipStream_t st) {
    return launch_null_open_h(0, n, pkt, pkt_stride, pkt_len, pkt_all, ad_len, ad_all, out,
                              out_stride, out_len, st);
}

hipError_t launch_open_groups(int form, int k, int m, int bb, long long groups,
                              const uint8_t* pkt, long long pkt_stride, const int32_t* pkt_len,
                              const int32_t* ad_len, int ad_all, uint8_t* blocks,
                              uint8_t* rows, int32_t* open_len, hipStream_t st) {
    const long long n = groups * (k + m);
    if (n <= 0) return hipSuccess;
    if (k + m > 256 || !pp_grid_ok(n)) return hipErrorInvalidValue;
    const long long wg = (groups + kAsmWaves - 1) / kAsmWaves;
    if (wg > 0x7fffffffLL) return hipErrorInvalidValue;
    note_kernel("open_group_kernel + open_assemble_kernel");
    QPP_GO(open_group_kernel, dim3(pp_grid(n)), dim3(kPPThreads), 0, st, k, m, bb, n, pkt,
           pkt_stride, pkt_len, ad_len, ad_all, blocks, open_len);
    qlaunch(open_assemble_kernel, dim3((unsigned)wg), dim3(kAsmWaves * 64), 0, st, k, m, bb,
            groups, pkt, pkt_stride, ad_len, ad_all, open_len, blocks, rows);
    return hipGetLastError();
}
hipError_t launch_open_status(int k, int rmax, long long groups, const uint8_t* rows,
                              uint8_t* rec_rows, int32_t* status, hipStream_t st) {
    if (groups <= 0) return hipSuccess;
    if (!pp_grid_ok(groups)) return hipErrorInvalidValue;
    qlaunch(open_status_kernel, dim3(pp_grid(groups)), dim3(kPPThreads), 0, st, groups, k, rmax,
            rows, rec_rows, status);
    return hipGetLastError();
}
#undef QPP_GO

}  // namespace qfec
