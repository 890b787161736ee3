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
// The hash is a serial chain over the bytes of one packet, so one lane owns one packet's
// chain, while the bytes move in wave tiles (tile_stream): a wave's 64 packets stream through
// an 8 KB LDS tile in 128-byte windows.  Per window, 8 global_load_lds_dwordx4 bring 8
// packets x 128 contiguous bytes each (chunk c of packet q at slot c ^ (q & 7), an XOR
// swizzle so the lanes reading their own rows hit distinct banks); lane q hashes its packet's
// valid bytes from LDS and writes each full 16-byte output line (realigned to the output's byte
// phase, zeros past the source) back into the slot it consumed; then 8 coalesced
// global_store_dwordx4 in the same shape.  The two partial output lines at a packet's ends are
// written from registers after the loop.  Then the tag.
//
// The chain: h mod 2^96 (the tag is its low 96 bits) in three 32-bit words, one 64-bit
// multiply-add per word and byte (Fnv below).  Bound: the VALU of the chain and the tile's
// LDS round trips at four to five waves per SIMD.
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

// FNV-1a-128 modulo 2^96: the tag is the low 96 bits of the hash (quic_utils.cc:175-181,
// null_encrypter.cc:23-43; the decrypter compares the same bits), and arithmetic mod 2^128
// reduces to arithmetic mod 2^96, so bits 96..127 are never formed.  h is three 32-bit words;
// h * P = h * 315 + (h << 88): h * 315 is one 32 x 32 -> 64-bit multiply-add per word
// (v_mad_u64_u32; the low word's high half carries into the next, the top word's product is
// kept mod 2^32), and (h ^ byte) << 88 mod 2^96 is the XORed low byte shifted into bits 24..31
// of the top word.  About 8 VALU per byte, where r02-r06's five 22-bit limbs in carry-save form
// (v_mul_u32_u24 per limb, masks and shifts between) took 17; the chain alone runs 2.4x as
// fast (tools/microbench/fnv_rate.hip).
struct Fnv {
    uint32_t h0, h1, h2;
    // kOffset = 144066263297769815596495629667062367629 (quic_utils.cc:116-118) mod 2^96
    __device__ __forceinline__ void init() {
        h0 = 0x6295C58Du;
        h1 = 0x62B82175u;
        h2 = 0x07BB0142u;
    }
    __device__ __forceinline__ void byte(uint32_t b) {
        const uint32_t x0 = h0 ^ b;
        const uint64_t p0 = (uint64_t)x0 * 315u;
        const uint64_t p1 = (uint64_t)h1 * 315u + (p0 >> 32);
        h2 = h2 * 315u + (uint32_t)(p1 >> 32) + (x0 << 24);
        h0 = (uint32_t)p0;
        h1 = (uint32_t)p1;
    }
    __device__ __forceinline__ void word(uint32_t w) {
        byte(w & 0xFFu);
        byte((w >> 8) & 0xFFu);
        byte((w >> 16) & 0xFFu);
        byte(w >> 24);
    }
    // the low 96 bits of h, little-endian dwords (SerializeUint128Short, quic_utils.cc:175-181)
    __device__ __forceinline__ void tag(uint32_t& t0, uint32_t& t1, uint32_t& t2) const {
        t0 = h0, t1 = h1, t2 = h2;
    }
};

// stores through the global address space (a generic pointer compiles to flat stores, which
// also count on the LDS counter that tile_stream's waits after each ds_read use)
__device__ __forceinline__ void gst32(uint8_t* a, uint32_t v) {
    *(__attribute__((address_space(1))) uint32_t*)(uintptr_t)a = v;
}
__device__ __forceinline__ void gst8(uint8_t* a, uint32_t v) {
    *(__attribute__((address_space(1))) uint8_t*)(uintptr_t)a = (uint8_t)v;
}

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
            gst32(a, v);
        } else {
            for (int q = (int)(start - a); q < 4; ++q) gst8(a + q, v >> (8 * q));
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
            if (a + q >= start) gst8(a + q, carry >> (8 * q));
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
template <bool HASH, bool WRITE, int CHN = CH, class H>
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
    const int nc = rest / (16 * CHN);   // 16 * CHN-byte chunks
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
                *(__attribute__((address_space(1))) u32x4*)(uintptr_t)line = o;
            }
            P0 = d0, P1 = d1, P2 = d2, P3 = d3;
            s.carry = nc4;
            s.ptr += 16;
        }
    };
    u32x4 a[CHN], b[CHN];
    if (nc > 0) {
#pragma unroll
        for (int u = 0; u < CHN; ++u) a[u] = __builtin_nontemporal_load(q + u);
    }
    for (int j = 0; j < nc; j += 2) {
        if (j + 1 < nc) {
#pragma unroll
            for (int u = 0; u < CHN; ++u) b[u] = __builtin_nontemporal_load(q + CHN * (j + 1) + u);
        }
        eat4(a[0], j == 0);
#pragma unroll
        for (int u = 1; u < CHN; ++u) eat4(a[u], false);
        if (j + 1 < nc) {
            if (j + 2 < nc) {
#pragma unroll
                for (int u = 0; u < CHN; ++u)
                    a[u] = __builtin_nontemporal_load(q + CHN * (j + 2) + u);
            }
#pragma unroll
            for (int u = 0; u < CHN; ++u) eat4(b[u], false);
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
    const u32x4* r = q + CHN * nc;
    const int nr = (rest % (16 * CHN)) >> 4;
#pragma unroll 1
    for (int u = 0; u < nr; ++u) eat(__builtin_nontemporal_load(r + u));
    const uint8_t* tb = (const uint8_t*)(r + nr);
    for (int i = 0; i < (rest & 15); ++i) by(tb[i]);
}

__device__ __forceinline__ int len_of(const int32_t* a, int all, long long i) {
    return a ? a[i] : all;
}

// ------------------------------------------------------------------ wave-tiled stream
// The packets of a wave are streamed through an 8 KB LDS tile in 128-byte windows, so that
// both the loads and the stores are coalesced: one wave instruction moves 8 packets x 128
// contiguous bytes (8 lanes per packet, 16 bytes each) instead of 64 packets x 16 bytes, which
// touched 64 cache lines per instruction and cost 1.4x the reads (L2 re-fetches) and 1.55x
// the writes (partial lines) of the one-lane-per-packet streamer (profiles/r05/pp/).  Each lane
// still owns its packet's serial FNV chain.
//   window w of packet q: source chunks 8w .. 8w + 7 (16 bytes each) counted from the source's
//   128-byte aligned line, so that a window is one whole cache line; the tile row of packet q
//   is 128 bytes at q * 128, chunk c at slot c ^ (q & 7) (an XOR swizzle: lanes reading their
//   rows at one chunk index hit distinct banks).
//   1. loads: 8 global_load_lds_dwordx4 (instruction j: packets 8j .. 8j + 7, lane = 8 (q % 8)
//      + slot), each lane's address from its packet's lane by ds_bpermute (all 8 exchanges
//      issued before the first load, so their latency is paid once, not 8 times);
//   2. lane q reads its 8 chunks, hashes the valid bytes, and writes each FULL 16-byte output
//      line (realigned to the output's phase, zeros past the source) back into the slot of the
//      chunk it just consumed; the partial lines at the output's two ends stay in registers;
//   3. stores: 8 global_store_dwordx4 in the same shape (full lines only; exchanges and LDS
//      reads four instructions at a time), plain stores: the
//      next window's vmcnt(0) waits for them too, and non-temporal stores were acknowledged
//      later for the same bytes written (r06: 1.13 -> 0.73 ms for all of A's packets, WRITE_SIZE
//      unchanged).
// After the last window, the two partial end lines are written from registers, whole dwords
// where the output covers them.
// Measured and not kept: 64-byte windows double-buffered, two packets
// per lane, 16-byte aligned windows (each window straddled two lines), and (r06) two window
// buffers with the next window's DMA in flight during the hash (64- and 128-byte windows).
constexpr int kTileBytes = 64 * 128;   // one wave's tile
constexpr int kTilePackets = 64;       // packets per wave (one per lane)

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src_lane) {
    return (uint64_t)bperm((uint32_t)v, src_lane) | ((uint64_t)bperm((uint32_t)(v >> 32), src_lane) << 32);
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// The output line at per-lane dword offset mi (0..4) and byte offset ri (0..3) into the 32
// bytes P || C (the previous chunk, this chunk): dword t = bytes 4 (mi + t) + ri .. + 3, dwords
// past the pair clamped to C[3].  The five dwords it needs are selected by the bits of mi in
// three steps, then realigned by ri.
__device__ __forceinline__ u32x4 line_of(const uint32_t (&P)[4], const uint32_t (&C)[4], int mi,
                                         int ri) {
    // bitwise selects: a conditional between array elements would be folded into one load
    // with a computed index, which puts the array in scratch memory
    const uint32_t A[8] = {P[0], P[1], P[2], P[3], C[0], C[1], C[2], C[3]};
    const uint32_t m0 = 0u - (uint32_t)(mi & 1), m1 = 0u - (uint32_t)((mi >> 1) & 1);
    const uint32_t m2 = 0u - (uint32_t)((mi >> 2) & 1);
    uint32_t B[7], Q[5], V[5];
#pragma unroll
    for (int t = 0; t < 7; ++t) B[t] = (A[t + 1] & m0) | (A[t] & ~m0);
#pragma unroll
    for (int t = 0; t < 5; ++t) Q[t] = (B[t + 2] & m1) | (B[t] & ~m1);
#pragma unroll
    for (int t = 0; t < 5; ++t) V[t] = (A[min(4 + t, 7)] & m2) | (Q[t] & ~m2);
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(V[1], V[0], ri);
    o.y = __builtin_amdgcn_alignbyte(V[2], V[1], ri);
    o.z = __builtin_amdgcn_alignbyte(V[3], V[2], ri);
    o.w = __builtin_amdgcn_alignbyte(V[4], V[3], ri);
    return o;
}

// bytes [lo, hi) of the 16-byte line at L (16-byte aligned) from o: dword stores for the
// dwords inside the range, byte stores for the rest
__device__ __forceinline__ void part_line(uint8_t* L, const uint32_t (&o)[4], int lo, int hi) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (lo <= 4 * t && 4 * t + 4 <= hi) {
            gst32(L + 4 * t, o[t]);
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (lo <= 4 * t + b && 4 * t + b < hi) gst8(L + 4 * t + b, o[t] >> (8 * b));
        }
    }
}

// Hash pl source bytes at src into h and write them to dst, followed by zeros up to olen
// bytes (olen == 0: hash only).  Called by every lane of the wave together (wave-uniform
// loop); a lane with pl == 0 and olen == 0 only takes part.  tile: this wave's kTileBytes of
// LDS.  Every memory access of the routine is complete when it returns.  The first window
// starts at the source's 128-byte aligned line: the bytes before src that it loads lie in
// that line (never another page) and are neither hashed nor written.
template <class H>
__device__ void tile_stream(H& h, const uint8_t* src, int pl, uint8_t* dst, int olen,
                            uint8_t* tile) {
    const int lane = (int)__lane_id();
    const uintptr_t sp = (uintptr_t)src;
    const int hoff = pl > 0 ? (int)(sp & 127u) : 0;
    const uint64_t s128 = (uint64_t)(sp - hoff);
    const int cmax = pl > 0 ? (hoff + pl - 1) >> 4 : -1;   // last chunk holding a source byte
    const int send = hoff + pl;                             // source end, chunk coordinates
    // output: stream byte x goes to D + x, D = dst - hoff; 16-byte lines from A0 = D rounded
    // down; the full lines jf .. jl lie inside [dst, dst + olen)
    const uint64_t D = (uint64_t)(uintptr_t)dst - (uint64_t)hoff;
    const int e = (int)(D & 15u);
    const uint64_t A0 = D - (uint64_t)e;
    int jf = 0, jl = -1;
    if (olen > 0) {
        jf = (int)(((uint64_t)(uintptr_t)dst - A0 + 15u) >> 4);
        jl = (int)(((uint64_t)(uintptr_t)dst + (uint64_t)olen - A0) >> 4) - 1;
    }
    // the partial output lines at the two ends: line jf - 1 (when dst is inside it) and line
    // jl + 1 (when the output ends inside it); the same line when the output lies in one line
    const bool hpart = olen > 0 && (uint64_t)(uintptr_t)dst != A0 + 16u * (uint64_t)jf;
    const bool tpart = olen > 0 && (uint64_t)(uintptr_t)dst + (uint64_t)olen != A0 + 16u * (uint64_t)(jl + 1);
    const int last = max(cmax, tpart ? jl + 1 : jl);
    const int nwin_l = last >= 0 ? (last >> 3) + 1 : 0;
    const int nwin = wave_max(nwin_l);
    // line g = stream bytes [16 g - e, 16 g - e + 16): from (previous chunk, this chunk)
    const int mi = (16 - e) >> 2, ri = (16 - e) & 3;
    uint32_t P[4] = {0u, 0u, 0u, 0u};
    uint32_t Hd[4] = {0u, 0u, 0u, 0u}, Tl[4] = {0u, 0u, 0u, 0u};
    const int lq = lane >> 3, pos = lane & 7;
    const int rowoff = lane * 128, sw = lane & 7;
    const uint32_t tb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)tile;
#pragma unroll 1
    for (int w = 0; w < nwin; ++w) {
        // 1. coalesced loads: instruction j brings packets 8j .. 8j + 7
        {
            uint64_t qs[8];
            int qc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {   // every exchange first: one wait for all of them
                qs[j] = bperm64(s128, 8 * j + lq);
                qc[j] = (int)bperm((uint32_t)cmax, 8 * j + lq);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int q = 8 * j + lq;
                const int cg = 8 * w + (pos ^ (q & 7));
                if (cg <= qc[j])
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(uintptr_t)(qs[j] + 16u * (uint64_t)cg),
                        (__attribute__((address_space(3))) void*)(tile + 1024 * j), 16, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // 2. this lane's row: hash, full output lines back into the tile, end lines kept
        if (w < nwin_l) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int g = 8 * w + c;
                const uint32_t a = tb + (uint32_t)(rowoff + ((c ^ sw) << 4));
                uint32_t C[4] = {0u, 0u, 0u, 0u};
                if (g <= cmax && 16 * g + 16 > hoff) {   // chunks before the source stay zero
                    u32x4 v;
                    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
                    C[0] = v.x, C[1] = v.y, C[2] = v.z, C[3] = v.w;
                    const int x0 = 16 * g;
                    if (x0 >= hoff && x0 + 16 <= send) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) h.word(C[t]);
                    } else {
                        // a partial chunk: hash its valid bytes, zero the bytes past the source
#pragma unroll 1
                        for (int b = 0; b < 16; ++b) {
                            const int x = x0 + b;
                            if (x >= hoff && x < send) h.byte((C[b >> 2] >> (8 * (b & 3))) & 0xFFu);
                        }
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int keep = min(max(send - (x0 + 4 * t), 0), 4);
                            C[t] = keep >= 4 ? C[t] : keep <= 0 ? 0u : (C[t] & ((1u << (8 * keep)) - 1u));
                        }
                    }
                }
                const bool full = g >= jf && g <= jl;
                const bool hl = hpart && g == jf - 1, tl = tpart && g == jl + 1;
                if (full || hl || tl) {
                    const u32x4 o = line_of(P, C, mi, ri);
                    if (hl) Hd[0] = o.x, Hd[1] = o.y, Hd[2] = o.z, Hd[3] = o.w;
                    if (tl) Tl[0] = o.x, Tl[1] = o.y, Tl[2] = o.z, Tl[3] = o.w;
                    if (full) asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(o) : "memory");
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) P[t] = C[t];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // 3. coalesced stores of the full lines: instruction j, packets 8j .. 8j + 7
#pragma unroll
        for (int h4 = 0; h4 < 8; h4 += 4) {   // four instructions at a time: exchanges and
            int qf[4], ql[4];                  // LDS reads issued together, one wait each
            uint64_t qa[4];
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = 8 * (h4 + u) + lq;
                qf[u] = (int)bperm((uint32_t)jf, q);
                ql[u] = (int)bperm((uint32_t)jl, q);
                qa[u] = bperm64(A0, q);
                const uint32_t a = tb + (uint32_t)(q * 128 + ((pos ^ (q & 7)) << 4));
                asm volatile("ds_read_b128 %0, %1" : "=v"(v[u]) : "v"(a) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int g = 8 * w + pos;
                if (g >= qf[u] && g <= ql[u])
                    *(__attribute__((address_space(1))) u32x4*)(uintptr_t)(qa[u] + 16u * (uint64_t)g) = v[u];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // 4. the partial lines at both ends, from registers
    if (hpart) {
        uint8_t* L = (uint8_t*)(uintptr_t)(A0 + 16u * (uint64_t)(jf - 1));
        part_line(L, Hd, (int)(dst - L), min(16, (int)(dst + olen - L)));
    }
    if (tpart && !(hpart && jl + 1 == jf - 1)) {
        uint8_t* L = (uint8_t*)(uintptr_t)(A0 + 16u * (uint64_t)(jl + 1));
        part_line(L, Tl, max(0, (int)(dst - L)), (int)(dst + olen - L));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// One wave seals 64 packets (one per lane): the AD through the lane's own streamer (a few
// bytes), the plaintext through the wave's LDS tile (tile_stream), then the tag.
template <class H>
__global__ __launch_bounds__(64) void null_seal_kernel(
    long long n, const uint8_t* __restrict__ ad, long long ad_stride,
    const int32_t* __restrict__ ad_len, int ad_all, PtRows pr, const int32_t* __restrict__ pt_len,
    int pt_all, uint8_t* out, long long out_stride, int32_t* out_len) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const long long i = (long long)blockIdx.x * 64 + threadIdx.x;
    bool ok = false;
    int al = 0, pl = 0;
    if (i < n) {
        al = len_of(ad_len, ad_all, i);
        pl = len_of(pt_len, pt_all, i);
        // a row longer than its stride would read the next packet's bytes (or past the buffer
        // for the last one): rejected like a packet that does not fit
        ok = al >= 0 && pl >= 0 && (ad_stride == 0 || al <= ad_stride) &&
             (pr.stride == 0 || pl <= pr.stride) && (long long)al + 12 + pl <= out_stride;
        out_len[i] = ok ? al + 12 + pl : -1;
    }
    uint8_t* o = out + (ok ? i : 0) * out_stride;
    H h;
    h.init();
    Sink s, t;
    s.begin(o);
    if (ok) span<true, true, 1>(h, s, ad + i * ad_stride, al);   // a few bytes: 16-byte pieces
    t = s;   // AD's unstored tail bytes; the tag follows them once it is known
    tile_stream(h, ok ? pt_row(pr, i) : nullptr, ok ? pl : 0, o + al + 12, ok ? pl : 0, smem);
    if (!ok) return;
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

// The open's length checks alone (the tag is checked later): a packet that fails them is
// rejected whatever its bytes.
__device__ __forceinline__ bool open_len_ok(const int32_t* __restrict__ pkt_len,
                                            const int32_t* __restrict__ ad_len, int ad_all,
                                            long long p, int bb, long long pkt_stride) {
    const int tl = pkt_len[p];
    const int al = len_of(ad_len, ad_all, p);
    const int cl = tl - al;
    return tl >= 0 && al >= 0 && cl >= 12 && cl - 12 <= bb && tl <= pkt_stride;
}

// The slot FEC packet i (>= k) of group g is written to by the open, before any tag is known:
// the holes and the available FEC packets as the length checks alone leave them, matched in
// ascending order as open_assemble_kernel matches them (the j-th available FEC packet fills
// the j-th hole); -1 when it fills none.  Where a tag check then changes the match,
// open_assemble_kernel copies the right packet over.
__device__ int fec_pre_slot(const int32_t* __restrict__ pkt_len,
                            const int32_t* __restrict__ ad_len, int ad_all, long long g, int i,
                            int k, int m, int bb, long long pkt_stride) {
    const long long p0 = g * (k + m);
    int j = 0;
#pragma unroll 4
    for (int q = k; q < i; ++q) j += open_len_ok(pkt_len, ad_len, ad_all, p0 + q, bb, pkt_stride) ? 1 : 0;
#pragma unroll 8
    for (int x = 0; x < k; ++x) {
        if (open_len_ok(pkt_len, ad_len, ad_all, p0 + x, bb, pkt_stride)) continue;
        if (j == 0) return x;
        --j;
    }
    return -1;
}

// Receiver, grouped: packet p = g * (k + m) + i, one wave per 64 packets; a data packet's
// plaintext goes to its block slot, zero-padded to bb, through the wave's LDS tile, and so
// does an FEC packet's, into the hole it fills if the tags change nothing (fec_pre_slot).
template <class H>
__global__ __launch_bounds__(64) void open_group_kernel(
    int k, int m, int bb, long long n, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ pkt_len, const int32_t* __restrict__ ad_len, int ad_all,
    uint8_t* blocks, int32_t* open_len) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const long long p = (long long)blockIdx.x * 64 + threadIdx.x;
    const int per = k + m;
    const long long g = p / per;
    const int i = (int)(p - g * per);
    bool ok = false;
    int al = 0, cl = 0;
    if (p < n) {
        const int tl = pkt_len[p];
        al = len_of(ad_len, ad_all, p);
        cl = tl - al;
        ok = tl >= 0 && al >= 0 && cl >= 12 && cl - 12 <= bb && tl <= pkt_stride;
        if (!ok) open_len[p] = -1;
    }
    const uint8_t* pp = pkt + (ok ? p : 0) * pkt_stride;
    const uint8_t* c = pp + al;
    H h;
    h.init();
    Sink s;
    if (ok) span<true, false, 1>(h, s, pp, al);
    const int slot = !ok ? -1 : i < k ? i
                   : fec_pre_slot(pkt_len, ad_len, ad_all, g, i, k, m, bb, pkt_stride);
    tile_stream(h, ok ? c + 12 : nullptr, ok ? cl - 12 : 0,
                slot >= 0 ? blocks + (g * k + slot) * (long long)bb : nullptr, slot >= 0 ? bb : 0,
                smem);
    if (!ok) return;
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
// the opened FEC packets, ascending (row k + j); 255 where none is left (the decode then
// reports the group as malformed, status -3).  The open has already written each FEC packet
// into the hole the length checks alone give it (fec_pre_slot); a pair the tag checks
// changed is copied here.
__global__ __launch_bounds__(kAsmWaves * 64) void open_assemble_kernel(
    int k, int m, int bb, long long groups, const uint8_t* __restrict__ pkt, long long pkt_stride,
    const int32_t* __restrict__ pkt_len, const int32_t* __restrict__ ad_len, int ad_all,
    const int32_t* __restrict__ open_len, uint8_t* blocks, uint8_t* rows) {
    __shared__ uint8_t lavail[kAsmWaves][256], lhole[kAsmWaves][256];
    __shared__ uint8_t prank[kAsmWaves][256], phole[kAsmWaves][256];
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
    // the match the open wrote by (fec_pre_slot): ranks of the FEC packets and the holes by
    // the length checks alone
    int npa = 0, nph = 0;
    for (int b0 = 0; b0 < m; b0 += 64) {
        const int j = b0 + lane;
        const bool v = j < m && open_len_ok(pkt_len, ad_len, ad_all, g * per + k + j, bb, pkt_stride);
        const unsigned long long bal = __ballot(v);
        if (j < m) prank[w][j] = v ? (uint8_t)(npa + __popcll(bal & below)) : (uint8_t)255;
        npa += __popcll(bal);
    }
    for (int b0 = 0; b0 < k; b0 += 64) {
        const int i = b0 + lane;
        const bool miss = i < k && !open_len_ok(pkt_len, ad_len, ad_all, g * per + i, bb, pkt_stride);
        const unsigned long long bal = __ballot(miss);
        if (miss) phole[w][nph + __popcll(bal & below)] = (uint8_t)i;
        nph += __popcll(bal);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int nfill = min(nh, na);
    for (int h = 0; h < nfill; ++h) {
        const int j = lavail[w][h], i = lhole[w][h];
        const int pr = prank[w][j];
        if (pr < nph && phole[w][pr] == i) continue;   // written there by the open
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
    return (n + 63) / 64 <= 0x7fffffffLL;
}

unsigned tile_grid(long long n) {   // one wave (kTilePackets packets) per workgroup
    return (unsigned)((n + kTilePackets - 1) / kTilePackets);
}

}  // namespace

#define QPP_GO(KERNEL, ...) qlaunch(KERNEL<Fnv>, __VA_ARGS__)

hipError_t launch_null_seal_h(long long n, const uint8_t* ad, long long ad_stride,
                              const int32_t* ad_len, int ad_all, const uint8_t* pt,
                              long long pt_stride, const int32_t* pt_len, int pt_all,
                              uint8_t* out, long long out_stride, int32_t* out_len,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (!pp_grid_ok(n)) return hipErrorInvalidValue;
    const PtRows pr{nullptr, pt, pt_stride, 0, 1};
    note_kernel("null_seal_kernel");
    QPP_GO(null_seal_kernel, dim3(tile_grid(n)), dim3(64), kTileBytes, st, n, ad, ad_stride,
           ad_len, ad_all, pr, pt_len, pt_all, out, out_stride, out_len);
    return hipGetLastError();
}

hipError_t launch_null_seal(long long n, const uint8_t* ad, long long ad_stride,
                            const int32_t* ad_len, int ad_all, const uint8_t* pt,
                            long long pt_stride, const int32_t* pt_len, int pt_all, uint8_t* out,
                            long long out_stride, int32_t* out_len, hipStream_t st) {
    return launch_null_seal_h(n, ad, ad_stride, ad_len, ad_all, pt, pt_stride, pt_len, pt_all,
                              out, out_stride, out_len, st);
}

hipError_t launch_null_seal_groups(int k, int m, int bb, long long groups,
                                   const uint8_t* data, const uint8_t* parity, const uint8_t* hdr,
                                   long long hdr_stride, const int32_t* hdr_len, int hdr_all,
                                   const int32_t* pt_len, int pt_all, uint8_t* out,
                                   long long out_stride, int32_t* out_len, hipStream_t st) {
    const long long n = groups * (k + m);
    if (n <= 0) return hipSuccess;
    if (!pp_grid_ok(n)) return hipErrorInvalidValue;
    const PtRows pr{data, parity, bb, k, m};
    note_kernel("null_seal_kernel<groups>");
    QPP_GO(null_seal_kernel, dim3(tile_grid(n)), dim3(64), kTileBytes, st, n, hdr, hdr_stride,
           hdr_len, hdr_all, pr, pt_len, pt_all, out, out_stride, out_len);
    return hipGetLastError();
}

hipError_t launch_null_open_h(long long n, const uint8_t* pkt, long long pkt_stride,
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
    return launch_null_open_h(n, pkt, pkt_stride, pkt_len, pkt_all, ad_len, ad_all, out,
                              out_stride, out_len, st);
}

hipError_t launch_open_groups(int k, int m, int bb, long long groups,
                              const uint8_t* pkt, long long pkt_stride, const int32_t* pkt_len,
                              const int32_t* ad_len, int ad_all, uint8_t* blocks,
                              uint8_t* rows, int32_t* open_len, hipStream_t st) {
    const long long n = groups * (k + m);
    if (n <= 0) return hipSuccess;
    if (k + m > 256 || !pp_grid_ok(n)) return hipErrorInvalidValue;
    const long long wg = (groups + kAsmWaves - 1) / kAsmWaves;
    if (wg > 0x7fffffffLL) return hipErrorInvalidValue;
    note_kernel("open_group_kernel + open_assemble_kernel");
    QPP_GO(open_group_kernel, dim3(tile_grid(n)), dim3(64), kTileBytes, st, k, m, bb, n, pkt,
           pkt_stride, pkt_len, ad_len, ad_all, blocks, open_len);
    qlaunch(open_assemble_kernel, dim3((unsigned)wg), dim3(kAsmWaves * 64), 0, st, k, m, bb,
            groups, pkt, pkt_stride, pkt_len, ad_len, ad_all, open_len, blocks, rows);
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
