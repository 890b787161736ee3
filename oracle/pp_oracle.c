/*
 * pp_oracle.c — CPU ORACLE for the packet-protection step adjacent to the FEC path
 * (SURVEY.md §8 f, rank 4).  TEST INFRASTRUCTURE ONLY: linked into
 * oracle/liboracle_fec.so next to fec_oracle.c, never into the product.
 *
 * What the reference does to a packet around the codec:
 *  - sender: QuicPacketCreator::SerializeFec builds the FEC packet (header + parity) and
 *    calls QuicFramer::EncryptInPlace with the header as associated data
 *    (quic_packet_creator.cc:948-953, quic_framer.cc:1921-1939);
 *  - receiver: the framer decrypts every packet before the group sees it
 *    (quic_framer.cc:657, DecryptPayload).
 * In this fork QuicEncrypter::Create maps kNULL to NullEncrypter and kAESG / kCC20 /
 * kNone to MyEncrypter, an identity copy (crypto/quic_encrypter.cc:18-29,
 * crypto/none_encrypter.cc EncryptPacket: memcpy, no tag).  NullEncrypter is the one with
 * arithmetic, restated here:
 *  - seal  (null_encrypter.cc:23-43): h = FNV-1a-128(AD || PT); out = h[0..12) || PT,
 *    h serialised little-endian, low 8 bytes then the low 4 of the high half
 *    (quic_utils.cc:175-181 SerializeUint128Short);
 *  - open  (null_decrypter.cc DecryptPacket, ReadHash, ComputeHash): output first gets a
 *    copy of the ciphertext; fail if fewer than 12 bytes; tag = u64 LE || u32 LE; accept iff
 *    tag == FNV-1a-128(AD || CT[12..]) with the top 32 bits cleared; then output = CT[12..];
 *  - FNV-1a-128 (quic_utils.cc:38-56,110-125): offset 144066263297769815596495629667062367629,
 *    prime 2^88 + 315, h = (h ^ byte) * prime mod 2^128, over data1 then data2.
 *
 * Parity: pinned by the reference's own known-answer tests,
 * null_encrypter_test.cc:16-27 and null_decrypter_test.cc (Decrypt / BadHash / ShortInput),
 * which tests/test_pp_oracle.py replays.  quic_utils.cc needs Chromium base/ and cannot be
 * compiled here, so the reference itself is not run.
 */
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;

static u128 fnv_offset(void) {
    /* kOffset(7809847782465536322, 7113472399480571277), quic_utils.cc:117-118 */
    return ((u128)UINT64_C(7809847782465536322) << 64) | UINT64_C(7113472399480571277);
}

static u128 fnv_run(u128 h, const uint8_t *p, long long n) {
    const u128 prime = ((u128)16777216 << 64) + 315; /* quic_utils.cc:46-47 */
    for (long long i = 0; i < n; ++i) h = (h ^ p[i]) * prime;
    return h;
}

/* FNV1a_128_Hash_Two(d1, l1, d2, l2) -> out[0] = low 64 bits, out[1] = high 64 bits */
void oracle_fnv1a_128_two(const uint8_t *d1, long long l1, const uint8_t *d2, long long l2,
                          uint64_t out[2]) {
    u128 h = fnv_run(fnv_offset(), d1, l1);
    if (d2) h = fnv_run(h, d2, l2);
    out[0] = (uint64_t)h;
    out[1] = (uint64_t)(h >> 64);
}

/* NullEncrypter::EncryptPacket: writes hash12 || PT to out; returns the output length, or
 * -1 when max_out is too small (the reference returns false). */
long long oracle_null_seal(const uint8_t *ad, long long ad_len, const uint8_t *pt,
                           long long pt_len, uint8_t *out, long long max_out) {
    const long long len = pt_len + 12;
    if (max_out < len) return -1;
    uint64_t h[2];
    oracle_fnv1a_128_two(ad, ad_len, pt, pt_len, h);
    memmove(out + 12, pt, (size_t)pt_len);
    memcpy(out, &h[0], 8);
    memcpy(out + 8, &h[1], 4);
    return len;
}

/* NullDecrypter::DecryptPacket: returns the plaintext length written to out, or -1 on
 * rejection (short input, output too small, hash mismatch).  Like the reference, out first
 * receives a copy of the ciphertext, so a rejected packet leaves that copy behind. */
long long oracle_null_open(const uint8_t *ad, long long ad_len, const uint8_t *ct,
                           long long ct_len, uint8_t *out, long long max_out) {
    memcpy(out, ct, (size_t)ct_len);
    if (ct_len < 12) return -1;
    uint64_t lo;
    uint32_t hi;
    memcpy(&lo, ct, 8);
    memcpy(&hi, ct + 8, 4);
    const long long pl = ct_len - 12;
    if (pl > max_out) return -1;
    uint64_t h[2];
    oracle_fnv1a_128_two(ad, ad_len, ct + 12, pl, h);
    if (h[0] != lo || (uint32_t)h[1] != hi) return -1; /* top 32 bits masked off */
    memmove(out, ct + 12, (size_t)pl);
    return pl;
}

/* Batches over packet arrays with fixed strides and per-packet lengths (the GPU ABI's
 * layout).  Seal: packet i's AD at ad + i*ad_stride (ad_len[i] bytes), its plaintext at
 * in + i*in_stride (in_len[i] bytes); the wire packet AD || hash12 || PT goes to
 * out + i*out_stride.  Open: wire packet i at in + i*in_stride (in_len[i] bytes, of which the
 * first ad_len[i] are the AD); its plaintext goes to out + i*out_stride.  res[i] = output
 * length or -1. */
void oracle_null_seal_batch(long long n, const uint8_t *ad, long long ad_stride,
                            const int32_t *ad_len, const uint8_t *in, long long in_stride,
                            const int32_t *in_len, uint8_t *out, long long out_stride,
                            int32_t *res) {
    for (long long i = 0; i < n; ++i) {
        uint8_t *o = out + i * out_stride;
        const long long al = ad_len[i];
        if (al < 0 || in_len[i] < 0 || out_stride < al + 12 + in_len[i] ||
            (ad_stride && al > ad_stride) || (in_stride && in_len[i] > in_stride)) {
            res[i] = -1; /* nothing written */
            continue;
        }
        memcpy(o, ad + i * ad_stride, (size_t)al);
        const long long r =
            oracle_null_seal(ad + i * ad_stride, al, in + i * in_stride, in_len[i], o + al,
                             out_stride - al);
        res[i] = r < 0 ? -1 : (int32_t)(al + r);
    }
}

void oracle_null_open_batch(long long n, const uint8_t *in, long long in_stride,
                            const int32_t *in_len, const int32_t *ad_len, uint8_t *out,
                            long long out_stride, int32_t *res) {
    for (long long i = 0; i < n; ++i) {
        const uint8_t *p = in + i * in_stride;
        const long long al = ad_len[i];
        if (al < 0 || al > in_len[i] || out_stride < in_len[i] - al ||
            (in_stride && in_len[i] > in_stride)) {
            res[i] = -1;
            continue;
        }
        res[i] = (int32_t)oracle_null_open(p, al, p + al, in_len[i] - al, out + i * out_stride,
                                           out_stride);
    }
}
