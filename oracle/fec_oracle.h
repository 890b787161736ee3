/*
 * fec_oracle.h — CPU ORACLE for the FEC hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline.  The product path
 * (quic_amd/libquic_fec.so) never links, loads or calls it.
 *
 * Parity: pinned against golden vectors produced by the reference codec itself
 * (oracle/_ref/libref_cauchy.so compiled from /root/reference by
 * oracle/Makefile; vectors in tests/golden/, script tests/golden/gen_golden.py).
 */
#ifndef QUIC_AMD_FEC_ORACLE_H
#define QUIC_AMD_FEC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    unsigned char *data;
    unsigned char row;
} OracleBlock; /* same layout as cauchy_256.h:52-55 `Block` */

/* Load the Cauchy table blob (quic_amd/data/cauchy_256_tables.bin). 0 = ok. */
int oracle_init(const char *tables_path);

/* GF(256), poly 0x187 (cauchy_256.cpp:272-412). */
uint8_t oracle_gf_mul(uint8_t x, uint8_t y);
uint8_t oracle_gf_div(uint8_t x, uint8_t y);
uint8_t oracle_gf_inv(uint8_t x);

/* Rows y = 1..m-1 of the Cauchy matrix, (m-1) x k, row-major (cauchy_256.cpp:422-480).
 * Returns 0, or -1 if m < 2 or k + m > 256. */
int oracle_cauchy_matrix(int k, int m, uint8_t *out);

/* Drop-in semantics of cauchy_256_encode / cauchy_256_decode (cauchy_256.cpp:1502,1254). */
int oracle_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery, int block_bytes);
int oracle_decode(int k, int m, OracleBlock *blocks, int block_bytes);

/* Batched helpers over contiguous layouts (used by tests and the CPU baseline):
 *   data   [G][k][bb]      parity [G][m][bb]
 *   blocks [G][k][bb] (in place)   rows [G][k] (in place)   status [G] (may be NULL)
 * `threads` > 1 splits groups contiguously over pthreads. */
int oracle_encode_batch(int k, int m, int bb, long long groups, const uint8_t *data,
                        uint8_t *parity, int threads);
int oracle_decode_batch(int k, int m, int bb, long long groups, uint8_t *blocks,
                        uint8_t *rows, int32_t *status, int threads);

/* Same batch loops, but calling an arbitrary codec with the cauchy_256 ABI
 * (used to time the compiled reference, oracle/_ref). */
typedef int (*cauchy_encode_fn)(int, int, const unsigned char **, void *, int);
typedef int (*cauchy_decode_fn)(int, int, OracleBlock *, int);
int oracle_run_encode_batch(cauchy_encode_fn fn, int k, int m, int bb, long long groups,
                            const uint8_t *data, uint8_t *parity, int threads);
int oracle_run_decode_batch(cauchy_decode_fn fn, int k, int m, int bb, long long groups,
                            uint8_t *blocks, uint8_t *rows, int32_t *status, int threads);

/* Synthetic input stream: 8-byte word i = splitmix64_mix(seed + (i+1)*0x9E3779B97F4A7C15),
 * little-endian, i.e. the sequential splitmix64 generator.  Fills n bytes starting at
 * byte offset `byte_offset` of the stream. */
void oracle_fill_stream(uint64_t seed, uint64_t byte_offset, uint8_t *out, uint64_t n);

/* Monotonic wall clock in seconds (for the CPU baseline). */
double oracle_now(void);

/* Packet protection next to the FEC path (pp_oracle.c; null_encrypter.cc:23-43,
 * null_decrypter.cc, quic_utils.cc:38-56,110-125,175-181).  out[0] = low, out[1] = high. */
void oracle_fnv1a_128_two(const uint8_t *d1, long long l1, const uint8_t *d2, long long l2,
                          uint64_t out[2]);
long long oracle_null_seal(const uint8_t *ad, long long ad_len, const uint8_t *pt,
                           long long pt_len, uint8_t *out, long long max_out);
long long oracle_null_open(const uint8_t *ad, long long ad_len, const uint8_t *ct,
                           long long ct_len, uint8_t *out, long long max_out);
void oracle_null_seal_batch(long long n, const uint8_t *ad, long long ad_stride,
                            const int32_t *ad_len, const uint8_t *in, long long in_stride,
                            const int32_t *in_len, uint8_t *out, long long out_stride,
                            int32_t *res);
void oracle_null_open_batch(long long n, const uint8_t *in, long long in_stride,
                            const int32_t *in_len, const int32_t *ad_len, uint8_t *out,
                            long long out_stride, int32_t *res);

#ifdef __cplusplus
}
#endif
#endif
