/*
 * fec_oracle.c — CPU ORACLE for the FEC encode/recover hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  A plain-C restatement of the reference codec
 * (Longhair "cauchy_256", vendored at /root/reference/net/quic/core/libcat/)
 * used as the checker for the HIP path and as the CPU baseline when the compiled
 * reference (oracle/_ref) is not available.  The product library never links,
 * loads or calls this file.
 *
 * Parity of this restatement is pinned by tests/test_oracle_golden.py against
 * golden vectors that the reference codec itself produced (tests/golden/).
 *
 * Each function cites the reference lines it restates.  This file restates the
 * NON-windowed algorithm (naive bitmatrix encode, cauchy_256.cpp:1561-1593;
 * eliminate_original + generate_bitmatrix + gaussian_elimination +
 * back_substitution, :655-795, :1020-1082, :1233-1252).  The windowed variants
 * the reference switches to for m > 4 / more than 4 erasures (:1419-1500,
 * :578-653, :809-1231) compute the same outputs.
 */
#define _POSIX_C_SOURCE 199309L
#include "fec_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- GF(2^8) */
/* Field GF(2^8) with the reduction polynomial 0x187 and generator 2
 * (cauchy_256.cpp:272).  The reference carries literal LOG/EXP/INV tables
 * (:274-343) and expands 64 KB MUL/DIV tables from them (:348-387); here the
 * same field is generated from the polynomial. */
static uint8_t g_exp[512];
static int g_log[256];
static uint8_t g_inv[256];

/* Cauchy table blob: M2|M3|M4|M5|M6|Y|X (tools/gen_cauchy_tables.py). */
enum { T_M2 = 0, T_M3 = T_M2 + 254, T_M4 = T_M3 + 506, T_M5 = T_M4 + 756,
       T_M6 = T_M5 + 1004, T_Y = T_M6 + 1250, T_X = T_Y + 256, T_SIZE = T_X + 30876 };
static uint8_t g_tables[T_SIZE];
static int g_ready = 0;

static void gf_build(void)
{
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)v;
        g_log[v] = i;
        v <<= 1;
        if (v & 0x100) v ^= 0x187;
    }
    for (int i = 255; i < 512; ++i) g_exp[i] = g_exp[i - 255];
    g_log[0] = -1;
    g_inv[0] = 0;
    for (int x = 1; x < 256; ++x) g_inv[x] = g_exp[(255 - g_log[x]) % 255];
}

uint8_t oracle_gf_mul(uint8_t x, uint8_t y)
{
    /* GFC256Multiply (cauchy_256.cpp:402-405) */
    if (!x || !y) return 0;
    return g_exp[g_log[x] + g_log[y]];
}

uint8_t oracle_gf_div(uint8_t x, uint8_t y)
{
    /* GFC256Divide (cauchy_256.cpp:409-412); the reference's y = 0 row is all zeros */
    if (!x || !y) return 0;
    return g_exp[g_log[x] + 255 - g_log[y]];
}

uint8_t oracle_gf_inv(uint8_t x) { return g_inv[x]; }

int oracle_init(const char *tables_path)
{
    gf_build();
    FILE *f = fopen(tables_path, "rb");
    if (!f) return -1;
    size_t n = fread(g_tables, 1, sizeof(g_tables), f);
    int extra = fgetc(f);
    fclose(f);
    if (n != sizeof(g_tables) || extra != EOF) return -2;
    g_ready = 1;
    return 0;
}

/* ------------------------------------------------------------ Cauchy matrix */
int oracle_cauchy_matrix(int k, int m, uint8_t *out)
{
    /* cauchy_matrix(), cauchy_256.cpp:422-480: rows y = 1..m-1 (row 0 is the
     * implicit all-ones row). */
    if (m < 2 || k < 1 || k + m > 256) return -1;
    static const int base[7] = {0, 0, T_M2, T_M3, T_M4, T_M5, T_M6};
    if (m <= 6) {
        const int stride = 256 - m; /* :428-442 */
        for (int y = 1; y < m; ++y)
            for (int x = 0; x < k; ++x)
                out[(y - 1) * k + x] = g_tables[base[m] + (y - 1) * stride + x];
        return 0;
    }
    const int n = m - 7; /* :452-455 */
    const uint8_t *X = g_tables + T_X + n * 249 - n * (n + 1) / 2;
    const uint8_t *Y = g_tables + T_Y;
    for (int y = 1; y < m; ++y) { /* :465-476 */
        const uint8_t G = Y[y - 1];
        out[(y - 1) * k] = g_inv[1 ^ G];
        for (int x = 1; x < k; ++x) {
            const uint8_t B = X[x - 1];
            out[(y - 1) * k + x] = oracle_gf_div(B, B ^ G);
        }
    }
    return 0;
}

/* ------------------------------------------------------------- XOR helpers */
/* memxor / memxor_set (MemXOR.cpp:36,132) and memswap (MemSwap.cpp:31) */
static void xor_into(uint8_t *dst, const uint8_t *src, int n)
{
    for (int i = 0; i < n; ++i) dst[i] ^= src[i];
}

static void swap_bytes(uint8_t *a, uint8_t *b, int n)
{
    for (int i = 0; i < n; ++i) {
        uint8_t t = a[i];
        a[i] = b[i];
        b[i] = t;
    }
}

/* The 8x8 expansion used everywhere: sub-row r of the output takes input
 * sub-rows t where bit t of (c * 2^r) is set (cauchy_256.cpp:90-125, :1576-1591). */
static void mul_add_subrows(uint8_t *dest, const uint8_t *src, uint8_t c, int subbytes)
{
    uint8_t slice = c;
    for (int bit_y = 0; bit_y < 8; ++bit_y) {
        for (int bit_x = 0; bit_x < 8; ++bit_x)
            if (slice & (1u << bit_x)) xor_into(dest + bit_y * subbytes, src + bit_x * subbytes, subbytes);
        slice = oracle_gf_mul(slice, 2);
    }
}

/* ------------------------------------------------------------------ encode */
int oracle_encode(int k, int m, const unsigned char *data[], void *vrecovery, int block_bytes)
{
    /* cauchy_256_encode, cauchy_256.cpp:1502-1601 */
    uint8_t *rec = (uint8_t *)vrecovery;
    if (k < 1 || m < 1 || block_bytes < 1) return -1; /* reference: undefined */
    if (k <= 1) { /* :1508-1516 */
        for (int i = 0; i < m; ++i) memcpy(rec + (size_t)i * block_bytes, data[0], block_bytes);
        return 0;
    }
    for (int i = 0; i < block_bytes; ++i) rec[i] = data[0][i] ^ data[1][i]; /* :1519 */
    for (int x = 2; x < k; ++x) xor_into(rec, data[x], block_bytes);       /* :1521-1523 */
    if (m == 1) return 0;                                                    /* :1526-1528 */
    if (k + m > 256 || block_bytes % 8 != 0) return -1;                      /* :1532-1534 */

    uint8_t *C = (uint8_t *)malloc((size_t)k * (m - 1));
    oracle_cauchy_matrix(k, m, C);
    const int subbytes = block_bytes / 8;
    uint8_t *out = rec + block_bytes;
    memset(out, 0, (size_t)block_bytes * (m - 1)); /* :1554 */
    for (int y = 1; y < m; ++y, out += block_bytes)           /* :1564 */
        for (int x = 0; x < k; ++x)                             /* :1568 */
            mul_add_subrows(out, data[x], C[(y - 1) * k + x], subbytes);
    free(C);
    return 0;
}

/* ------------------------------------------------------------------ decode */
static void decode_m1(int k, OracleBlock *blocks, int block_bytes)
{
    /* cauchy_decode_m1, cauchy_256.cpp:486-540 */
    OracleBlock *erased = NULL;
    for (int i = 0; i < k; ++i)
        if (blocks[i].row >= k) { erased = &blocks[i]; break; }
    if (!erased) return;
    unsigned char seen[256] = {0};
    for (int i = 0; i < k; ++i) {
        OracleBlock *b = blocks + i;
        if (b == erased) continue;
        if (b->row < k) seen[b->row] = 1;
        xor_into(erased->data, b->data, block_bytes);
    }
    for (int i = 0; i < k; ++i)
        if (!seen[i]) { erased->row = (unsigned char)i; break; }
}

int oracle_decode(int k, int m, OracleBlock *blocks, int block_bytes)
{
    /* cauchy_256_decode, cauchy_256.cpp:1254-1413 */
    if (k <= 1) { blocks[0].row = 0; return 0; } /* :1257-1261 */
    if (m == 1) { decode_m1(k, blocks, block_bytes); return 0; } /* :1264-1267 */

    /* sort_blocks, :543-575 */
    OracleBlock *original[256], *recovery[256];
    int noriginal = 0, nrecovery = 0;
    uint8_t erasures[256];
    memset(erasures, 0, sizeof(erasures));
    for (int i = 0; i < k; ++i) {
        if (blocks[i].row < k) {
            original[noriginal++] = &blocks[i];
            erasures[blocks[i].row] = 1;
        } else {
            recovery[nrecovery++] = &blocks[i];
        }
    }
    for (int i = 0, n = 0; i < 256 && n < nrecovery; ++i)
        if (!erasures[i]) erasures[n++] = (uint8_t)i;
    if (nrecovery <= 0) return 0;                                  /* :1287-1289 */
    if (k + m > 256 || block_bytes % 8 != 0) return -1;           /* :1292-1294 */

    const int subbytes = block_bytes / 8;
    uint8_t *C = (uint8_t *)malloc((size_t)k * (m - 1));
    oracle_cauchy_matrix(k, m, C);

    /* eliminate_original, :655-710 (row k is the all-ones parity) */
    for (int i = 0; i < nrecovery; ++i) {
        const int y = recovery[i]->row - k;
        for (int j = 0; j < noriginal; ++j) {
            const uint8_t c = y == 0 ? 1 : C[(y - 1) * k + original[j]->row];
            if (c == 1) xor_into(recovery[i]->data, original[j]->data, block_bytes);
            else mul_add_subrows(recovery[i]->data, original[j]->data, c, subbytes);
        }
    }

    /* generate_bitmatrix, :712-795: bit row (8i + r), bit column (8j + t) is
     * bit t of C[y_i][erasure_j] * 2^r; identity pattern for the parity-0 row. */
    const int R = nrecovery * 8;
    const int W = (R + 63) / 64;
    uint64_t *bm = (uint64_t *)calloc((size_t)R * W, sizeof(uint64_t));
    for (int i = 0; i < nrecovery; ++i) {
        const int y = recovery[i]->row - k;
        for (int j = 0; j < nrecovery; ++j) {
            uint8_t slice = y == 0 ? 1 : C[(y - 1) * k + erasures[j]];
            for (int r = 0; r < 8; ++r) {
                for (int t = 0; t < 8; ++t)
                    if (slice & (1u << t)) {
                        const int col = 8 * j + t;
                        bm[(size_t)(8 * i + r) * W + col / 64] |= (uint64_t)1 << (col % 64);
                    }
                slice = oracle_gf_mul(slice, 2);
            }
        }
        recovery[i]->row = erasures[i]; /* :791 */
    }

#define SUBROW(p) (recovery[(p) >> 3]->data + ((p)&7) * subbytes)
#define BIT(row, col) ((bm[(size_t)(row)*W + (col) / 64] >> ((col) % 64)) & 1)
    /* gaussian_elimination, :1020-1082 */
    for (int pivot = 0; pivot < R - 1; ++pivot) {
        for (int option = pivot; option < R; ++option) {
            if (!BIT(option, pivot)) continue;
            if (option != pivot) {
                swap_bytes(SUBROW(pivot), SUBROW(option), subbytes);
                for (int w = 0; w < W; ++w) {
                    uint64_t t = bm[(size_t)pivot * W + w];
                    bm[(size_t)pivot * W + w] = bm[(size_t)option * W + w];
                    bm[(size_t)option * W + w] = t;
                }
            }
            for (int other = option + 1; other < R; ++other) {
                if (!BIT(other, pivot)) continue;
                for (int w = 0; w < W; ++w) bm[(size_t)other * W + w] ^= bm[(size_t)pivot * W + w];
                xor_into(SUBROW(other), SUBROW(pivot), subbytes);
            }
            break;
        }
    }
    /* back_substitution, :1233-1252 */
    for (int pivot = R - 1; pivot > 0; --pivot)
        for (int other = pivot - 1; other >= 0; --other)
            if (BIT(other, pivot)) xor_into(SUBROW(other), SUBROW(pivot), subbytes);
#undef SUBROW
#undef BIT
    free(bm);
    free(C);
    return 0;
}

/* ----------------------------------------------------------- batch helpers */
typedef struct {
    int k, m, bb;
    long long g0, g1;
    const uint8_t *data;
    uint8_t *out;
    uint8_t *rows;
    int32_t *status;
    cauchy_encode_fn enc;
    cauchy_decode_fn dec;
    int rc;
} job_t;

static void *enc_worker(void *p)
{
    job_t *j = (job_t *)p;
    const unsigned char *ptrs[256];
    for (long long g = j->g0; g < j->g1; ++g) {
        const uint8_t *base = j->data + (size_t)g * j->k * j->bb;
        for (int x = 0; x < j->k && x < 256; ++x) ptrs[x] = base + (size_t)x * j->bb;
        int rc = j->enc(j->k, j->m, ptrs, j->out + (size_t)g * j->m * j->bb, j->bb);
        if (rc) j->rc = rc;
    }
    return NULL;
}

static void *dec_worker(void *p)
{
    job_t *j = (job_t *)p;
    OracleBlock blk[256];
    for (long long g = j->g0; g < j->g1; ++g) {
        uint8_t *base = j->out + (size_t)g * j->k * j->bb;
        uint8_t *rows = j->rows + (size_t)g * j->k;
        for (int x = 0; x < j->k && x < 256; ++x) {
            blk[x].data = base + (size_t)x * j->bb;
            blk[x].row = rows[x];
        }
        int rc = j->dec(j->k, j->m, blk, j->bb);
        for (int x = 0; x < j->k && x < 256; ++x) rows[x] = blk[x].row;
        if (j->status) j->status[g] = rc;
        if (rc) j->rc = rc;
    }
    return NULL;
}

static int run_jobs(job_t *proto, long long groups, int threads, void *(*fn)(void *))
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if (proto->k > 256) return -1;
    job_t jobs[256];
    pthread_t tid[256];
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = *proto;
        jobs[t].g0 = groups * t / threads;
        jobs[t].g1 = groups * (t + 1) / threads;
        jobs[t].rc = 0;
        if (threads == 1) fn(&jobs[t]);
        else pthread_create(&tid[t], NULL, fn, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) {
        if (threads > 1) pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}

static int oracle_decode_cb(int k, int m, OracleBlock *b, int bb) { return oracle_decode(k, m, b, bb); }

int oracle_run_encode_batch(cauchy_encode_fn fn, int k, int m, int bb, long long groups,
                            const uint8_t *data, uint8_t *parity, int threads)
{
    job_t p = {k, m, bb, 0, 0, data, parity, NULL, NULL, fn, NULL, 0};
    return run_jobs(&p, groups, threads, enc_worker);
}

int oracle_run_decode_batch(cauchy_decode_fn fn, int k, int m, int bb, long long groups,
                            uint8_t *blocks, uint8_t *rows, int32_t *status, int threads)
{
    job_t p = {k, m, bb, 0, 0, NULL, blocks, rows, status, NULL, fn, 0};
    return run_jobs(&p, groups, threads, dec_worker);
}

int oracle_encode_batch(int k, int m, int bb, long long groups, const uint8_t *data,
                        uint8_t *parity, int threads)
{
    return oracle_run_encode_batch(oracle_encode, k, m, bb, groups, data, parity, threads);
}

int oracle_decode_batch(int k, int m, int bb, long long groups, uint8_t *blocks,
                        uint8_t *rows, int32_t *status, int threads)
{
    return oracle_run_decode_batch(oracle_decode_cb, k, m, bb, groups, blocks, rows, status, threads);
}

/* ------------------------------------------------------- synthetic stream */
static inline uint64_t splitmix64_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_fill_stream(uint64_t seed, uint64_t byte_offset, uint8_t *out, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t b = byte_offset + i;
        const uint64_t w = splitmix64_mix(seed + (b / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        out[i] = (uint8_t)(w >> (8 * (b % 8)));
    }
}

double oracle_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
