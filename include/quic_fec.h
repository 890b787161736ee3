/*
 * quic_fec.h — C ABI of the MI355X-native FEC engine (libquic_fec.so).
 *
 * Drop-in boundary for the QuicR packet-group FEC path.  The reference calls the
 * Longhair codec through three extern "C" entry points
 * (/root/reference/net/quic/core/libcat/cauchy_256.h:47,78,103); this library exports
 * the same three symbols with identical semantics, executed by hand-written gfx950
 * kernels, plus batched device-pointer and host-pointer entry points that process
 * thousands of independent groups per launch.  Plain pointers and sizes only.
 *
 * Return codes (all entry points): 0 = OK; -1 = unsupported parameters, exactly where
 * the reference returns -1 (m > 1 and (k + m > 256 or block_bytes % 8 != 0));
 * <= -2 = errors the reference has no code for (bad arguments, GPU runtime failure;
 * see qfec_last_error()).
 */
#ifndef QUIC_AMD_QUIC_FEC_H
#define QUIC_AMD_QUIC_FEC_H

#ifdef __cplusplus
extern "C" {
#endif

#define CAUCHY_256_VERSION 2

#if defined(QFEC_BUILD)
#define QFEC_API __attribute__((visibility("default")))
#else
#define QFEC_API
#endif

/* Same layout as cauchy_256.h:52-55. */
typedef struct _Block {
    unsigned char *data;
    unsigned char row;
} Block;

/* ---------------------------------------------------------------------------------
 * Single-group drop-ins (host pointers; synchronous).
 * ------------------------------------------------------------------------------- */

/* Replaces _cauchy_256_init (cauchy_256.h:47, cauchy_256.cpp:389-398).  Returns 0 on
 * success and -1 on a version mismatch — what the reference code does (its header
 * comment says otherwise).  Also brings up the default GPU context. */
QFEC_API int _cauchy_256_init(int expected_version);
#ifndef cauchy_256_init
#define cauchy_256_init() _cauchy_256_init(CAUCHY_256_VERSION)
#endif

/* Replaces cauchy_256_encode (cauchy_256.h:78, cauchy_256.cpp:1502-1601): k data blocks
 * (pointer array) -> m recovery blocks stored end to end.  k <= 1 copies data[0] into
 * every output.  For m > 1 with k + m > 256 or block_bytes % 8 != 0 it writes the XOR
 * parity into the first recovery block and returns -1, like the reference. */
QFEC_API int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks,
                      int block_bytes);

/* Replaces cauchy_256_decode (cauchy_256.h:103, cauchy_256.cpp:1254-1413): in place.  The
 * i-th block (array order) tagged row >= k receives the i-th smallest missing data row:
 * its data is overwritten with that row's data and its row field rewritten. */
QFEC_API int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes);

/* ---------------------------------------------------------------------------------
 * Batched engine.  Layouts (row-major, bb = block_bytes):
 *   data   [G][k][bb]   parity [G][m][bb]
 *   blocks [G][k][bb]   rows   [G][k]  (u8 row tags, data 0..k-1, parity k..k+m-1)
 *   status [G]          per-group return code of the equivalent cauchy_256_decode call,
 *                       or -3 for a malformed receive set whose reference result is not
 *                       defined (a row tag >= k + m, the same recovery row twice, fewer
 *                       missing data rows than recovery blocks); such a group is left as
 *                       it was
 * `stream` is a hipStream_t (NULL = HIP's null stream, as everywhere in HIP).  Device
 * entry points only enqueue work on that stream; they do not synchronise.
 *
 * Streams and contexts: a context may be used from several streams.  Its eager decodes
 * share one workspace, so the library orders a decode behind the previous eager decode of
 * the same context when they are enqueued on different streams (an event, not a host
 * wait); calls on one stream are ordered by the stream.  Decodes captured into a HIP graph
 * use a second workspace of the context, so a graph replay, on whatever stream it is
 * launched, never races an eager call.  Graphs captured on one context share that second
 * workspace: replay them in one stream order (or capture on separate contexts), and capture
 * the calls of one context on one stream.  A capture allocates nothing when qfec_reserve
 * covered its batch; a workspace outgrown by a later capture stays allocated until the
 * context is destroyed, so earlier graphs stay valid.  Independent contexts (one per
 * stream, or one per device) share nothing and run concurrently.  Calls on one context are
 * serialised on the host by a mutex (the reference codec is single-threaded per
 * connection).
 * ------------------------------------------------------------------------------- */
typedef struct qfec_ctx qfec_ctx;

QFEC_API int qfec_ctx_create(int device, qfec_ctx **out);
QFEC_API void qfec_ctx_destroy(qfec_ctx *ctx);
/* Launch-shape options of one context (the defaults are the measured best):
 * "xor_slots" 2..4, "xor_waves" 1..4, "dma" 0/1, "stream" 0/1, "stream_ring" 4..36,
 * "stream_grid" 0.., "const_enc" 0/1, "stream_static" 0/1 (gf_ring encodes), "ring_wide" 0/1
 * (their wide parity stores), "dcol" 0/1, "dcol_grid" 0.., "dcol_depth" 6/8, "bsyn" 0/1,
 * "bsyn_depth" 3/5/7, "psyn" 0/1, "psyn_wide" 0..2 (wide recovered-block stores: none,
 * (10, 10), every code), "pd" 1..3, "flat" 0/1, "enc_rc" 2/4/8, "prep_lane" 0/1,
 * "host_chunk_mb" 1..4096, "host_min_groups" 1.., "ring_split" 0/1 ((10, 20) encode in two
 * units), and the grid shares "ring_wg", "bsyn_wg", "stream_wg" (-1 = the measured choice),
 * "psyn_wg", "dcol_wg", "xor_wg" (groups per wave of an oversubscribed grid; 0 = the resident
 * persistent grid).  get also reads "cus" (compute units of the device).  -2 for an unknown name or a value out of range (also for the measured-and-removed
 * variants of earlier versions).  No environment variable changes what the library launches. */
QFEC_API int qfec_ctx_set_option(qfec_ctx *ctx, const char *name, int value);
QFEC_API int qfec_ctx_get_option(qfec_ctx *ctx, const char *name, int *value);
/* Pre-size every per-(k, m) table and both decode workspaces (eager and graph) for up to
 * `groups` groups so that later calls allocate nothing (call it before capturing calls
 * into a HIP graph). */
QFEC_API int qfec_reserve(qfec_ctx *ctx, int k, int m, int block_bytes, long long groups);

QFEC_API int qfec_encode_batch(qfec_ctx *ctx, int k, int m, int block_bytes, long long groups,
                      const unsigned char *d_data, unsigned char *d_parity, void *stream);

/* d_out may equal d_blocks (in place, the reference semantics) or be a separate
 * [G][k][bb] buffer that receives only the recovered blocks.  d_rows_out may equal
 * d_rows_in.  d_status may be NULL. */
QFEC_API int qfec_decode_batch(qfec_ctx *ctx, int k, int m, int block_bytes, long long groups,
                      const unsigned char *d_blocks, const unsigned char *d_rows_in,
                      unsigned char *d_out, unsigned char *d_rows_out, int *d_status,
                      void *stream);

/* Receiver-side decode, recovered-blocks layout.  Same per-group decode as
 * qfec_decode_batch, but d_blocks and d_rows_in are left untouched and only the recovered
 * blocks are written, densely: with rmax = min(k, m), recovered block j of group g goes to
 * d_rec + (g * rmax + j) * block_bytes and the data row it restores to
 * d_rec_rows[g * rmax + j] -- ascending, the order cauchy_256_decode assigns them
 * (cauchy_256.cpp:570-574) -- and 255 past the group's erasure count (the d_rec bytes of
 * such entries are unspecified).  This is what QuicFecGroup::getRevivedPackets consumes
 * (quic_fec_group.cc:280-293).  d_status may be NULL. */
QFEC_API int qfec_decode_batch_recovered(qfec_ctx *ctx, int k, int m, int block_bytes,
                                long long groups, const unsigned char *d_blocks,
                                const unsigned char *d_rows_in, unsigned char *d_rec,
                                unsigned char *d_rec_rows, int *d_status, void *stream);

/* Host-pointer variants: H2D, kernels, D2H, chunked and pipelined; synchronous (pass
 * pinned memory for full PCIe speed).  qfec_decode_batch_host works in place on h_blocks /
 * h_rows like cauchy_256_decode; qfec_decode_batch_recovered_host returns only the
 * recovered blocks, as qfec_decode_batch_recovered does. */
QFEC_API int qfec_encode_batch_host(qfec_ctx *ctx, int k, int m, int block_bytes, long long groups,
                           const unsigned char *h_data, unsigned char *h_parity);
QFEC_API int qfec_decode_batch_host(qfec_ctx *ctx, int k, int m, int block_bytes, long long groups,
                           unsigned char *h_blocks, unsigned char *h_rows, int *h_status);
QFEC_API int qfec_decode_batch_recovered_host(qfec_ctx *ctx, int k, int m, int block_bytes,
                                     long long groups, const unsigned char *h_blocks,
                                     const unsigned char *h_rows, unsigned char *h_rec,
                                     unsigned char *h_rec_rows, int *h_status);

/* ---------------------------------------------------------------------------------
 * Packet protection next to the FEC path (SURVEY.md §8 f, rank 4).
 *
 * The reference encrypts every packet after serialisation -- the FEC packets right after
 * the encode (QuicPacketCreator::SerializeFec -> QuicFramer::EncryptInPlace,
 * quic_packet_creator.cc:948-953, quic_framer.cc:1921-1939) -- and decrypts before the
 * group sees a packet (quic_framer.cc:657).  In this fork QuicEncrypter::Create yields
 * NullEncrypter for kNULL and an identity copy for every negotiated AEAD
 * (crypto/quic_encrypter.cc:18-29), so NullEncrypter is the packet protection with
 * arithmetic: tag12 = low 12 bytes of FNV-1a-128(AD || PT) (null_encrypter.cc:23-43,
 * quic_utils.cc:38-56,110-125,175-181).
 *
 * Batches of n packets, all device pointers.  Per-packet lengths come from the int32 arrays,
 * or, where an array is NULL, from the `_all` scalar.  d_out and out_stride must be 4-byte
 * aligned.  d_out_len[i] = bytes written for packet i, or -1 where the reference returns
 * false.  A length larger than its row's stride is rejected (-1, nothing written); a stride
 * of 0 (every packet reads the same row) is not checked.
 * ------------------------------------------------------------------------------- */
/* NullEncrypter::EncryptPacket in the EncryptInPlace layout: packet i is
 * AD_i || tag12 || PT_i at d_out + i*out_stride (AD_i at d_ad + i*ad_stride, PT_i at
 * d_pt + i*pt_stride).  -1 (nothing written) when it does not fit in out_stride. */
QFEC_API int qfec_null_seal_batch(qfec_ctx *ctx, long long n, const unsigned char *d_ad,
                                  long long ad_stride, const int *d_ad_len, int ad_len_all,
                                  const unsigned char *d_pt, long long pt_stride,
                                  const int *d_pt_len, int pt_len_all, unsigned char *d_out,
                                  long long out_stride, int *d_out_len, void *stream);
/* NullDecrypter::DecryptPacket: wire packet i at d_pkt + i*pkt_stride (pkt_len bytes, the
 * first ad_len of them the associated data).  The output first receives the ciphertext, as
 * in the reference.  Accepted: the plaintext overwrites its start (the last 12 ciphertext
 * bytes stay behind it) and d_out_len[i] is the plaintext length.  Rejected (ciphertext
 * shorter than 12 bytes or tag mismatch): -1, the output holds the ciphertext copy; -1 with
 * nothing written when the ciphertext exceeds out_stride. */
QFEC_API int qfec_null_open_batch(qfec_ctx *ctx, long long n, const unsigned char *d_pkt,
                                  long long pkt_stride, const int *d_pkt_len, int pkt_len_all,
                                  const int *d_ad_len, int ad_len_all, unsigned char *d_out,
                                  long long out_stride, int *d_out_len, void *stream);
/* Sender side of SerializeFec (quic_packet_creator.cc:935-957): encode the groups into
 * d_parity [G][m][bb] (qfec_encode_batch), then seal parity block (g, i) as FEC packet
 * g*m + i with header g*m + i (d_hdr + (g*m+i)*hdr_stride) as the associated data:
 * d_pkt + (g*m+i)*pkt_stride = header || tag12 || parity.  One call, two launches on one
 * stream; the parity does not leave the device. */
QFEC_API int qfec_encode_seal_batch(qfec_ctx *ctx, int k, int m, int block_bytes,
                                    long long groups, const unsigned char *d_data,
                                    unsigned char *d_parity, const unsigned char *d_hdr,
                                    long long hdr_stride, const int *d_hdr_len, int hdr_len_all,
                                    unsigned char *d_pkt, long long pkt_stride, int *d_pkt_len,
                                    void *stream);

/* Every packet of each group in one launch: the reference seals each data packet
 * (quic_packet_creator.cc:733-736) as well as each FEC packet (:948-953).  Packet
 * p = g*(k+m) + i is sealed with header row p (d_hdr + p*hdr_stride, d_hdr_len[p] or
 * hdr_len_all bytes) as the associated data and, as plaintext, data block (g, i) of d_data
 * [G][k][bb] for i < k or parity block (g, i-k) of d_parity [G][m][bb] otherwise, its first
 * d_pt_len[p] (or pt_len_all <= bb) bytes: d_pkt + p*pkt_stride = header || tag12 || PT,
 * d_pkt_len[p] as in qfec_null_seal_batch.  k + m <= 256. */
QFEC_API int qfec_seal_groups_batch(qfec_ctx *ctx, int k, int m, int block_bytes,
                                    long long groups, const unsigned char *d_data,
                                    const unsigned char *d_parity, const unsigned char *d_hdr,
                                    long long hdr_stride, const int *d_hdr_len, int hdr_len_all,
                                    const int *d_pt_len, int pt_len_all, unsigned char *d_pkt,
                                    long long pkt_stride, int *d_pkt_len, void *stream);
/* qfec_encode_batch into d_parity, then qfec_seal_groups_batch: one call, two launches. */
QFEC_API int qfec_encode_seal_groups_batch(qfec_ctx *ctx, int k, int m, int block_bytes,
                                           long long groups, const unsigned char *d_data,
                                           unsigned char *d_parity, const unsigned char *d_hdr,
                                           long long hdr_stride, const int *d_hdr_len,
                                           int hdr_len_all, const int *d_pt_len, int pt_len_all,
                                           unsigned char *d_pkt, long long pkt_stride,
                                           int *d_pkt_len, void *stream);
/* Receiver side: NullDecrypter::DecryptPacket on every packet of each group (the framer
 * decrypts before the group sees a packet, quic_framer.cc:657), then the group decode.
 * Wire packet p = g*(k+m) + i at d_pkt + p*pkt_stride, d_pkt_len[p] bytes (< 0: not
 * received), the first d_ad_len[p] (or ad_len_all) of them the associated data.
 *   d_open_len [G][k+m]  plaintext bytes of packet p, or -1 (not received, malformed,
 *                        plaintext longer than bb, or tag mismatch)
 *   d_blocks [G][k][bb]  data packet i's plaintext, zero-padded, in slot i; each slot whose
 *                        data packet did not open holds the plaintext of the next opened FEC
 *                        packet (ascending)
 *   d_rows [G][k]        the row tag of each slot (i, or k + j for FEC packet j; 255 when no
 *                        opened FEC packet is left, and the group's status is then -3; the
 *                        bytes of a slot tagged 255 are unspecified)
 * followed by qfec_decode_batch_recovered(d_blocks, d_rows) into d_rec / d_rec_rows /
 * d_status (a group with an unfilled slot: status -3, recovered rows all 255).  Four
 * launches on one stream.  k + m <= 255. */
QFEC_API int qfec_open_decode_batch(qfec_ctx *ctx, int k, int m, int block_bytes,
                                    long long groups, const unsigned char *d_pkt,
                                    long long pkt_stride, const int *d_pkt_len,
                                    const int *d_ad_len, int ad_len_all, unsigned char *d_blocks,
                                    unsigned char *d_rows, int *d_open_len, unsigned char *d_rec,
                                    unsigned char *d_rec_rows, int *d_status, void *stream);

/* Host-pointer variants of the two protected paths: the sender's and the receiver's per-packet
 * work starting and ending in host memory (packets off and onto a socket), chunked and
 * pipelined like qfec_*_batch_host (H2D, kernels and D2H of successive chunks overlap);
 * synchronous; pass pinned memory for full PCIe speed.  Lengths, headers and packets are
 * indexed by packet p = g*(k+m) + i as in the device calls; h_hdr may be NULL (no associated
 * data: h_hdr_len NULL and hdr_len_all 0); h_pkt_len, h_pt_len and h_ad_len are int32 host
 * arrays (NULL where the `_all` scalar applies, except h_pkt_len).  Row strides must be > 0.
 *   qfec_encode_seal_groups_batch_host: data [G][k][bb] -> every packet of each group sealed,
 *     h_pkt [G*(k+m)][pkt_stride], h_pkt_len [G*(k+m)] (qfec_encode_seal_groups_batch); the
 *     bytes of a packet row past h_pkt_len[p] are zero (rows are copied back whole); -1 with
 *     nothing written where the encode returns -1 (m > 1, k > 1 and (k + m > 256 or
 *     block_bytes % 8 != 0));
 *   qfec_open_decode_batch_host: wire packets -> h_rec [G][min(k,m)][bb], h_rec_rows,
 *     h_status [G] (may be NULL) and h_open_len [G*(k+m)] (may be NULL)
 *     (qfec_open_decode_batch). */
QFEC_API int qfec_encode_seal_groups_batch_host(qfec_ctx *ctx, int k, int m, int block_bytes,
                                                long long groups, const unsigned char *h_data,
                                                const unsigned char *h_hdr, long long hdr_stride,
                                                const int *h_hdr_len, int hdr_len_all,
                                                const int *h_pt_len, int pt_len_all,
                                                unsigned char *h_pkt, long long pkt_stride,
                                                int *h_pkt_len);
QFEC_API int qfec_open_decode_batch_host(qfec_ctx *ctx, int k, int m, int block_bytes,
                                         long long groups, const unsigned char *h_pkt,
                                         long long pkt_stride, const int *h_pkt_len,
                                         const int *h_ad_len, int ad_len_all,
                                         unsigned char *h_rec, unsigned char *h_rec_rows,
                                         int *h_status, int *h_open_len);

/* ---------------------------------------------------------------------------------
 * Support: the coefficient tables, a seeded synthetic workload, diagnostics.
 * ------------------------------------------------------------------------------- */
/* Rows 1..m-1 of the Cauchy matrix the reference selects (cauchy_256.cpp:422-480),
 * (m-1) x k bytes, row-major.  Host only.  Returns -1 if m < 2 or k + m > 256. */
QFEC_API int qfec_cauchy_matrix(int k, int m, unsigned char *out);

/* Fill d_dst with bytes [byte_offset, byte_offset + bytes) of the splitmix64 stream
 * (byte_offset % 8 == 0); see quic_amd/synth.py for the definition. */
QFEC_API int qfec_synth_fill(void *d_dst, unsigned long long bytes, unsigned long long seed,
                    unsigned long long byte_offset, void *stream);
/* blocks[g][i] = (src[g][i] < k ? data[g][src] : parity[g][src - k]); src is int16 [G][k]. */
QFEC_API int qfec_synth_gather(const unsigned char *d_data, const unsigned char *d_parity,
                      const short *d_src, unsigned char *d_blocks, int k, int m,
                      int block_bytes, long long groups, void *stream);

QFEC_API const char *qfec_last_error(void);
/* Names of the kernels this thread's last engine call launched, " + "-separated, e.g.
 * "decode_prep_lane_kernel + gf_stream_kernel<decode>" (bench.py reports it). */
QFEC_API const char *qfec_last_kernels(void);
/* Grids of the persistent kernels the last call on this thread launched, as space-separated
 * "kernel=workgroups" entries (e.g. "gf_psyn_kernel=1024"); diagnostics and tests. */
QFEC_API const char *qfec_last_grids(void);
/* Measurement hook (bench.py's roofline timing).  While set, every engine call on this
 * thread records start_event (a hipEvent_t) at the start of its first kernel and
 * stop_event at the end of its last, through hipExtLaunchKernel, so the pair brackets the
 * call's kernels only.  Pass NULL, NULL to stop.  Returns -2 if only one is NULL. */
QFEC_API int qfec_set_timing_events(void *start_event, void *stop_event);
QFEC_API int qfec_version(void);

#ifdef __cplusplus
}
#endif
#endif /* QUIC_AMD_QUIC_FEC_H */
