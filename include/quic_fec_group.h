/*
 * quic_fec_group.h — packet-group FEC state (sender + receiver) over the GPU codec.
 *
 * C++ counterpart of QuicFecGroup (/root/reference/net/quic/core/quic_fec_group.h:22-109,
 * quic_fec_group.cc) with the same method names and wire-visible behaviour:
 *   - 2-byte little-endian prefix  len | (packet_number_length << 14)  truncated to 16 bits
 *     (quic_fec_group.cc:109-121; 4-byte packet numbers read back as 0, 6-byte as 2);
 *   - zero padding to block_bytes = max(len + 2) rounded up to a multiple of 8 (:344-352);
 *   - parity packet i numbered min + k + i, returned in the reference's list order
 *     (i = m-1 .. 0; the creator sends the list back to front, :382-386);
 *   - the receiver decodes the FIRST k packets in arrival order (:259-274) and extracts
 *     each missing data packet from its prefix (:280-293).
 * Differences, on purpose: the codec is always called (the
 * reference calls it inside assert(), compiled out under NDEBUG) and its return code is
 * reported; packets are returned by value (no leaks).
 *
 * Plus a C ABI (qfec_group_*) for bindings, and a batching front end (qfec_batch_*) that
 * aggregates many groups into one batched GPU launch.
 */
#ifndef QUIC_AMD_QUIC_FEC_GROUP_H
#define QUIC_AMD_QUIC_FEC_GROUP_H

#include <stddef.h>
#include <stdint.h>

#include "quic_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* FecConfiguration (quic_protocol.h:65-73). */
enum { QFEC_FEC_OFF = 0, QFEC_FEC_5_5, QFEC_FEC_10_10, QFEC_FEC_10_15, QFEC_FEC_10_20,
       QFEC_FEC_15_15, QFEC_FEC_250_5 };

/* kDefaultMaxPacketsPerFecGroup (k) / kDefaultRecoveryBlocksCount (m) overrides
 * (quic_protocol.cc:23-24); 0 = use the preset table.  Note the reference CLI maps
 * --m to k and --k to m (quic_protocol.cc:35). */
QFEC_API void qfec_set_fec_overrides(size_t max_packets_per_group_k, size_t recovery_blocks_m);
QFEC_API size_t qfec_k_from_conf(int fec_configuration);   /* quic_fec_group.cc:22-50 */
QFEC_API size_t qfec_m_from_conf(int fec_configuration);   /* quic_fec_group.cc:52-82 */

/* The prefixed block of one data packet (quic_fec_group.cc:109-121): writes len + 2
 * bytes to out; returns len + 2, or -1 if len > 0x3fff. */
QFEC_API long qfec_prefix_payload(const unsigned char *payload, size_t len, int packet_number_len,
                                  unsigned char *out);
/* block_bytes for a group whose largest prefixed packet is max_len bytes (:344-352). */
QFEC_API int qfec_block_bytes(size_t max_prefixed_len);

typedef struct qfec_group qfec_group;
typedef struct qfec_packets qfec_packets;

QFEC_API qfec_group *qfec_group_new(unsigned long long fec_group_number, int fec_configuration);
/* Same, with an explicit codec of the cauchy_256 ABI (NULL, NULL = the GPU drop-ins).  Used
 * by the loopback tool to run the reference CPU codec beside the GPU path. */
typedef int (*qfec_encode_fn)(int, int, const unsigned char **, void *, int);
typedef int (*qfec_decode_fn)(int, int, Block *, int);
QFEC_API qfec_group *qfec_group_new_with_codec(unsigned long long fec_group_number,
                                               int fec_configuration, qfec_encode_fn enc,
                                               qfec_decode_fn dec);
QFEC_API void qfec_group_free(qfec_group *g);
QFEC_API int qfec_group_update_sent(qfec_group *g, int encryption_level, unsigned long long pn,
                                    int packet_number_len, const unsigned char *payload, size_t len);
QFEC_API int qfec_group_update_received(qfec_group *g, int encryption_level,
                                        unsigned long long pn, int packet_number_len,
                                        const unsigned char *payload, size_t len, int is_fec_data);
QFEC_API int qfec_group_update_fec(qfec_group *g, int encryption_level, unsigned long long pn,
                                   int packet_number_len, const unsigned char *redundancy,
                                   size_t len);
QFEC_API int qfec_group_can_revive(const qfec_group *g);
QFEC_API int qfec_group_is_waiting_for_packet_before(const qfec_group *g, unsigned long long num);
QFEC_API size_t qfec_group_num_received(const qfec_group *g);
QFEC_API size_t qfec_group_num_sent(const qfec_group *g);
QFEC_API int qfec_group_effective_encryption_level(const qfec_group *g);
QFEC_API unsigned long long qfec_group_number(const qfec_group *g);
QFEC_API size_t qfec_group_total_size(const qfec_group *g);        /* k + m */
QFEC_API size_t qfec_group_redundancy_size(const qfec_group *g);   /* m */
/* getRedundancyPackets / getRevivedPackets; *status = the codec's return code. */
QFEC_API qfec_packets *qfec_group_redundancy(qfec_group *g, int *status);
QFEC_API qfec_packets *qfec_group_revived(qfec_group *g, int *status);

QFEC_API size_t qfec_packets_count(const qfec_packets *l);
QFEC_API int qfec_packets_get(const qfec_packets *l, size_t i, unsigned long long *pn,
                              const unsigned char **data, size_t *len, int *packet_number_len);
QFEC_API void qfec_packets_free(qfec_packets *l);

/* ---------------------------------------------------------------------------------
 * Batching front end: sender groups that reached k packets are queued; a flush runs
 * ONE batched GPU encode per (k, m, block_bytes) bucket and stores the parity packets
 * back into each group, whose qfec_group_redundancy() then returns them without a
 * codec call.  Receiver groups that CanRevive() are queued the same way for decode.
 * Flush policy: when a bucket holds max_groups groups, or on qfec_batch_poll() once the
 * oldest queued group is older than max_delay_us, or on an explicit qfec_batch_flush().
 * ------------------------------------------------------------------------------- */
typedef struct qfec_batch qfec_batch;
QFEC_API qfec_batch *qfec_batch_new(qfec_ctx *ctx, size_t max_groups, unsigned max_delay_us);
QFEC_API void qfec_batch_free(qfec_batch *b);
QFEC_API int qfec_batch_add_encode(qfec_batch *b, qfec_group *g);   /* group must stay alive */
QFEC_API int qfec_batch_add_decode(qfec_batch *b, qfec_group *g);
QFEC_API int qfec_batch_poll(qfec_batch *b);    /* flushes if the timeout expired; >= 0 = groups done */
QFEC_API int qfec_batch_flush(qfec_batch *b);   /* >= 0 = groups processed */
QFEC_API size_t qfec_batch_pending(const qfec_batch *b);

/* ---- QuicR FEC wire format (the private part of the packet header + the FEC packet) ----
 * What the framer adds to a QUIC packet for FEC (quic_framer.cc:850-893 write,
 * :1219-1256 parse, :469-494 BuildFecPacket; flag bits quic_protocol.h:411-427):
 *   private flags byte  bit 0 entropy, bit 1 FEC_GROUP, bit 2 FEC (payload is parity),
 *                       bits 3..7 FecConfiguration (written as config << 3 into a byte)
 *   FEC group offset    1 byte, packet_number - fec_group, only when FEC_GROUP is set
 *   FEC packet          header bytes followed by the block_bytes parity block
 * The public header before it (flags, connection id, version, nonce, packet number) is
 * the QUIC stack's and out of scope; its size enters through qfec_wire_header_size. */
typedef struct qfec_private_header {
    unsigned long long packet_number;   /* write: this packet; read: from the public header */
    unsigned long long fec_group;       /* first FEC-protected packet number (0 = none) */
    int entropy_flag;
    int fec_flag;                       /* payload is FEC redundancy */
    int in_fec_group;
    int fec_configuration;              /* FecConfiguration */
} qfec_private_header;

/* AppendPacketHeader's private part.  QUIC versions <= 33 write the flags byte a second
 * time after the offset (quic_framer.cc:885-891, kept: the wire is the wire).  Returns the
 * bytes written; -1 if in a group with fec_group > packet_number or an offset >= 255 (the
 * reference's DCHECKs, :873-874); -2 if cap is too small. */
QFEC_API int qfec_wire_write_private(const qfec_private_header *h, int quic_version,
                                     unsigned char *out, size_t cap);
/* ProcessAuthenticatedHeader.  h->packet_number must hold the packet number from the
 * public header; the other fields are filled (0 when not in a group).  Returns the bytes
 * consumed; -1 "Unable to read private flags", -2 "Unable to read first fec protected
 * packet offset", -3 "First fec protected packet offset must be less than the packet
 * number" (QUIC_INVALID_PACKET_HEADER in the reference). */
QFEC_API int qfec_wire_read_private(const unsigned char *in, size_t len,
                                    qfec_private_header *h);
/* GetPacketHeaderSize (quic_protocol.cc:74-88): public flags + connection id + version
 * (4) + path id (1) + packet number + diversification nonce (32) + FEC group offset (1,
 * in a group) + private flags (1).  Also GetStartOfFecProtectedData with in_fec_group = 1. */
QFEC_API size_t qfec_wire_header_size(int connection_id_length, int include_version,
                                      int include_path_id, int include_nonce,
                                      int packet_number_length, int in_fec_group);
/* BuildFecPacket's body: header bytes then the redundancy block.  Returns the packet
 * length, or -2 if cap is too small. */
QFEC_API long qfec_wire_fec_packet(const unsigned char *header, size_t header_len,
                                   const unsigned char *redundancy, size_t redundancy_len,
                                   unsigned char *out, size_t cap);

#ifdef __cplusplus
}
#endif

#endif /* QUIC_AMD_QUIC_FEC_GROUP_H */
