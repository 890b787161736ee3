// fec_wire.cpp — the QuicR FEC wire format: private-flags byte, FEC group offset and the
// FEC packet body (include/quic_fec_group.h).  Host byte work, no GPU.
//
// Reference: AppendPacketHeader's private part (net/quic/core/quic_framer.cc:850-893),
// ProcessAuthenticatedHeader (:1219-1256), BuildFecPacket (:469-494), GetPacketHeaderSize
// (quic_protocol.cc:74-88), flag bits QuicPacketPrivateFlags (quic_protocol.h:411-427).
#include <cstring>

#include "../../include/quic_fec_group.h"

namespace {

constexpr unsigned kFlagEntropy = 1u << 0;    // PACKET_PRIVATE_FLAGS_ENTROPY
constexpr unsigned kFlagFecGroup = 1u << 1;   // PACKET_PRIVATE_FLAGS_FEC_GROUP
constexpr unsigned kFlagFec = 1u << 2;        // PACKET_PRIVATE_FLAGS_FEC
constexpr unsigned kFlagFecConfig = 0x1fu << 3;
constexpr int kQuicVersion33 = 33;

}  // namespace

extern "C" {

QFEC_API int qfec_wire_write_private(const qfec_private_header *h, int quic_version,
                                     unsigned char *out, size_t cap) {
    if (!h || (!out && cap)) return -2;
    uint8_t flags = 0;
    if (h->entropy_flag) flags |= kFlagEntropy;
    if (h->in_fec_group) {
        flags |= kFlagFecGroup;
        flags |= (uint8_t)(h->fec_configuration << 3);   // as the reference: no mask
    }
    if (h->fec_flag) flags |= kFlagFec;
    size_t n = 1;
    uint8_t offset = 0;
    if (h->in_fec_group) {
        // DCHECK_LE(fec_group, packet_number); DCHECK_LT(packet_number - fec_group, 255)
        if (h->fec_group > h->packet_number || h->packet_number - h->fec_group >= 255) return -1;
        offset = (uint8_t)(h->packet_number - h->fec_group);
        ++n;
    }
    if (quic_version <= kQuicVersion33) ++n;   // flags written again (:885-891)
    if (cap < n) return -2;
    size_t i = 0;
    out[i++] = flags;
    if (h->in_fec_group) out[i++] = offset;
    if (quic_version <= kQuicVersion33) out[i++] = flags;
    return (int)i;
}

QFEC_API int qfec_wire_read_private(const unsigned char *in, size_t len,
                                    qfec_private_header *h) {
    if (!h) return -1;
    if (!in || len < 1) return -1;                   // "Unable to read private flags."
    const uint8_t flags = in[0];
    h->entropy_flag = (flags & kFlagEntropy) != 0;
    h->fec_flag = (flags & kFlagFec) != 0;
    h->in_fec_group = 0;
    h->fec_group = 0;
    h->fec_configuration = 0;
    if (!(flags & kFlagFecGroup)) return 1;
    if (len < 2) return -2;     // "Unable to read first fec protected packet offset."
    const uint8_t offset = in[1];
    if (offset >= h->packet_number) return -3;   // offset must be < the packet number
    h->in_fec_group = 1;
    h->fec_group = h->packet_number - offset;
    h->fec_configuration = (int)((flags & kFlagFecConfig) >> 3);
    return 2;
}

QFEC_API size_t qfec_wire_header_size(int connection_id_length, int include_version,
                                      int include_path_id, int include_nonce,
                                      int packet_number_length, int in_fec_group) {
    return 1 /* public flags */ + (size_t)connection_id_length + (include_version ? 4 : 0) +
           (include_path_id ? 1 : 0) + (size_t)packet_number_length +
           (include_nonce ? 32 : 0) + (in_fec_group ? 1 : 0) + 1 /* private flags */;
}

QFEC_API long qfec_wire_fec_packet(const unsigned char *header, size_t header_len,
                                   const unsigned char *redundancy, size_t redundancy_len,
                                   unsigned char *out, size_t cap) {
    const size_t n = header_len + redundancy_len;
    if (cap < n || (!out && n)) return -2;
    if (header_len) std::memcpy(out, header, header_len);
    if (redundancy_len) std::memcpy(out + header_len, redundancy, redundancy_len);
    return (long)n;
}

}  // extern "C"
