// quic_fec_group.hpp — QuicFecGroup as a C++ class with the reference's method names
// (/root/reference/net/quic/core/quic_fec_group.h:34-79), header-only over the C ABI of
// quic_fec_group.h (libquic_fec.so).  A caller of the reference class
// (quic_packet_creator.cc:929-990 on the sender, quic_connection.cc:2472-2523 on the
// receiver) swaps `net::QuicFecGroup` for `qfec::QuicFecGroup` and passes the header fields
// it already reads (packet number, packet number length) and the payload as pointer + size
// instead of QuicPacketHeader / StringPiece; the rest reads the same:
//
//   reference                                         here
//   QuicFecGroup(n, conf)                              QuicFecGroup(n, conf)
//   UpdateSentList(level, header, payload)             UpdateSentList(level, pn, pnlen, p, len)
//   UpdateReceivedList(level, header, payload, fec)    UpdateReceivedList(level, pn, pnlen, p, len, fec)
//   UpdateFec(level, header, redundancy)               UpdateFec(level, pn, pnlen, p, len)
//   CanRevive, IsWaitingForPacketBefore, NumReceivedPackets, NumSentPackets,
//   EffectiveEncryptionLevel, FecGroupNumber, GroupTotalSize, GroupReduntancySize,
//   m_from_conf / k_from_conf                          the same
//   std::list<ParityPacket*> getRedundancyPackets()    std::list<ParityPacket> (by value)
//   std::list<ParityPacket*> getRevivedPackets()       std::list<ParityPacket> (by value)
//
// Differences are the C ABI's (quic_fec_group.h): the codec is always called and its status
// is kept (last_status()), and packets are returned by value (the reference leaks them).
// IsFinished, Revive and PayloadParity are declared by the reference but never defined
// (quic_fec_group.cc has no body for them), so no caller can use them; they are not here.
#ifndef QUIC_AMD_QUIC_FEC_GROUP_HPP
#define QUIC_AMD_QUIC_FEC_GROUP_HPP

#include <cstddef>
#include <cstdint>
#include <list>
#include <string>

#include "quic_fec_group.h"

namespace qfec {

// ParityPacket (quic_fec_group.h:25-33): a parity packet to send, or a revived data packet.
struct ParityPacket {
    uint64_t packet_number;
    std::string packet_data;
    int packet_number_len;   // QuicPacketNumberLength
    ParityPacket(uint64_t pn, std::string data, int pnlen)
        : packet_number(pn), packet_data(std::move(data)), packet_number_len(pnlen) {}
};

class QuicFecGroup {
   public:
    explicit QuicFecGroup(uint64_t fec_group_number, int fec_configuration)
        : fec_configuration(fec_configuration),
          g_(qfec_group_new(fec_group_number, fec_configuration)) {}
    ~QuicFecGroup() { qfec_group_free(g_); }
    QuicFecGroup(const QuicFecGroup&) = delete;             // DISALLOW_COPY_AND_ASSIGN
    QuicFecGroup& operator=(const QuicFecGroup&) = delete;

    int fec_configuration;   // FecConfiguration (public, as in the reference)
    static size_t m_from_conf(int conf) { return qfec_m_from_conf(conf); }
    static size_t k_from_conf(int conf) { return qfec_k_from_conf(conf); }

    bool UpdateReceivedList(int encryption_level, uint64_t packet_number, int packet_number_len,
                            const unsigned char* payload, size_t len, bool is_fec_data) {
        return qfec_group_update_received(g_, encryption_level, packet_number,
                                          packet_number_len, payload, len, is_fec_data) != 0;
    }
    bool UpdateSentList(int encryption_level, uint64_t packet_number, int packet_number_len,
                        const unsigned char* payload, size_t len) {
        return qfec_group_update_sent(g_, encryption_level, packet_number, packet_number_len,
                                      payload, len) != 0;
    }
    bool UpdateFec(int encryption_level, uint64_t packet_number, int packet_number_len,
                   const unsigned char* redundancy, size_t len) {
        return qfec_group_update_fec(g_, encryption_level, packet_number, packet_number_len,
                                     redundancy, len) != 0;
    }
    bool CanRevive() const { return qfec_group_can_revive(g_) != 0; }
    bool IsWaitingForPacketBefore(uint64_t num) const {
        return qfec_group_is_waiting_for_packet_before(g_, num) != 0;
    }
    size_t NumReceivedPackets() const { return qfec_group_num_received(g_); }
    size_t NumSentPackets() const { return qfec_group_num_sent(g_); }
    int EffectiveEncryptionLevel() const { return qfec_group_effective_encryption_level(g_); }
    uint64_t FecGroupNumber() const { return qfec_group_number(g_); }
    size_t GroupTotalSize() const { return qfec_group_total_size(g_); }
    size_t GroupReduntancySize() const { return qfec_group_redundancy_size(g_); }

    // getRedundancyPackets (quic_fec_group.cc:338-389): the m parity packets, in the
    // reference's list order
    std::list<ParityPacket> getRedundancyPackets() { return take(qfec_group_redundancy(g_, &st_)); }
    // getRevivedPackets (quic_fec_group.cc:234-297): the missing data packets
    std::list<ParityPacket> getRevivedPackets() { return take(qfec_group_revived(g_, &st_)); }
    // the codec's return code of the last get*Packets call (the reference asserts it is 0)
    int last_status() const { return st_; }
    // the C handle, for the batching front end (qfec_batch_add_encode / _decode)
    qfec_group* handle() { return g_; }

   private:
    static std::list<ParityPacket> take(qfec_packets* l) {
        std::list<ParityPacket> out;
        if (!l) return out;
        for (size_t i = 0, n = qfec_packets_count(l); i < n; ++i) {
            unsigned long long pn = 0;
            const unsigned char* d = nullptr;
            size_t len = 0;
            int pnlen = 0;
            if (qfec_packets_get(l, i, &pn, &d, &len, &pnlen) == 0)
                out.emplace_back(pn, std::string((const char*)d, len), pnlen);
        }
        qfec_packets_free(l);
        return out;
    }
    qfec_group* g_;
    int st_ = 0;
};

}  // namespace qfec

#endif  // QUIC_AMD_QUIC_FEC_GROUP_HPP
