// group_roundtrip.cpp — the QuicFecGroup C++ class (include/quic_fec_group.hpp) used the way
// the reference's creator and connection use net::QuicFecGroup: the sender adds k packets
// (UpdateSentList) and takes the m parity packets (getRedundancyPackets); the receiver gets
// the data packets but `lose`, then parity packets in order (UpdateReceivedList /
// UpdateFec) until CanRevive(), and revives the lost ones (getRevivedPackets).  Checks that
// each revived packet equals the lost one; prints "ok <revived>" and exits 0.
//   group_roundtrip <fec_configuration> <losses> <seed>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "quic_fec_group.hpp"

int main(int argc, char** argv) {
    const int conf = argc > 1 ? atoi(argv[1]) : QFEC_FEC_10_10;
    const int losses = argc > 2 ? atoi(argv[2]) : 3;
    const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 1;
    const size_t k = qfec::QuicFecGroup::k_from_conf(conf);
    const size_t m = qfec::QuicFecGroup::m_from_conf(conf);
    if (k == 0 || m == 0 || losses < 0 || (size_t)losses > std::min(k, m)) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    std::mt19937 rng(seed);
    const uint64_t first = 1000;
    const int pnlen = 1;   // PACKET_1BYTE_PACKET_NUMBER
    std::vector<std::string> sent(k);
    qfec::QuicFecGroup tx(first, conf);
    for (size_t i = 0; i < k; ++i) {
        sent[i].resize(1000 + rng() % 351);   // ragged payloads up to 1350 bytes
        for (auto& c : sent[i]) c = (char)(rng() & 0xff);
        if (!tx.UpdateSentList(0, first + i, pnlen, (const unsigned char*)sent[i].data(),
                               sent[i].size()))
            return fprintf(stderr, "UpdateSentList failed\n"), 1;
    }
    const auto parity = tx.getRedundancyPackets();
    if (tx.last_status() != 0 || parity.size() != m)
        return fprintf(stderr, "encode status %d, %zu parity packets\n", tx.last_status(),
                       parity.size()), 1;
    std::set<size_t> lost;
    while (lost.size() < (size_t)losses) lost.insert(rng() % k);
    qfec::QuicFecGroup rx(first, conf);
    for (size_t i = 0; i < k; ++i)
        if (!lost.count(i))
            rx.UpdateReceivedList(0, first + i, pnlen, (const unsigned char*)sent[i].data(),
                                  sent[i].size(), false);
    // the reference's list is parity m-1 .. 0 (sent back to front): deliver in packet order
    std::vector<const qfec::ParityPacket*> ps;
    for (const auto& p : parity) ps.push_back(&p);
    std::sort(ps.begin(), ps.end(), [](auto a, auto b) { return a->packet_number < b->packet_number; });
    for (const auto* p : ps) {
        if (rx.CanRevive()) break;
        rx.UpdateFec(0, p->packet_number, p->packet_number_len,
                     (const unsigned char*)p->packet_data.data(), p->packet_data.size());
    }
    if (!rx.CanRevive()) return fprintf(stderr, "cannot revive\n"), 1;
    const auto revived = rx.getRevivedPackets();
    if (rx.last_status() != 0 || revived.size() != lost.size())
        return fprintf(stderr, "decode status %d, %zu revived\n", rx.last_status(),
                       revived.size()), 1;
    for (const auto& r : revived) {
        const size_t i = (size_t)(r.packet_number - first);
        if (!lost.count(i) || r.packet_data != sent[i] || r.packet_number_len != pnlen)
            return fprintf(stderr, "revived packet %llu differs\n",
                           (unsigned long long)r.packet_number), 1;
    }
    printf("ok %zu\n", revived.size());
    return 0;
}
