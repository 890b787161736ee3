// fec_group.cpp — QuicFecGroup counterpart (sender + receiver framing) and the batching
// front end, host C++ over the GPU codec.  See include/quic_fec_group.h for the contract
// and the reference lines each piece follows (net/quic/core/quic_fec_group.cc).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <list>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/quic_fec_group.h"

namespace qfec {

static size_t g_override_k = 0;   // kDefaultMaxPacketsPerFecGroup
static size_t g_override_m = 0;   // kDefaultRecoveryBlocksCount

constexpr int kPacket1BytePn = 1;   // PACKET_1BYTE_PACKET_NUMBER (quic_protocol.h:342)
constexpr int kNumEncryptionLevels = 3;

struct ParityPacket {
    uint64_t packet_number;
    std::string packet_data;
    int packet_number_len;
};

size_t k_from_conf(int conf) {   // quic_fec_group.cc:22-50
    if (g_override_k != 0) return g_override_k;
    switch (conf) {
        case QFEC_FEC_5_5: return 5;
        case QFEC_FEC_10_10: case QFEC_FEC_10_15: case QFEC_FEC_10_20: return 10;
        case QFEC_FEC_15_15: return 15;
        case QFEC_FEC_250_5: return 250;
        default: return 0;   // FEC_OFF / unknown
    }
}

size_t m_from_conf(int conf) {   // quic_fec_group.cc:52-82
    if (g_override_m != 0) return g_override_m;
    switch (conf) {
        case QFEC_FEC_5_5: case QFEC_FEC_250_5: return 5;
        case QFEC_FEC_10_10: return 10;
        case QFEC_FEC_15_15: case QFEC_FEC_10_15: return 15;
        case QFEC_FEC_10_20: return 20;
        default: return 0;
    }
}

// appendLenToPayload (quic_fec_group.cc:109-121): u16 LE  len | (pnlen << 14), truncated.
static std::string prefixed(const unsigned char* p, size_t len, int pnlen) {
    const uint16_t ext = (uint16_t)((unsigned)len | ((unsigned)pnlen << 14));
    std::string s(len + 2, '\0');
    s[0] = (char)(ext & 0xff);
    s[1] = (char)(ext >> 8);
    if (len) memcpy(&s[2], p, len);
    return s;
}

static int round8(size_t n) { return (int)((n + 7) & ~(size_t)7); }

class QuicFecGroup {
   public:
    QuicFecGroup(uint64_t fec_group_number, int conf, qfec_encode_fn enc = nullptr,
                 qfec_decode_fn dec = nullptr)
        : fec_configuration(conf), min_(fec_group_number), eff_level_(kNumEncryptionLevels),
          enc_(enc ? enc : cauchy_256_encode), dec_(dec ? dec : cauchy_256_decode) {
        k_ = k_from_conf(conf);
        m_ = m_from_conf(conf);
        max_ = fec_group_number - 1 + k_;   // :93-94
    }

    size_t k() const { return k_; }
    size_t m() const { return m_; }

    // :125-146
    bool UpdateSentList(int, uint64_t pn, int pnlen, const unsigned char* p, size_t len) {
        sent_.push_back(ParityPacket{pn, prefixed(p, len, pnlen), pnlen});
        return true;
    }

    // :150-196
    bool UpdateReceivedList(int level, uint64_t pn, int pnlen, const unsigned char* p,
                            size_t len, bool is_fec) {
        if (received_set_.count(pn)) return false;
        if (pn < min_) return false;
        std::string data = is_fec ? std::string((const char*)p, len) : prefixed(p, len, pnlen);
        received_.push_back(ParityPacket{pn, std::move(data), pnlen});
        received_set_.insert(pn);
        if (level < eff_level_) eff_level_ = level;
        return true;
    }

    // :199-208
    bool UpdateFec(int level, uint64_t pn, int pnlen, const unsigned char* p, size_t len) {
        if (level < eff_level_) eff_level_ = level;
        return UpdateReceivedList(level, pn, pnlen, p, len, true);
    }

    bool CanRevive() const { return received_set_.size() >= k_; }   // :210-213

    // :300-325
    bool IsWaitingForPacketBefore(uint64_t num) const {
        if (min_ >= num) return false;
        if (received_set_.empty() ? min_ < num : *received_set_.rbegin() + 1 < num) return true;
        uint64_t target = min_;
        for (uint64_t pn : received_set_) {
            if (target++ != pn) return true;
            if (target >= num) return false;
        }
        return false;
    }

    size_t NumReceivedPackets() const { return received_set_.size(); }
    size_t NumSentPackets() const { return sent_.size(); }
    int EffectiveEncryptionLevel() const { return eff_level_; }
    uint64_t FecGroupNumber() const { return min_; }
    size_t GroupTotalSize() const { return k_ + m_; }
    size_t GroupReduntancySize() const { return m_; }

    // ------------------------------------------------------------------- sender side
    // Blocks the codec sees (:344-368): k prefixed packets zero-padded to block_bytes.
    bool EncodeInput(int* bb, std::vector<unsigned char>* blocks) const {
        if (sent_.size() != k_ || k_ == 0) return false;   // :354 (an assert there)
        size_t mx = 0;
        for (auto& s : sent_) mx = std::max(mx, s.packet_data.size());
        *bb = round8(mx);
        blocks->assign((size_t)k_ * *bb, 0);
        for (size_t i = 0; i < k_; ++i)
            memcpy(blocks->data() + i * *bb, sent_[i].packet_data.data(),
                   sent_[i].packet_data.size());
        return true;
    }

    // Parity packets from the recovery blocks (:380-386): list order m-1 .. 0.
    void SetRedundancy(const unsigned char* rec, int bb, int status) {
        red_.clear();
        for (size_t i = 0; i < m_; ++i) {
            const size_t e = m_ - i - 1;
            red_.push_back(ParityPacket{min_ + k_ + e,
                                        std::string((const char*)rec + e * bb, (size_t)bb),
                                        kPacket1BytePn});
        }
        red_status_ = status;
        have_red_ = true;
    }

    std::vector<ParityPacket> getRedundancyPackets(int* status) {
        if (have_red_) {   // produced by a batched flush
            have_red_ = false;
            if (status) *status = red_status_;
            return std::move(red_);
        }
        int bb = 0;
        std::vector<unsigned char> blocks;
        if (!EncodeInput(&bb, &blocks)) {
            if (status) *status = -2;
            return {};
        }
        if (enc_ == cauchy_256_encode) _cauchy_256_init(CAUCHY_256_VERSION);   // :342
        std::vector<const unsigned char*> ptrs(k_);
        for (size_t i = 0; i < k_; ++i) ptrs[i] = blocks.data() + i * bb;
        std::vector<unsigned char> rec((size_t)m_ * bb, 0);
        // always executed and checked (the reference wraps it in assert(), :378)
        const int rc = enc_((int)k_, (int)m_, ptrs.data(), rec.data(), bb);
        SetRedundancy(rec.data(), bb, rc);
        have_red_ = false;
        if (status) *status = rc;
        return std::move(red_);
    }

    // ----------------------------------------------------------------- receiver side
    // Decode input (:243-274): missing data packet numbers, the first k received
    // packets in arrival order padded to block_bytes = the largest stored packet, and
    // their row tags.  Marks the missing packets as received (:249).
    bool DecodeInput(std::vector<uint64_t>* missing, int* bb, std::vector<unsigned char>* blocks,
                     std::vector<unsigned char>* rows) {
        if (!CanRevive()) return false;
        missing->clear();
        for (uint64_t pn = min_; pn <= max_; ++pn)
            if (!received_set_.count(pn)) {
                missing->push_back(pn);
                received_set_.insert(pn);
            }
        if (missing->empty()) return false;
        size_t mx = 0;
        for (auto& r : received_) mx = std::max(mx, r.packet_data.size());
        *bb = (int)mx;
        blocks->assign((size_t)k_ * mx, 0);
        rows->assign(k_, 0);
        size_t i = 0;
        for (auto it = received_.begin(); it != received_.end() && i < k_; ++it, ++i) {
            memcpy(blocks->data() + i * mx, it->packet_data.data(), it->packet_data.size());
            (*rows)[i] = (unsigned char)(it->packet_number - min_);
        }
        return true;
    }

    // Extraction after the decode (:280-293).  `blocks` / `rows` hold `nblk` decoded blocks
    // and their row tags: all k of the in-place layout, or the recovered ones only.
    void SetRevived(const std::vector<uint64_t>& missing, const unsigned char* blocks,
                    const unsigned char* rows, int bb, int status, size_t nblk = 0) {
        if (nblk == 0) nblk = k_;
        rev_.clear();
        for (uint64_t pn : missing) {
            const unsigned char* payload = nullptr;
            for (size_t i = 0; i < nblk; ++i)
                if (rows[i] == (unsigned char)(pn - min_)) {
                    payload = blocks + i * bb;
                    break;
                }
            if (!payload) break;
            uint16_t len = (uint16_t)(payload[0] | (payload[1] << 8));
            const int pnlen = len >> 14;
            len &= 0x3fff;
            const size_t n = std::min<size_t>(len, bb >= 2 ? (size_t)bb - 2 : 0);
            rev_.push_back(ParityPacket{pn, std::string((const char*)payload + 2, n), pnlen});
        }
        rev_status_ = status;
        have_rev_ = true;
    }

    std::vector<ParityPacket> getRevivedPackets(int* status) {
        if (have_rev_) {
            have_rev_ = false;
            if (status) *status = rev_status_;
            return std::move(rev_);
        }
        if (status) *status = 0;
        std::vector<uint64_t> missing;
        int bb = 0;
        std::vector<unsigned char> blocks, rows;
        if (!DecodeInput(&missing, &bb, &blocks, &rows)) return {};
        std::vector<Block> blk(k_);
        for (size_t i = 0; i < k_; ++i) {
            blk[i].data = blocks.data() + i * bb;
            blk[i].row = rows[i];
        }
        const int rc = dec_((int)k_, (int)m_, blk.data(), bb);   // :277
        for (size_t i = 0; i < k_; ++i) rows[i] = blk[i].row;
        SetRevived(missing, blocks.data(), rows.data(), bb, rc);
        have_rev_ = false;
        if (status) *status = rc;
        return std::move(rev_);
    }

    const int fec_configuration;   // public in the reference too (quic_fec_group.h:43)

   private:
    uint64_t min_, max_;
    size_t k_ = 0, m_ = 0;
    int eff_level_;
    std::vector<ParityPacket> sent_;
    std::list<ParityPacket> received_;   // arrival order
    std::set<uint64_t> received_set_;
    bool have_red_ = false, have_rev_ = false;
    int red_status_ = 0, rev_status_ = 0;
    std::vector<ParityPacket> red_, rev_;
    qfec_encode_fn enc_;
    qfec_decode_fn dec_;
};

}  // namespace qfec

struct qfec_group {
    qfec::QuicFecGroup g;
    qfec_group(unsigned long long n, int conf, qfec_encode_fn e = nullptr, qfec_decode_fn d = nullptr)
        : g(n, conf, e, d) {}
};
struct qfec_packets {
    std::vector<qfec::ParityPacket> v;
};

// ------------------------------------------------------------------ batching front end
struct qfec_batch {
    qfec_ctx* ctx;
    size_t max_groups;
    unsigned max_delay_us;
    struct Enc {
        qfec_group* g;
        std::vector<unsigned char> blocks;
        std::chrono::steady_clock::time_point t;
    };
    struct Dec {
        qfec_group* g;
        std::vector<uint64_t> missing;
        std::vector<unsigned char> blocks, rows;
        std::chrono::steady_clock::time_point t;
    };
    std::map<std::tuple<int, int, int>, std::vector<Enc>> enc;   // (k, m, bb)
    std::map<std::tuple<int, int, int>, std::vector<Dec>> dec;
    std::vector<unsigned char> hbuf, hrows;
    std::vector<int> hstatus;
};

namespace {

int flush_enc(qfec_batch* b, const std::tuple<int, int, int>& key) {
    auto& v = b->enc[key];
    if (v.empty()) return 0;
    const int k = std::get<0>(key), m = std::get<1>(key), bb = std::get<2>(key);
    const size_t G = v.size();
    b->hbuf.resize(G * (size_t)(k + m) * bb);
    unsigned char* data = b->hbuf.data();
    unsigned char* par = data + G * (size_t)k * bb;
    for (size_t i = 0; i < G; ++i) memcpy(data + i * (size_t)k * bb, v[i].blocks.data(), (size_t)k * bb);
    memset(par, 0, G * (size_t)m * bb);
    const int rc = qfec_encode_batch_host(b->ctx, k, m, bb, (long long)G, data, par);
    for (size_t i = 0; i < G; ++i) v[i].g->g.SetRedundancy(par + i * (size_t)m * bb, bb, rc);
    v.clear();
    return rc < -1 ? rc : (int)G;
}

int flush_dec(qfec_batch* b, const std::tuple<int, int, int>& key) {
    auto& v = b->dec[key];
    if (v.empty()) return 0;
    const int k = std::get<0>(key), m = std::get<1>(key), bb = std::get<2>(key);
    const size_t G = v.size();
    const size_t rmax = (size_t)std::min(k, m);
    // inputs [G][k][bb] + [G][k]; outputs: only the recovered blocks (rmax per group)
    b->hbuf.resize(G * ((size_t)k + rmax) * bb);
    b->hrows.resize(G * ((size_t)k + rmax));
    b->hstatus.assign(G, 0);
    unsigned char* in = b->hbuf.data();
    unsigned char* rec = in + G * (size_t)k * bb;
    unsigned char* rows = b->hrows.data();
    unsigned char* rec_rows = rows + G * (size_t)k;
    for (size_t i = 0; i < G; ++i) {
        memcpy(in + i * (size_t)k * bb, v[i].blocks.data(), (size_t)k * bb);
        memcpy(rows + i * (size_t)k, v[i].rows.data(), (size_t)k);
    }
    const int rc = qfec_decode_batch_recovered_host(b->ctx, k, m, bb, (long long)G, in, rows,
                                                    rec, rec_rows, b->hstatus.data());
    for (size_t i = 0; i < G; ++i)
        v[i].g->g.SetRevived(v[i].missing, rec + i * rmax * bb, rec_rows + i * rmax, bb,
                             rc ? rc : b->hstatus[i], rmax);
    v.clear();
    return rc ? rc : (int)G;
}

}  // namespace

extern "C" {

void qfec_set_fec_overrides(size_t k, size_t m) {
    qfec::g_override_k = k;
    qfec::g_override_m = m;
}
size_t qfec_k_from_conf(int c) { return qfec::k_from_conf(c); }
size_t qfec_m_from_conf(int c) { return qfec::m_from_conf(c); }

long qfec_prefix_payload(const unsigned char* p, size_t len, int pnlen, unsigned char* out) {
    if (len > 0x3fff) return -1;   // DCHECK_LE(payload_len, 0xffff >> 2), :113
    const std::string s = qfec::prefixed(p, len, pnlen);
    memcpy(out, s.data(), s.size());
    return (long)s.size();
}
int qfec_block_bytes(size_t n) { return qfec::round8(n); }

qfec_group* qfec_group_new(unsigned long long n, int conf) { return new qfec_group(n, conf); }
qfec_group* qfec_group_new_with_codec(unsigned long long n, int conf, qfec_encode_fn e,
                                      qfec_decode_fn d) {
    return new qfec_group(n, conf, e, d);
}
void qfec_group_free(qfec_group* g) { delete g; }

int qfec_group_update_sent(qfec_group* g, int level, unsigned long long pn, int pnlen,
                           const unsigned char* p, size_t len) {
    return g->g.UpdateSentList(level, pn, pnlen, p, len);
}
int qfec_group_update_received(qfec_group* g, int level, unsigned long long pn, int pnlen,
                               const unsigned char* p, size_t len, int is_fec) {
    return g->g.UpdateReceivedList(level, pn, pnlen, p, len, is_fec != 0);
}
int qfec_group_update_fec(qfec_group* g, int level, unsigned long long pn, int pnlen,
                          const unsigned char* p, size_t len) {
    return g->g.UpdateFec(level, pn, pnlen, p, len);
}
int qfec_group_can_revive(const qfec_group* g) { return g->g.CanRevive(); }
int qfec_group_is_waiting_for_packet_before(const qfec_group* g, unsigned long long num) {
    return g->g.IsWaitingForPacketBefore(num);
}
size_t qfec_group_num_received(const qfec_group* g) { return g->g.NumReceivedPackets(); }
size_t qfec_group_num_sent(const qfec_group* g) { return g->g.NumSentPackets(); }
int qfec_group_effective_encryption_level(const qfec_group* g) {
    return g->g.EffectiveEncryptionLevel();
}
unsigned long long qfec_group_number(const qfec_group* g) { return g->g.FecGroupNumber(); }
size_t qfec_group_total_size(const qfec_group* g) { return g->g.GroupTotalSize(); }
size_t qfec_group_redundancy_size(const qfec_group* g) { return g->g.GroupReduntancySize(); }

qfec_packets* qfec_group_redundancy(qfec_group* g, int* status) {
    auto* l = new qfec_packets;
    l->v = g->g.getRedundancyPackets(status);
    return l;
}
qfec_packets* qfec_group_revived(qfec_group* g, int* status) {
    auto* l = new qfec_packets;
    l->v = g->g.getRevivedPackets(status);
    return l;
}

size_t qfec_packets_count(const qfec_packets* l) { return l ? l->v.size() : 0; }
int qfec_packets_get(const qfec_packets* l, size_t i, unsigned long long* pn,
                     const unsigned char** data, size_t* len, int* pnlen) {
    if (!l || i >= l->v.size()) return -2;
    const auto& p = l->v[i];
    if (pn) *pn = p.packet_number;
    if (data) *data = (const unsigned char*)p.packet_data.data();
    if (len) *len = p.packet_data.size();
    if (pnlen) *pnlen = p.packet_number_len;
    return 0;
}
void qfec_packets_free(qfec_packets* l) { delete l; }

qfec_batch* qfec_batch_new(qfec_ctx* ctx, size_t max_groups, unsigned max_delay_us) {
    if (!ctx || max_groups == 0) return nullptr;
    auto* b = new qfec_batch;
    b->ctx = ctx;
    b->max_groups = max_groups;
    b->max_delay_us = max_delay_us;
    return b;
}
void qfec_batch_free(qfec_batch* b) { delete b; }

int qfec_batch_add_encode(qfec_batch* b, qfec_group* g) {
    qfec_batch::Enc e;
    int bb = 0;
    if (!g->g.EncodeInput(&bb, &e.blocks)) return -2;
    e.g = g;
    e.t = std::chrono::steady_clock::now();
    auto key = std::make_tuple((int)g->g.k(), (int)g->g.m(), bb);
    auto& v = b->enc[key];
    v.push_back(std::move(e));
    return v.size() >= b->max_groups ? flush_enc(b, key) : 0;
}

int qfec_batch_add_decode(qfec_batch* b, qfec_group* g) {
    qfec_batch::Dec d;
    int bb = 0;
    if (!g->g.DecodeInput(&d.missing, &bb, &d.blocks, &d.rows)) return -2;
    d.g = g;
    d.t = std::chrono::steady_clock::now();
    auto key = std::make_tuple((int)g->g.k(), (int)g->g.m(), bb);
    auto& v = b->dec[key];
    v.push_back(std::move(d));
    return v.size() >= b->max_groups ? flush_dec(b, key) : 0;
}

int qfec_batch_flush(qfec_batch* b) {
    int n = 0;
    for (auto& kv : b->enc) {
        const int r = flush_enc(b, kv.first);
        if (r < 0) return r;
        n += r;
    }
    for (auto& kv : b->dec) {
        const int r = flush_dec(b, kv.first);
        if (r < 0) return r;
        n += r;
    }
    return n;
}

int qfec_batch_poll(qfec_batch* b) {
    const auto now = std::chrono::steady_clock::now();
    const auto lim = std::chrono::microseconds(b->max_delay_us);
    int n = 0;
    for (auto& kv : b->enc)
        if (!kv.second.empty() && now - kv.second.front().t >= lim) {
            const int r = flush_enc(b, kv.first);
            if (r < 0) return r;
            n += r;
        }
    for (auto& kv : b->dec)
        if (!kv.second.empty() && now - kv.second.front().t >= lim) {
            const int r = flush_dec(b, kv.first);
            if (r < 0) return r;
            n += r;
        }
    return n;
}

size_t qfec_batch_pending(const qfec_batch* b) {
    size_t n = 0;
    for (auto& kv : b->enc) n += kv.second.size();
    for (auto& kv : b->dec) n += kv.second.size();
    return n;
}

}  // extern "C"
