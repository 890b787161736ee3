// fec_loopback — standalone UDP loopback sender/receiver with packet-group FEC.
//
// Counterpart of the QuicR loopback file transfer (net/tools/quic/quic_simple_server_bin.cc
// send_file_fifo :480-518, quic_simple_client_bin.cc recv_file :814-859) reduced to what the
// FEC path needs: the file is cut into 1350-byte payloads, grouped k at a time, protected by
// m parity packets (QuicFecGroup counterpart, include/quic_fec_group.h), sent over UDP on
// 127.0.0.1 through a seeded dropper (cf. PacketDroppingTestWriter,
// test_tools/packet_dropping_test_writer.h:28-80, and the LOSS macro,
// quic_connection.cc:1646-1659), revived on the receiver and checked end to end by
// SHA-256 (cf. the MD5 check in Script/tests.py:104-108).
//
//   --gpu-fec            codec = the MI355X engine (default: required unless --cpu-codec)
//   --cpu-codec=PATH     codec = a cauchy_256-ABI shared library (e.g. the reference codec
//                        compiled into oracle/_ref by oracle/Makefile) — the CPU baseline
//   --fec --m=K --k=M    group size: as in the reference CLI, --m is the DATA count and --k
//                        the PARITY count (quic_protocol.cc:35 "m and k are reversed here")
//   --loss=P --seed=S    drop each packet with probability P (seeded)
//   --drop=a,b,...       also drop these packet numbers
//   --batch=N            GPU only: queue groups and run one batched launch per N groups
//   --tables=F           coefficient tables for an oracle/liboracle_fec.so codec
//   --input_file=F | --bytes=N   payload source (synthetic splitmix64 stream by default)
//   --output_file=F      write the received stream
//
// Wire format (this tool's own, not QUIC's; see SURVEY.md 8f for the QUIC FEC framing):
//   24-byte header {u8 type (1 data, 2 fec, 3 fin), u8 pn_len, u16 len, u32 pad, u64 pn,
//   u64 group} + len payload bytes.  Parity packets take packet numbers min + k .. min + k
//   + m - 1 exactly like quic_packet_creator.cc:929-990, so groups are k + m apart.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "quic_fec_group.h"

namespace {

// ------------------------------------------------------------------------- SHA-256
struct Sha256 {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                     0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[64];
    size_t n = 0;
    uint64_t total = 0;
    static uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
    void block(const uint8_t* p) {
        static const uint32_t K[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
            0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
            0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
            0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
            0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
            0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
            0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
            0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
            0xc67178f2};
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
                   (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                                K[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t* p, size_t len) {
        total += len;
        while (len) {
            const size_t t = std::min(len, 64 - n);
            memcpy(buf + n, p, t);
            n += t; p += t; len -= t;
            if (n == 64) { block(buf); n = 0; }
        }
    }
    std::string hex() {
        const uint64_t bits = total * 8;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while (n != 56) update(&zero, 1);
        uint8_t lb[8];
        for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(lb, 8);
        char s[65];
        for (int i = 0; i < 8; ++i) snprintf(s + 8 * i, 9, "%08x", h[i]);
        return std::string(s, 64);
    }
};

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct Hdr {
    uint8_t type, pn_len;
    uint16_t len;
    uint32_t pad;
    uint64_t pn, group;
};
static_assert(sizeof(Hdr) == 24, "wire header");
constexpr int kPayload = 1350;   // BASELINE payload size
enum { T_DATA = 1, T_FEC = 2, T_FIN = 3 };

struct Opts {
    bool gpu = false;
    std::string cpu_codec;
    int k = 10, m = 1;
    double loss = 0.0;
    uint64_t seed = 1;
    std::set<uint64_t> drop;
    int batch = 0;
    std::string in_file, out_file, tables = "quic_amd/data/cauchy_256_tables.bin";
    size_t bytes = 10 * kPayload;
    int port = 0;
};

struct Codec {
    qfec_encode_fn enc = nullptr;
    qfec_decode_fn dec = nullptr;
};

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct RecvStats {
    size_t data = 0, fec = 0, revived = 0, dup = 0, unrecovered = 0;
    double codec_s = 0;
    uint64_t fin_packets = 0, fin_bytes = 0;
    bool fin = false;
};

// Receiver: groups by number, payloads by stream position; revive on CanRevive().
void receiver(int sock, const Opts& o, const Codec& cd, qfec_ctx* ctx, std::vector<uint8_t>* out,
              RecvStats* st) {
    const int gsz = o.k + o.m;
    std::map<uint64_t, qfec_group*> groups;
    std::set<uint64_t> done;
    std::map<uint64_t, std::vector<uint8_t>> payload;   // data pn -> payload
    std::unique_ptr<qfec_batch, void (*)(qfec_batch*)> batch(
        o.gpu && o.batch > 0 ? qfec_batch_new(ctx, o.batch, 2000) : nullptr, qfec_batch_free);
    std::vector<qfec_group*> queued;
    std::vector<uint8_t> buf(65536);
    auto harvest = [&](qfec_group* g) {
        int status = 0;
        const double t0 = now();
        qfec_packets* l = qfec_group_revived(g, &status);
        st->codec_s += now() - t0;
        for (size_t i = 0; i < qfec_packets_count(l); ++i) {
            unsigned long long pn;
            const unsigned char* d;
            size_t n;
            int pl;
            qfec_packets_get(l, i, &pn, &d, &n, &pl);
            if (!payload.count(pn)) {
                payload[pn].assign(d, d + n);
                ++st->revived;
            }
        }
        qfec_packets_free(l);
    };
    auto flush_batch = [&] {
        if (!batch) return;
        const double t0 = now();
        qfec_batch_flush(batch.get());
        st->codec_s += now() - t0;
        for (auto* g : queued) harvest(g);
        queued.clear();
    };
    while (true) {
        const ssize_t r = recv(sock, buf.data(), buf.size(), 0);
        if (r < 0) break;   // timeout: sender gone
        if ((size_t)r < sizeof(Hdr)) continue;
        Hdr h;
        memcpy(&h, buf.data(), sizeof h);
        const uint8_t* p = buf.data() + sizeof h;
        if (h.type == T_FIN) {
            st->fin = true;
            st->fin_packets = h.pn;
            st->fin_bytes = h.group;
            break;
        }
        if (done.count(h.group)) {
            if (h.type == T_DATA && !payload.count(h.pn)) payload[h.pn].assign(p, p + h.len);
            continue;
        }
        qfec_group*& g = groups[h.group];
        if (!g) g = cd.enc ? qfec_group_new_with_codec(h.group, QFEC_FEC_5_5, cd.enc, cd.dec)
                           : qfec_group_new(h.group, QFEC_FEC_5_5);
        bool fresh;
        if (h.type == T_DATA) {
            fresh = qfec_group_update_received(g, 2, h.pn, h.pn_len, p, h.len, 0);
            if (fresh) { payload[h.pn].assign(p, p + h.len); ++st->data; }
        } else {
            fresh = qfec_group_update_fec(g, 2, h.pn, h.pn_len, p, h.len);
            if (fresh) ++st->fec;
        }
        if (!fresh) { ++st->dup; continue; }
        if (qfec_group_can_revive(g)) {
            done.insert(h.group);
            if (batch) {
                if (qfec_batch_add_decode(batch.get(), g) == 0) queued.push_back(g);
                if (queued.size() >= (size_t)o.batch) flush_batch();
            } else {
                harvest(g);
            }
        }
    }
    flush_batch();
    // reassemble: data packet numbers in stream order (groups are k + m apart)
    out->clear();
    for (uint64_t i = 0; i < st->fin_packets; ++i) {
        const uint64_t pn = 1 + (i / o.k) * gsz + (i % o.k);
        auto it = payload.find(pn);
        if (it == payload.end()) {   // more than m losses in the group: zero-fill, count it
            ++st->unrecovered;
            out->resize(out->size() + kPayload, 0);
            continue;
        }
        out->insert(out->end(), it->second.begin(), it->second.end());
    }
    if (st->fin && out->size() > st->fin_bytes) out->resize(st->fin_bytes);
    for (auto& kv : groups) qfec_group_free(kv.second);
}

int parse(int argc, char** argv, Opts* o) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&](const char* key) -> const char* {
            const size_t n = strlen(key);
            return a.compare(0, n, key) == 0 ? a.c_str() + n : nullptr;
        };
        const char* v;
        if (a == "--gpu-fec") o->gpu = true;
        else if (a == "--fec") {}
        else if ((v = val("--cpu-codec="))) o->cpu_codec = v;
        else if ((v = val("--m="))) o->k = atoi(v);   // reversed, as in quic_protocol.cc:35
        else if ((v = val("--k="))) o->m = atoi(v);
        else if ((v = val("--loss="))) o->loss = atof(v);
        else if ((v = val("--seed="))) o->seed = strtoull(v, nullptr, 10);
        else if ((v = val("--batch="))) o->batch = atoi(v);
        else if ((v = val("--input_file="))) o->in_file = v;
        else if ((v = val("--output_file="))) o->out_file = v;
        else if ((v = val("--bytes="))) o->bytes = strtoull(v, nullptr, 10);
        else if ((v = val("--port="))) o->port = atoi(v);
        else if ((v = val("--tables="))) o->tables = v;
        else if ((v = val("--drop="))) {
            std::string s = v;
            size_t pos = 0;
            while (pos < s.size()) {
                const size_t c = s.find(',', pos);
                o->drop.insert(strtoull(s.substr(pos, c - pos).c_str(), nullptr, 10));
                if (c == std::string::npos) break;
                pos = c + 1;
            }
        } else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return -1;
        }
    }
    if (o->k < 1 || o->m < 1 || o->k + o->m > 255) return -1;
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    Opts o;
    if (parse(argc, argv, &o)) return 2;
    if (!o.gpu && o.cpu_codec.empty()) {
        fprintf(stderr, "choose --gpu-fec or --cpu-codec=PATH\n");
        return 2;
    }
    Codec cd;
    if (!o.cpu_codec.empty()) {
        void* h = dlopen(o.cpu_codec.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) { fprintf(stderr, "dlopen %s: %s\n", o.cpu_codec.c_str(), dlerror()); return 2; }
        cd.enc = (qfec_encode_fn)dlsym(h, "cauchy_256_encode");
        cd.dec = (qfec_decode_fn)dlsym(h, "cauchy_256_decode");
        int rc = -1;
        if (auto init = (int (*)(int))dlsym(h, "_cauchy_256_init")) {
            rc = init(2);
        } else if (auto oinit = (int (*)(const char*))dlsym(h, "oracle_init")) {
            // the test oracle (oracle/fec_oracle.h): same encode/decode ABI, tables from a file
            cd.enc = (qfec_encode_fn)dlsym(h, "oracle_encode");
            cd.dec = (qfec_decode_fn)dlsym(h, "oracle_decode");
            rc = oinit(o.tables.c_str());
        }
        if (!cd.enc || !cd.dec || rc != 0) { fprintf(stderr, "bad codec library\n"); return 2; }
        o.batch = 0;
    }
    qfec_set_fec_overrides(o.k, o.m);
    qfec_ctx* ctx = nullptr;
    if (o.gpu) {
        if (int rc = qfec_ctx_create(0, &ctx)) { fprintf(stderr, "GPU: %d %s\n", rc, qfec_last_error()); return 3; }
        if (_cauchy_256_init(CAUCHY_256_VERSION) != 0) { fprintf(stderr, "GPU init failed: %s\n", qfec_last_error()); return 3; }
    }

    // payload source
    std::vector<uint8_t> input;
    if (!o.in_file.empty()) {
        FILE* f = fopen(o.in_file.c_str(), "rb");
        if (!f) { perror("input_file"); return 2; }
        uint8_t b[65536];
        size_t n;
        while ((n = fread(b, 1, sizeof b, f)) > 0) input.insert(input.end(), b, b + n);
        fclose(f);
    } else {
        uint64_t s = o.seed * 1000003;
        input.resize(o.bytes);
        for (size_t i = 0; i < o.bytes; i += 8) {
            const uint64_t w = splitmix(s);
            memcpy(input.data() + i, &w, std::min<size_t>(8, o.bytes - i));
        }
    }

    // sockets on 127.0.0.1
    int rs = socket(AF_INET, SOCK_DGRAM, 0), ss = socket(AF_INET, SOCK_DGRAM, 0);
    int big = 64 << 20;
    setsockopt(rs, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    timeval tv{2, 0};
    setsockopt(rs, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    addr.sin_port = htons((uint16_t)o.port);
    if (bind(rs, (sockaddr*)&addr, sizeof addr)) { perror("bind"); return 2; }
    socklen_t al = sizeof addr;
    getsockname(rs, (sockaddr*)&addr, &al);

    RecvStats rst;
    std::vector<uint8_t> output;
    std::thread rt(receiver, rs, std::cref(o), std::cref(cd), ctx, &output, &rst);

    // sender: groups of k payloads + m parity packets
    const int gsz = o.k + o.m;
    const size_t npk = (input.size() + kPayload - 1) / kPayload;
    const size_t ngroups = (npk + o.k - 1) / o.k;
    uint64_t rng = o.seed;
    size_t sent = 0, dropped = 0, sent_fec = 0;
    double enc_s = 0;
    std::vector<uint8_t> wire(sizeof(Hdr) + 16384);
    auto send_pkt = [&](uint8_t type, uint64_t pn, uint64_t grp, int pnlen, const uint8_t* d, size_t n) {
        const bool drop = o.drop.count(pn) ||
                          (o.loss > 0 && (double)(splitmix(rng) >> 11) * 0x1.0p-53 < o.loss);
        ++sent;
        if (type == T_FEC) ++sent_fec;
        if (drop && type != T_FIN) { ++dropped; return; }
        Hdr h{type, (uint8_t)pnlen, (uint16_t)n, 0, pn, grp};
        memcpy(wire.data(), &h, sizeof h);
        if (n) memcpy(wire.data() + sizeof h, d, n);
        sendto(ss, wire.data(), sizeof h + n, 0, (sockaddr*)&addr, sizeof addr);
        if (sent % 256 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
    };
    const double t_start = now();
    std::unique_ptr<qfec_batch, void (*)(qfec_batch*)> sbatch(
        o.gpu && o.batch > 0 ? qfec_batch_new(ctx, o.batch, 1u << 30) : nullptr, qfec_batch_free);
    std::vector<std::pair<qfec_group*, std::vector<std::pair<uint64_t, std::vector<uint8_t>>>>> pend;
    auto emit_parity = [&] {
        for (auto& gp : pend) {
            int status = 0;
            const double t0 = now();
            qfec_packets* l = qfec_group_redundancy(gp.first, &status);
            enc_s += now() - t0;
            if (status) fprintf(stderr, "encode status %d\n", status);
            const unsigned long long base = qfec_group_number(gp.first);
            for (auto& dp : gp.second)
                send_pkt(T_DATA, dp.first, base, 2, dp.second.data(), dp.second.size());
            // the creator sends the list back to front: parity 0 .. m-1 on the wire
            for (size_t i = qfec_packets_count(l); i-- > 0;) {
                unsigned long long pn;
                const unsigned char* d;
                size_t n;
                int pl;
                qfec_packets_get(l, i, &pn, &d, &n, &pl);
                send_pkt(T_FEC, pn, base, pl, d, n);
            }
            qfec_packets_free(l);
            qfec_group_free(gp.first);
        }
        pend.clear();
    };
    for (size_t gi = 0; gi < ngroups; ++gi) {
        const uint64_t base = 1 + gi * gsz;
        qfec_group* g = cd.enc ? qfec_group_new_with_codec(base, QFEC_FEC_5_5, cd.enc, cd.dec)
                               : qfec_group_new(base, QFEC_FEC_5_5);
        std::vector<std::pair<uint64_t, std::vector<uint8_t>>> data;
        for (int i = 0; i < o.k; ++i) {
            const size_t off = (gi * o.k + i) * kPayload;
            const size_t n = off < input.size() ? std::min<size_t>(kPayload, input.size() - off) : 0;
            std::vector<uint8_t> pl(input.begin() + std::min(off, input.size()),
                                    input.begin() + std::min(off + n, input.size()));
            qfec_group_update_sent(g, 2, base + i, 2, pl.data(), pl.size());
            data.emplace_back(base + i, std::move(pl));
        }
        pend.emplace_back(g, std::move(data));
        if (sbatch) {
            qfec_batch_add_encode(sbatch.get(), g);
            if (pend.size() >= (size_t)o.batch) {
                const double t0 = now();
                qfec_batch_flush(sbatch.get());
                enc_s += now() - t0;
                emit_parity();
            }
        } else {
            emit_parity();
        }
    }
    if (sbatch) {
        const double t0 = now();
        qfec_batch_flush(sbatch.get());
        enc_s += now() - t0;
    }
    emit_parity();
    for (int i = 0; i < 5; ++i) {   // FIN: data packet count and byte count
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        Hdr h{T_FIN, 0, 0, 0, (uint64_t)npk, (uint64_t)input.size()};
        sendto(ss, &h, sizeof h, 0, (sockaddr*)&addr, sizeof addr);
    }
    rt.join();
    const double wall = now() - t_start;

    if (!o.out_file.empty()) {
        FILE* f = fopen(o.out_file.c_str(), "wb");
        if (f) { fwrite(output.data(), 1, output.size(), f); fclose(f); }
    }
    Sha256 a, b;
    a.update(input.data(), input.size());
    b.update(output.data(), output.size());
    const std::string ha = a.hex(), hb = b.hex();
    const bool match = ha == hb;
    printf("{\"codec\": \"%s\", \"k\": %d, \"m\": %d, \"groups\": %zu, \"packets_sent\": %zu, "
           "\"fec_sent\": %zu, \"dropped\": %zu, \"received_data\": %zu, \"received_fec\": %zu, "
           "\"revived\": %zu, \"unrecovered\": %zu, \"bytes\": %zu, \"bytes_out\": %zu, \"sha256_in\": \"%s\", "
           "\"sha256_out\": \"%s\", \"match\": %s, \"encode_s\": %.6f, \"decode_s\": %.6f, "
           "\"wall_s\": %.4f}\n",
           o.gpu ? "gpu" : ("cpu:" + o.cpu_codec).c_str(), o.k, o.m, ngroups, sent, sent_fec,
           dropped, rst.data, rst.fec, rst.revived, rst.unrecovered, input.size(), output.size(), ha.c_str(),
           hb.c_str(), match ? "true" : "false", enc_s, rst.codec_s, wall);
    if (ctx) qfec_ctx_destroy(ctx);
    close(rs);
    close(ss);
    return match ? 0 : 1;
}
