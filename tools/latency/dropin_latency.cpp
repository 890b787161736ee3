// dropin_latency.cpp — microseconds per single-group codec call, GPU drop-in vs CPU codec.
//
// The reference calls the codec once per group, synchronously, on the QUIC thread:
// cauchy_256_encode from QuicFecGroup::getRedundancyPackets (quic_fec_group.cc:378) and
// cauchy_256_decode from getRevivedPackets (quic_fec_group.cc:277).  libquic_fec.so exports
// the same two symbols (include/quic_fec.h); each call stages the group through pinned
// memory, runs the gfx950 kernels and copies the result back before returning.  This tool
// times both implementations of the ABI on the same inputs:
//   --ref=PATH   a cauchy_256-ABI library to compare against (oracle/_ref/libref_cauchy.so)
//   --iters=N    calls per measurement (default 2000)
// Output: one JSON line per (k, m, bb, losses) case with the median / p99 microseconds per
// call of each implementation, and whether the outputs agreed byte for byte.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "quic_fec.h"

namespace {

typedef int (*enc_fn)(int, int, const unsigned char**, void*, int);
typedef int (*dec_fn)(int, int, Block*, int);

struct Impl {
    const char* name;
    enc_fn enc;
    dec_fn dec;
};

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double now_us() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct Stat {
    double med, p99;
};
Stat stats(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return {v[v.size() / 2], v[std::min(v.size() - 1, v.size() * 99 / 100)]};
}

// one case: encode latency, then decode latency with `losses` data blocks replaced by the
// first `losses` parity blocks (rows k .. k+losses-1), fresh copies before every call
bool run_case(const Impl* impls, int nimpl, int k, int m, int bb, int losses, int iters) {
    uint64_t seed = 1234 + k * 131 + m;
    std::vector<uint8_t> data((size_t)k * bb);
    for (auto& b : data) b = (uint8_t)splitmix(seed);
    std::vector<const unsigned char*> ptrs(k);
    for (int x = 0; x < k; ++x) ptrs[x] = data.data() + (size_t)x * bb;
    std::vector<std::vector<uint8_t>> parity(nimpl, std::vector<uint8_t>((size_t)m * bb));
    std::vector<Stat> enc_s(nimpl), dec_s(nimpl);
    bool agree = true;
    for (int i = 0; i < nimpl; ++i) {
        std::vector<double> t;
        for (int it = 0; it < iters + 50; ++it) {
            const double t0 = now_us();
            const int rc = impls[i].enc(k, m, ptrs.data(), parity[i].data(), bb);
            const double t1 = now_us();
            if (rc != 0) { fprintf(stderr, "%s encode rc %d\n", impls[i].name, rc); return false; }
            if (it >= 50) t.push_back(t1 - t0);
        }
        enc_s[i] = stats(t);
        if (parity[i] != parity[0]) agree = false;
    }
    // receive set: data rows losses..k-1 then parity rows 0..losses-1 (row k + j)
    std::vector<uint8_t> recv((size_t)k * bb);
    std::vector<uint8_t> rows(k);
    for (int s = 0; s < k; ++s) {
        const int row = s < k - losses ? s + losses : k + (s - (k - losses));
        rows[s] = (uint8_t)row;
        const uint8_t* src = row < k ? data.data() + (size_t)row * bb
                                     : parity[0].data() + (size_t)(row - k) * bb;
        memcpy(recv.data() + (size_t)s * bb, src, bb);
    }
    std::vector<uint8_t> work(recv.size());
    std::vector<Block> blk(k);
    for (int i = 0; i < nimpl; ++i) {
        std::vector<double> t;
        for (int it = 0; it < iters + 50; ++it) {
            work = recv;
            for (int s = 0; s < k; ++s) {
                blk[s].data = work.data() + (size_t)s * bb;
                blk[s].row = rows[s];
            }
            const double t0 = now_us();
            const int rc = impls[i].dec(k, m, blk.data(), bb);
            const double t1 = now_us();
            if (rc != 0) { fprintf(stderr, "%s decode rc %d\n", impls[i].name, rc); return false; }
            if (it >= 50) t.push_back(t1 - t0);
        }
        dec_s[i] = stats(t);
        for (int s = 0; s < k; ++s)   // every slot now holds its data row
            if (blk[s].row >= k ||
                memcmp(blk[s].data, data.data() + (size_t)blk[s].row * bb, bb) != 0)
                agree = false;
    }
    printf("{\"k\": %d, \"m\": %d, \"block_bytes\": %d, \"losses\": %d, \"iters\": %d",
           k, m, bb, losses, iters);
    for (int i = 0; i < nimpl; ++i)
        printf(", \"%s\": {\"encode_us_median\": %.2f, \"encode_us_p99\": %.2f, "
               "\"decode_us_median\": %.2f, \"decode_us_p99\": %.2f}",
               impls[i].name, enc_s[i].med, enc_s[i].p99, dec_s[i].med, dec_s[i].p99);
    printf(", \"outputs_agree\": %s}\n", agree ? "true" : "false");
    fflush(stdout);
    return agree;
}

}  // namespace

int main(int argc, char** argv) {
    std::string ref;
    int iters = 2000;
    for (int i = 1; i < argc; ++i) {
        if (!strncmp(argv[i], "--ref=", 6)) ref = argv[i] + 6;
        else if (!strncmp(argv[i], "--iters=", 8)) iters = atoi(argv[i] + 8);
        else { fprintf(stderr, "usage: %s [--ref=PATH] [--iters=N]\n", argv[0]); return 2; }
    }
    Impl impls[2];
    int n = 0;
    if (_cauchy_256_init(CAUCHY_256_VERSION) != 0) {
        fprintf(stderr, "GPU drop-in init failed: %s\n", qfec_last_error());
        return 3;
    }
    impls[n++] = {"gpu_dropin", cauchy_256_encode, cauchy_256_decode};
    if (!ref.empty()) {
        void* h = dlopen(ref.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) { fprintf(stderr, "dlopen %s: %s\n", ref.c_str(), dlerror()); return 2; }
        auto init = (int (*)(int))dlsym(h, "_cauchy_256_init");
        impls[n] = {"cpu_reference", (enc_fn)dlsym(h, "cauchy_256_encode"),
                    (dec_fn)dlsym(h, "cauchy_256_decode")};
        if (!init || !impls[n].enc || !impls[n].dec || init(2) != 0) {
            fprintf(stderr, "%s is not a cauchy_256 codec\n", ref.c_str());
            return 2;
        }
        ++n;
    }
    bool ok = run_case(impls, n, 10, 1, 1352, 1, iters);
    ok = run_case(impls, n, 32, 4, 1352, 2, iters) && ok;
    ok = run_case(impls, n, 128, 16, 9008, 8, std::max(20, iters / 20)) && ok;
    return ok ? 0 : 1;
}
