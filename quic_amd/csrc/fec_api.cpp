// fec_api.cpp — host side of libquic_fec.so: the C ABI in include/quic_fec.h.
//
// Owns per-device contexts (stream, coefficient tables, decode workspace, pinned
// staging) and maps the reference's per-group codec calls (cauchy_256.h) and the batched
// calls onto the gfx950 kernels in fec_kernels.hip.  There is no CPU compute path: every
// parity / recovered byte is produced on the GPU; if the device is unusable the calls
// fail with a negative code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/quic_fec.h"
#include "fec_kernels.h"
#include "gf256.h"
#include "pp_null.h"

// ------------------------------------------------------------- Cauchy table blob
// quic_amd/data/cauchy_256_tables.bin (tools/gen_cauchy_tables.py) embedded at build time:
// M2[1*254] | M3[2*253] | M4[3*252] | M5[4*251] | M6[5*250] | Y[256] | X[30876]
#ifndef QFEC_TABLES_PATH
#error "QFEC_TABLES_PATH must name quic_amd/data/cauchy_256_tables.bin"
#endif
__asm__(".section .rodata\n"
        ".balign 16\n"
        ".hidden qfec_cauchy_blob\n"
        ".globl qfec_cauchy_blob\n"
        "qfec_cauchy_blob:\n"
        ".incbin \"" QFEC_TABLES_PATH "\"\n"
        ".hidden qfec_cauchy_blob_end\n"
        ".globl qfec_cauchy_blob_end\n"
        "qfec_cauchy_blob_end:\n"
        ".previous\n");
extern "C" const unsigned char qfec_cauchy_blob[];
extern "C" const unsigned char qfec_cauchy_blob_end[];

namespace {

enum {
    T_M2 = 0, T_M3 = T_M2 + 254, T_M4 = T_M3 + 506, T_M5 = T_M4 + 756, T_M6 = T_M5 + 1004,
    T_Y = T_M6 + 1250, T_X = T_Y + 256, T_SIZE = T_X + 30876
};

thread_local std::string g_err;
thread_local std::string g_kernels;   // kernels launched by this thread's last call
thread_local std::string g_grids;     // "name=grid" of its persistent kernels

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -100 - (int)e;
}

#define QF_HIP(expr)                                   \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

bool blob_ok() { return (qfec_cauchy_blob_end - qfec_cauchy_blob) == T_SIZE; }

// cauchy_matrix(), cauchy_256.cpp:422-480: rows y = 1..m-1, (m-1) x k.
int cauchy_rows(int k, int m, uint8_t* out) {
    if (m < 2 || k < 1 || k + m > 256) return -1;
    const uint8_t* tb = qfec_cauchy_blob;
    if (m <= 6) {
        static const int base[7] = {0, 0, T_M2, T_M3, T_M4, T_M5, T_M6};
        const int stride = 256 - m;
        for (int y = 1; y < m; ++y)
            for (int x = 0; x < k; ++x) out[(y - 1) * k + x] = tb[base[m] + (y - 1) * stride + x];
        return 0;
    }
    const int n = m - 7;
    const uint8_t* X = tb + T_X + n * 249 - n * (n + 1) / 2;
    const uint8_t* Y = tb + T_Y;
    for (int y = 1; y < m; ++y) {
        const uint8_t G = Y[y - 1];
        out[(y - 1) * k] = qfec::gf_inv(1 ^ G);
        for (int x = 1; x < k; ++x) {
            const uint8_t B = X[x - 1];
            out[(y - 1) * k + x] = qfec::gf_div(B, B ^ G);
        }
    }
    return 0;
}

int pow2_at_least(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}
int encode_rc(int m, const qfec::Tune& t) { return std::min(pow2_at_least(m), t.enc_rc); }
int decode_rc(int rmax) { return std::min(pow2_at_least(rmax), 8); }
// Encode table rows: gf_apply's chunk (<= 8), or 16 where gf_stream takes 9..16 outputs in
// one unit (m <= 8: one unit of m outputs; more than 16: chunks of 8; compiled codes read no
// table)
int stream_encode_rc(int k, int m, int bb, bool aligned, const qfec::Tune& t) {
    if (m > 8 && m <= 16 && aligned && qfec::gf_stream_supported(k, m, bb, 16, false, t)) return 16;
    return encode_rc(m, t);
}
// Output chunk of a decode.  gf_stream decodes in units of 8 recovered blocks: a group with
// at most 8 losses leaves its second unit empty, and empty units read nothing, while one unit
// of 16 accumulators halves the occupancy for every group ((10, 10) at 5 losses: 0.615 ms
// with 16 against 0.544 ms).
int stream_decode_rc(int rmax) { return decode_rc(rmax); }

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
};

struct HostBuf {
    void* p = nullptr;
    size_t n = 0;
    ~HostBuf() { if (p) (void)hipHostFree(p); }
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; n = 0; }
        hipError_t e = hipHostMalloc(&p, bytes, 0);
        if (e == hipSuccess) n = bytes;
        return e;
    }
};

}  // namespace

// One decode workspace: the prep's per-group tables and the in-place scratch.
struct Workspace {
    DevBuf dcoef, dslots, dnout, dscratch;
    // graph workspace: a buffer outgrown by a later capture is kept (not freed) until the
    // context is destroyed, since the graphs captured before still name it
    bool keep = false;
    std::vector<std::unique_ptr<DevBuf>> retired;
    hipError_t ensure(DevBuf& b, size_t bytes) {
        if (bytes <= b.n) return hipSuccess;
        if (keep && b.p) {
            auto old = std::make_unique<DevBuf>();
            std::swap(old->p, b.p);
            std::swap(old->n, b.n);
            retired.push_back(std::move(old));
        }
        return b.ensure(bytes);
    }
};

struct qfec_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    qfec::Tune tune;
    // Decode workspaces.  Eager calls share `ws`; they may enqueue on any stream: every
    // eager use records ws_ev after its kernels, and a use on another stream waits for it, so
    // eager uses are ordered across streams (ws_begin / ws_end).  Calls captured into a graph
    // use `ws_graph` instead, so a replay (on whatever stream it is launched) never shares
    // tables with an eager call; graphs captured on one context share ws_graph, so their
    // replays must be ordered with each other (include/quic_fec.h).
    hipEvent_t ws_ev = nullptr;      // on ws_helper, after the last eager use
    hipEvent_t ws_tmp = nullptr;     // on the last eager use's stream
    hipStream_t ws_helper = nullptr;
    hipStream_t ws_stream = nullptr;
    bool ws_used = false;
    // encode coefficient tables keyed by (k, m, rc): [nchunk][k][rcp]; decode cenc by (k, m)
    std::map<std::tuple<int, int, int>, std::unique_ptr<DevBuf>> enc_tab;
    std::map<std::pair<int, int>, std::unique_ptr<DevBuf>> cenc_tab;
    Workspace ws, ws_graph;
    HostBuf h_stage;
    DevBuf d_stage;
    // host-pointer batches: copy-in / copy-out streams around `stream` (compute), NB
    // rotating device staging buffers so H2D, kernels and D2H of successive chunks overlap
    static constexpr int NB = 3;
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev_in[NB] = {}, ev_done[NB] = {}, ev_out[NB] = {};
    DevBuf pbuf[NB];
    std::mutex mu;   // one caller at a time per context (the reference is single-threaded)
};

namespace {

int set_device(qfec_ctx* c) {
    g_kernels.clear();
    g_grids.clear();
    qfec::launch_timing().first = true;
    QF_HIP(hipSetDevice(c->device));
    return 0;
}

// Order this call's use of the context's decode workspace after the previous eager use
// (which may have been enqueued on another stream).  Not while `st` is capturing into a
// graph: there the calls of one capture are ordered by the capturing stream itself.
// ws_end records ws_ev on the stream of every eager use, right after its kernels, while that
// stream is still eager; ws_begin waits on it when a use arrives on another stream, whatever
// that previous stream is doing now (it may have started a capture since).  A use on the
// same stream as the last needs no wait (stream order).
int ws_begin(qfec_ctx* c, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    QF_HIP(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone) return 0;
    if (c->ws_used && c->ws_stream != st) QF_HIP(hipStreamWaitEvent(st, c->ws_ev, 0));
    return 0;
}
int ws_end(qfec_ctx* c, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    QF_HIP(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone) return 0;
    // HIP refuses any wait on an event whose stream is capturing at the time of the wait, even
    // if the event was recorded before the capture began.  So the completion event lives on a
    // private stream that never captures: it waits for `st` now, while `st` is eager.
    if (!c->ws_helper) QF_HIP(hipStreamCreateWithFlags(&c->ws_helper, hipStreamNonBlocking));
    QF_HIP(hipEventRecord(c->ws_tmp, st));
    QF_HIP(hipStreamWaitEvent(c->ws_helper, c->ws_tmp, 0));
    QF_HIP(hipEventRecord(c->ws_ev, c->ws_helper));
    c->ws_stream = st;
    c->ws_used = true;
    return 0;
}

// The workspace of a call on `st`: the graph workspace while `st` is capturing.
Workspace& ws_for(qfec_ctx* c, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        return c->ws_graph;
    return c->ws;
}

// A stream argument is a plain hipStream_t: NULL is HIP's null (default) stream, as
// everywhere in HIP, so calls order with the caller's other work on that stream.
hipStream_t pick(qfec_ctx*, void* s) { return (hipStream_t)s; }

// Encode coefficient table: output o = chunk*rc + j; o == 0 is the all-ones row.
int get_enc_table(qfec_ctx* c, int k, int m, int rc, const uint8_t** out) {
    auto key = std::make_tuple(k, m, rc);
    auto it = c->enc_tab.find(key);
    if (it != c->enc_tab.end()) { *out = (const uint8_t*)it->second->p; return 0; }
    const int rcp = std::max(rc, 4);
    const int nchunk = (m + rc - 1) / rc;
    std::vector<uint8_t> C((size_t)std::max(m - 1, 1) * k);
    if (cauchy_rows(k, m, C.data())) return fail(-1, "no Cauchy matrix for (k, m)");
    std::vector<uint8_t> tab((size_t)nchunk * k * rcp, 0);
    for (int o = 0; o < m; ++o) {
        const int ch = o / rc, j = o % rc;
        for (int x = 0; x < k; ++x)
            tab[((size_t)ch * k + x) * rcp + j] = o == 0 ? 1 : C[(size_t)(o - 1) * k + x];
    }
    auto buf = std::make_unique<DevBuf>();
    QF_HIP(buf->ensure(tab.size()));
    QF_HIP(hipMemcpy(buf->p, tab.data(), tab.size(), hipMemcpyHostToDevice));
    *out = (const uint8_t*)buf->p;
    c->enc_tab.emplace(key, std::move(buf));
    return 0;
}

int get_cenc(qfec_ctx* c, int k, int m, const uint8_t** out) {
    auto key = std::make_pair(k, m);
    auto it = c->cenc_tab.find(key);
    if (it != c->cenc_tab.end()) { *out = (const uint8_t*)it->second->p; return 0; }
    std::vector<uint8_t> t((size_t)m * k, 1);
    if (k + m <= 256 && m >= 2) {
        if (cauchy_rows(k, m, t.data() + k)) return fail(-1, "no Cauchy matrix for (k, m)");
    }
    auto buf = std::make_unique<DevBuf>();
    QF_HIP(buf->ensure(t.size() + 16));   // dword loads of the last row stay in the buffer
    QF_HIP(hipMemcpy(buf->p, t.data(), t.size(), hipMemcpyHostToDevice));
    *out = (const uint8_t*)buf->p;
    c->cenc_tab.emplace(key, std::move(buf));
    return 0;
}

int decode_workspace(Workspace& W, int k, int rmax, int rc, long long groups) {
    const int rcp = std::max(rc, 4);
    const int nchunk = (rmax + rc - 1) / rc;
    // per group: the apply coefficients, or a syndrome table (bsyn:: / syn::)
    const size_t per = std::max<size_t>({(size_t)nchunk * k * rcp, (size_t)qfec::bsyn::kBytes,
                                         (size_t)qfec::psyn::kBytes});
    QF_HIP(W.ensure(W.dcoef, (size_t)groups * per));
    QF_HIP(W.ensure(W.dslots, (size_t)groups * rmax));
    QF_HIP(W.ensure(W.dnout, (size_t)groups * sizeof(int32_t)));
    return 0;
}

// The (32, 4) x 1352 B syndrome decode (configs B / C): prep, then gf_bsyn.
int bsyn_decode(qfec_ctx* c, const uint8_t* d_blocks, const uint8_t* d_rows_in,
                uint8_t* d_rows_out, uint8_t* d_out, uint8_t* d_rec_rows, int32_t* d_status,
                const uint8_t* cenc, qfec::DecodeWork w, int k, int m, int bb, int rmax,
                long long G, long long out_gstride, const uint8_t* slots, hipStream_t st) {
    QF_HIP(qfec::launch_decode_prep_bsyn(d_rows_in, d_rows_out, d_status, cenc, w.coef, w.slots,
                                         w.nout, d_rec_rows, k, m, bb, rmax, G, st));
    QF_HIP(qfec::launch_gf_bsyn(d_blocks, d_out, w.coef, cenc, slots, w.nout, k, m, bb, G, rmax,
                                out_gstride, st, c->tune));
    return 0;
}

int check_common(qfec_ctx* c, int k, int m, int bb, long long groups) {
    if (!c) return fail(-2, "null context");
    if (!blob_ok()) return fail(-2, "embedded Cauchy tables have the wrong size");
    if (k < 1 || m < 1 || bb < 1 || groups < 0) return fail(-2, "bad k / m / block_bytes / groups");
    if (k > 255) return fail(-2, "k > 255 cannot be tagged by an 8-bit row");
    return 0;
}

int encode_impl(qfec_ctx* c, int k, int m, int bb, long long G, const uint8_t* d_data,
                uint8_t* d_par, hipStream_t st) {
    if (G == 0) return 0;
    if (k <= 1) {   // cauchy_256.cpp:1508-1516
        QF_HIP(qfec::launch_replicate(d_data, d_par, m, bb, G, st));
        return 0;
    }
    // P0 = XOR of the data (:1519-1523).  For m == 1 that is the whole answer; for
    // m > 1 with unsupported parameters the reference still writes it before
    // returning -1 (:1532-1534).
    if (m == 1 || k + m > 256 || bb % 8 != 0) {
        QF_HIP(qfec::launch_xor_encode(d_data, d_par, k, bb, G, (long long)m * bb, st, c->tune));
        return m == 1 ? 0 : fail(-1, "unsupported (k + m > 256 or block_bytes % 8 != 0)");
    }
    const bool aligned = ((uintptr_t)d_data & 15) == 0;
    const int rc = stream_encode_rc(k, m, bb, aligned, c->tune);
    const uint8_t* tab = nullptr;
    int rcode = get_enc_table(c, k, m, rc, &tab);
    if (rcode) return rcode;
    if ((m <= rc || rc == 8) && qfec::gf_stream_supported(k, m, bb, rc, false, c->tune) &&
        aligned) {
        QF_HIP(qfec::launch_gf_stream(d_data, d_par, tab, nullptr, nullptr, k, m, bb, G, rc, 0, 0,
                                      (long long)m * bb, false, st, c->tune));
        return 0;
    }
    if (qfec::gf_dcol_supported(k, m, bb, c->tune) && ((uintptr_t)d_data & 15) == 0) {
        QF_HIP(qfec::launch_gf_dcol_encode(d_data, d_par, k, m, bb, G, (long long)m * bb, st,
                                           c->tune));
        return 0;
    }
    QF_HIP(qfec::launch_gf_encode(d_data, d_par, tab, k, m, bb, G, rc, st, c->tune));
    return 0;
}

int decode_body(qfec_ctx* c, int k, int m, int bb, long long G, const uint8_t* d_blocks,
                const uint8_t* d_rows_in, uint8_t* d_out, uint8_t* d_rows_out, int32_t* d_status,
                hipStream_t st) {
    if (k <= 1) {   // cauchy_256.cpp:1257-1261
        QF_HIP(qfec::launch_rows_k1(d_rows_in, d_rows_out, d_status, G, st));
        return 0;
    }
    Workspace& W = ws_for(c, st);
    if (m == 1) {   // :1264-1267
        QF_HIP(W.ensure(W.dslots, (size_t)G));
        QF_HIP(qfec::launch_xor_decode(d_blocks, d_out, d_rows_in, d_rows_out, d_status,
                                       (uint8_t*)W.dslots.p, k, bb, G, st, c->tune));
        return 0;
    }
    const int rmax = std::min(k, m);
    const int rc = stream_decode_rc(rmax);
    const int nchunk = (rmax + rc - 1) / rc;
    const uint8_t* cenc = nullptr;
    int r = get_cenc(c, k, m, &cenc);
    if (r) return r;
    if ((r = decode_workspace(W, k, rmax, rc, G))) return r;
    qfec::DecodeWork w{(uint8_t*)W.dcoef.p, (uint8_t*)W.dslots.p, (int32_t*)W.dnout.p};
    const long long tab_gstride = (long long)nchunk * k * std::max(rc, 4);
    const bool dcol = qfec::gf_dcol_supported(k, m, bb, c->tune) && rmax <= 16;
    if (dcol && ((uintptr_t)d_blocks & 15) == 0) {
        // compiled (128, 16) code: syndromes, then the r x r solve (reads precede stores
        // within a group, so in place needs no scratch)
        QF_HIP(qfec::launch_decode_prep(d_rows_in, d_rows_out, d_status, cenc, w, k, m, bb, rc,
                                        rmax, G, st, c->tune, nullptr, true));
        QF_HIP(qfec::launch_gf_dcol_syndrome(d_blocks, d_out, w.coef, w.slots, w.nout, cenc, k,
                                             m, bb, G, rmax, tab_gstride, (long long)k * bb, st,
                                             c->tune));
        return 0;
    }
    if (qfec::gf_psyn_supported(k, m, bb, rmax, c->tune) && ((uintptr_t)d_blocks & 15) == 0) {
        // compiled QuicR preset code: syndromes of every parity row, then Gauss-Jordan in
        // place (a group's stores follow all of its reads: in place needs no scratch)
        QF_HIP(qfec::launch_decode_prep_psyn(d_rows_in, d_rows_out, d_status, cenc, w.coef,
                                             w.slots, w.nout, nullptr, k, m, bb, rmax, G, st));
        QF_HIP(qfec::launch_gf_psyn(d_blocks, d_out, w.coef, cenc, w.slots, w.nout, k, m, bb, G,
                                    rmax, (long long)k * bb, st, c->tune));
        return 0;
    }
    if (qfec::gf_bsyn_supported(k, m, bb, rmax, c->tune) && ((uintptr_t)d_blocks & 15) == 0) {
        // compiled (32, 4) code: syndromes of every parity row, then the r x r solve (a
        // group's stores follow all of its reads: in place needs no scratch)
        return bsyn_decode(c, d_blocks, d_rows_in, d_rows_out, d_out, nullptr, d_status, cenc,
                           w, k, m, bb, rmax, G, (long long)k * bb, w.slots, st);
    }
    QF_HIP(qfec::launch_decode_prep(d_rows_in, d_rows_out, d_status, cenc, w, k, m, bb, rc, rmax,
                                    G, st, c->tune));
    if (bb % 8 != 0 || k + m > 256) return 0;   // every group is a no-op or status -1
    if (qfec::gf_stream_supported(k, m, bb, rc, true, c->tune) &&
        ((uintptr_t)d_blocks & 15) == 0) {
        const int rcp = std::max(rc, 4);
        if (nchunk == 1 || d_out != d_blocks) {
            // one chunk: a group's stores follow all of its reads, so in place needs no
            // scratch; several chunks (units on different waves) write out of place only
            QF_HIP(qfec::launch_gf_stream(d_blocks, d_out, w.coef, w.slots, w.nout, k, m, bb, G,
                                          rc, rmax, (long long)nchunk * k * rcp,
                                          (long long)k * bb, true, st, c->tune));
            return 0;
        }
        // in place with several chunks: the recovered blocks go to scratch first, then to
        // their slots (a later chunk reads slots an earlier one would have overwritten)
        QF_HIP(W.ensure(W.dscratch, (size_t)G * rmax * bb));
        QF_HIP(qfec::launch_gf_stream(d_blocks, (uint8_t*)W.dscratch.p, w.coef, nullptr, w.nout,
                                      k, m, bb, G, rc, rmax, (long long)nchunk * k * rcp,
                                      (long long)rmax * bb, true, st, c->tune));
        QF_HIP(qfec::launch_scatter_recovered((const uint8_t*)W.dscratch.p, d_out, w, k, bb,
                                              rmax, G, st));
        return 0;
    }
    if (nchunk > 1 && d_out == d_blocks) {
        // in place with several output chunks: a later chunk would read slots an earlier
        // chunk already overwrote, so stage the recovered blocks first
        QF_HIP(W.ensure(W.dscratch, (size_t)G * rmax * bb));
        QF_HIP(qfec::launch_gf_decode_scratch(d_blocks, (uint8_t*)W.dscratch.p, w, k, m, bb, G,
                                              rc, rmax, st, c->tune));
        QF_HIP(qfec::launch_scatter_recovered((const uint8_t*)W.dscratch.p, d_out, w, k, bb,
                                              rmax, G, st));
        return 0;
    }
    QF_HIP(qfec::launch_gf_decode(d_blocks, d_out, w, k, m, bb, G, rc, rmax, st, c->tune));
    return 0;
}

int decode_impl(qfec_ctx* c, int k, int m, int bb, long long G, const uint8_t* d_blocks,
                const uint8_t* d_rows_in, uint8_t* d_out, uint8_t* d_rows_out, int32_t* d_status,
                hipStream_t st) {
    if (G == 0) return 0;
    int r = ws_begin(c, st);
    if (r) return r;
    r = decode_body(c, k, m, bb, G, d_blocks, d_rows_in, d_out, d_rows_out, d_status, st);
    const int r2 = ws_end(c, st);
    return r ? r : r2;
}

// Recovered-blocks layout (qfec_decode_batch_recovered): the same decode, but recovered
// block j of group g goes to d_rec + (g * rmax + j) * bb and its data row to
// d_rec_rows[g * rmax + j] (ascending, 255 past the erasure count); blocks and row tags
// are left as they are.  This is what the receiver consumes (getRevivedPackets,
// quic_fec_group.cc:280-293, only extracts the missing packets), and the writes are dense.
int decode_recovered_body(qfec_ctx* c, int k, int m, int bb, long long G,
                          const uint8_t* d_blocks, const uint8_t* d_rows_in, uint8_t* d_rec,
                          uint8_t* d_rec_rows, int32_t* d_status, hipStream_t st) {
    const int rmax = std::min(k, m);
    if (k <= 1) {
        QF_HIP(qfec::launch_rec_k1(d_blocks, d_rows_in, d_rec, d_rec_rows, d_status, bb, rmax, G,
                                   st));
        return 0;
    }
    Workspace& W = ws_for(c, st);
    if (m == 1) {
        QF_HIP(W.ensure(W.dslots, (size_t)G));
        QF_HIP(qfec::launch_xor_decode(d_blocks, d_rec, d_rows_in, d_rec_rows, d_status,
                                       (uint8_t*)W.dslots.p, k, bb, G, st, c->tune, true));
        return 0;
    }
    const int rc = stream_decode_rc(rmax);
    const uint8_t* cenc = nullptr;
    int r = get_cenc(c, k, m, &cenc);
    if (r) return r;
    if ((r = decode_workspace(W, k, rmax, rc, G))) return r;
    qfec::DecodeWork w{(uint8_t*)W.dcoef.p, (uint8_t*)W.dslots.p, (int32_t*)W.dnout.p};
    const bool dcol = qfec::gf_dcol_supported(k, m, bb, c->tune) && rmax <= 16;
    if (dcol && ((uintptr_t)d_blocks & 15) == 0) {
        const int nchunk = (rmax + rc - 1) / rc;
        QF_HIP(qfec::launch_decode_prep(d_rows_in, nullptr, d_status, cenc, w, k, m, bb, rc, rmax,
                                        G, st, c->tune, d_rec_rows, true));
        QF_HIP(qfec::launch_gf_dcol_syndrome(d_blocks, d_rec, w.coef, nullptr, w.nout, cenc, k, m,
                                             bb, G, rmax, (long long)nchunk * k * std::max(rc, 4),
                                             (long long)rmax * bb, st, c->tune));
        return 0;
    }
    if (qfec::gf_psyn_supported(k, m, bb, rmax, c->tune) && ((uintptr_t)d_blocks & 15) == 0) {
        QF_HIP(qfec::launch_decode_prep_psyn(d_rows_in, nullptr, d_status, cenc, w.coef, w.slots,
                                             w.nout, d_rec_rows, k, m, bb, rmax, G, st));
        QF_HIP(qfec::launch_gf_psyn(d_blocks, d_rec, w.coef, cenc, nullptr, w.nout, k, m, bb, G,
                                    rmax, (long long)rmax * bb, st, c->tune));
        return 0;
    }
    if (qfec::gf_bsyn_supported(k, m, bb, rmax, c->tune) && ((uintptr_t)d_blocks & 15) == 0) {
        return bsyn_decode(c, d_blocks, d_rows_in, nullptr, d_rec, d_rec_rows, d_status, cenc,
                           w, k, m, bb, rmax, G, (long long)rmax * bb, nullptr, st);
    }
    QF_HIP(qfec::launch_decode_prep(d_rows_in, nullptr, d_status, cenc, w, k, m, bb, rc, rmax, G,
                                    st, c->tune, d_rec_rows));
    if (bb % 8 != 0 || k + m > 256) return 0;   // every group is a no-op or status -1
    if (qfec::gf_stream_supported(k, m, bb, rc, true, c->tune) &&
        ((uintptr_t)d_blocks & 15) == 0) {
        const int rcp = std::max(rc, 4);
        const int nchunk = (rmax + rc - 1) / rc;
        QF_HIP(qfec::launch_gf_stream(d_blocks, d_rec, w.coef, nullptr, w.nout, k, m, bb, G, rc,
                                      rmax, (long long)nchunk * k * rcp, (long long)rmax * bb,
                                      true, st, c->tune));
        return 0;
    }
    QF_HIP(qfec::launch_gf_decode_scratch(d_blocks, d_rec, w, k, m, bb, G, rc, rmax, st,
                                          c->tune));
    return 0;
}

int decode_recovered_impl(qfec_ctx* c, int k, int m, int bb, long long G,
                          const uint8_t* d_blocks, const uint8_t* d_rows_in, uint8_t* d_rec,
                          uint8_t* d_rec_rows, int32_t* d_status, hipStream_t st) {
    if (G == 0) return 0;
    int r = ws_begin(c, st);
    if (r) return r;
    r = decode_recovered_body(c, k, m, bb, G, d_blocks, d_rows_in, d_rec, d_rec_rows, d_status,
                              st);
    const int r2 = ws_end(c, st);
    return r ? r : r2;
}

// Host-pointer batches, chunked and pipelined: chunk i's H2D (s_in), kernels (stream)
// and D2H (s_out) are ordered by events, and NB staging buffers rotate, so the copy-in of
// chunk i + 1 and the copy-out of chunk i - 1 overlap the kernels of chunk i (PCIe is
// full duplex).  The kernels of all chunks stay on one stream, so the decode workspace is
// never shared by two chunks in flight.  Chunk size: the host_chunk_mb option (64 MiB), and
// at least the host_min_groups option's groups (512).
// fn(g0, n, buf, phase): phase 0 enqueues the H2D, 1 the kernels, 2 the D2H.
template <class F>
int host_pipeline_body(qfec_ctx* c, long long groups, size_t per_group, size_t slack, F&& fn) {
    if (!c->s_in) {
        QF_HIP(hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking));
        QF_HIP(hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
        for (int b = 0; b < qfec_ctx::NB; ++b) {
            QF_HIP(hipEventCreateWithFlags(&c->ev_in[b], hipEventDisableTiming));
            QF_HIP(hipEventCreateWithFlags(&c->ev_done[b], hipEventDisableTiming));
            QF_HIP(hipEventCreateWithFlags(&c->ev_out[b], hipEventDisableTiming));
        }
    }
    // at least host_min_groups groups per chunk (up to 2 GiB of staging per buffer): a
    // 64 MiB chunk of D's 1.2 MB groups is 54 groups, too few to fill the device (D at
    // 16,384 groups: 16.1 GiB/s with 64 MiB chunks, 22.9 with 256 MiB, 23.3 with 1 GiB).
    // Both are options, so a caller (and the tests) can still force small chunks.
    const size_t target = (size_t)std::max(1, c->tune.host_chunk_mb) << 20;
    const long long by_bytes = (long long)(target / per_group);
    const long long floor_g = std::min<long long>(std::max(1, c->tune.host_min_groups),
                                                  (long long)((2ull << 30) / per_group));
    const long long chunk =
        std::max<long long>(1, std::min<long long>(groups, std::max(by_bytes, floor_g)));
    const size_t bytes = (size_t)chunk * per_group + slack;
    for (int b = 0; b < qfec_ctx::NB; ++b) QF_HIP(c->pbuf[b].ensure(bytes));
    int i = 0;
    for (long long g0 = 0; g0 < groups; g0 += chunk, ++i) {
        const long long n = std::min(chunk, groups - g0);
        const int b = i % qfec_ctx::NB;
        uint8_t* buf = (uint8_t*)c->pbuf[b].p;
        if (i >= qfec_ctx::NB) QF_HIP(hipStreamWaitEvent(c->s_in, c->ev_out[b], 0));
        int r = fn(g0, n, buf, 0);
        if (r) return r;
        QF_HIP(hipEventRecord(c->ev_in[b], c->s_in));
        QF_HIP(hipStreamWaitEvent(c->stream, c->ev_in[b], 0));
        if ((r = fn(g0, n, buf, 1))) return r;
        QF_HIP(hipEventRecord(c->ev_done[b], c->stream));
        QF_HIP(hipStreamWaitEvent(c->s_out, c->ev_done[b], 0));
        if ((r = fn(g0, n, buf, 2))) return r;
        QF_HIP(hipEventRecord(c->ev_out[b], c->s_out));
    }
    QF_HIP(hipStreamSynchronize(c->s_out));
    return 0;
}

// On any error, drain all three streams before returning, so no copy of an earlier chunk
// still writes into the caller's host buffers after the call has returned.
template <class F>
int host_pipeline(qfec_ctx* c, long long groups, size_t per_group, F&& fn, size_t slack = 16) {
    // the kernels of every chunk run on the context stream: order them after the last eager
    // use of the decode workspace, and the next use after them
    int r = ws_begin(c, c->stream);
    if (!r) r = host_pipeline_body(c, groups, per_group, slack, fn);
    if (!r) r = ws_end(c, c->stream);
    if (r)
        for (hipStream_t s : {c->s_in, c->stream, c->s_out})
            if (s) (void)hipStreamSynchronize(s);
    return r;
}

// Default context for the single-group drop-ins (created on the caller's current device;
// QFEC_DEVICE names another, read once when the context is first needed).
std::once_flag g_default_once;
qfec_ctx* g_default = nullptr;
int g_default_rc = 0;

int default_ctx(qfec_ctx** out) {
    std::call_once(g_default_once, [] {
        int dev = 0;
        if (const char* e = getenv("QFEC_DEVICE")) dev = atoi(e);
        else if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        g_default_rc = qfec_ctx_create(dev, &g_default);
    });
    *out = g_default;
    if (!g_default) return g_default_rc ? g_default_rc : fail(-2, "no default GPU context");
    return 0;
}

}  // namespace

namespace qfec {
LaunchTiming& launch_timing() {
    static thread_local LaunchTiming t;
    return t;
}

void note_kernel(const char* name) {
    // a host-pointer batch launches the same kernels once per chunk: list each once
    const std::string n(name);
    size_t at = 0;
    while ((at = g_kernels.find(n, at)) != std::string::npos) {
        const size_t end = at + n.size();
        if ((at == 0 || g_kernels.compare(at - 3, 3, " + ") == 0) &&
            (end == g_kernels.size() || g_kernels.compare(end, 3, " + ") == 0))
            return;
        at = end;
    }
    if (!g_kernels.empty()) g_kernels += " + ";
    g_kernels += n;
}

void note_grid(const char* name, unsigned grid) {
    if (!g_grids.empty()) g_grids += " ";
    g_grids += std::string(name) + "=" + std::to_string(grid);
}

int resident_blocks(const void* kern, int threads, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t>, int> cache;
    const auto key = std::make_tuple(kern, threads, lds);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, lds) != hipSuccess || n < 1)
        n = 1;
    cache.emplace(key, n);
    return n;
}
}  // namespace qfec

namespace {

// NullDecrypter on every packet of each group, placement into the receive set, the
// recovered-blocks decode, the unfilled-group status (qfec_open_decode_batch)
int open_decode_impl(qfec_ctx* c, int k, int m, int bb, long long groups, const uint8_t* d_pkt,
                     long long pkt_stride, const int* d_pkt_len, const int* d_ad_len,
                     int ad_len_all, uint8_t* d_blocks, uint8_t* d_rows, int* d_open_len,
                     uint8_t* d_rec, uint8_t* d_rec_rows, int* d_status, hipStream_t st) {
    QF_HIP(qfec::launch_open_groups(k, m, bb, groups, d_pkt, pkt_stride,
                                    (const int32_t*)d_pkt_len, (const int32_t*)d_ad_len,
                                    ad_len_all, d_blocks, d_rows, (int32_t*)d_open_len, st));
    int rc = decode_recovered_impl(c, k, m, bb, groups, d_blocks, d_rows, d_rec, d_rec_rows,
                                   (int32_t*)d_status, st);
    if (rc) return rc;
    QF_HIP(qfec::launch_open_status(k, std::min(k, m), groups, d_rows, d_rec_rows,
                                    (int32_t*)d_status, st));
    return 0;
}

// Carves consecutive 256-byte aligned sub-buffers out of one staging buffer.
struct Carve {
    uint8_t* p;
    uint8_t* take(size_t bytes) {
        uint8_t* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return r;
    }
};
constexpr size_t kCarveSlack = 16 * 256;   // alignment padding of up to 16 sub-buffers

}  // namespace

// ======================================================================== C ABI
extern "C" {

int qfec_version(void) { return 1; }

const char* qfec_last_error(void) { return g_err.c_str(); }

const char* qfec_last_kernels(void) { return g_kernels.c_str(); }

const char* qfec_last_grids(void) { return g_grids.c_str(); }

int qfec_set_timing_events(void* start_event, void* stop_event) {
    if (!start_event != !stop_event) return fail(-2, "set both timing events or neither");
    qfec::LaunchTiming& t = qfec::launch_timing();
    t.start = (hipEvent_t)start_event;
    t.stop = (hipEvent_t)stop_event;
    t.first = true;
    return 0;
}

int qfec_ctx_set_option(qfec_ctx* c, const char* name, int value) {
    if (!c || !name) return fail(-2, "null context or option name");
    std::lock_guard<std::mutex> lk(c->mu);
    struct Opt { const char* n; int* p; int lo, hi; };
    qfec::Tune& t = c->tune;
    const Opt opts[] = {
        {"xor_slots", &t.xor_slots, 2, 4},     {"xor_waves", &t.xor_waves, 1, 4},
        {"dma", &t.dma, 0, 1},                 {"stream", &t.stream, 0, 1},
        {"stream_ring", &t.stream_ring, 4, 36}, {"stream_grid", &t.stream_grid, 0, 1 << 20},
        {"const_enc", &t.const_enc, 0, 1},     {"stream_static", &t.stream_static, 0, 1},
        {"ring_wide", &t.ring_wide, 0, 1}, {"psyn_wide", &t.psyn_wide, 0, 2},
        {"ring_split", &t.ring_split, 0, 1},
        {"dcol", &t.dcol, 0, 1},               {"dcol_grid", &t.dcol_grid, 0, 1 << 20},
        {"dcol_depth", &t.dcol_depth, 6, 8},
        {"bsyn", &t.bsyn, 0, 1},               {"bsyn_depth", &t.bsyn_depth, 3, 7},
        {"psyn", &t.psyn, 0, 1},
        {"pd", &t.pd, 1, 3},                   {"flat", &t.flat, 0, 1},
        {"enc_rc", &t.enc_rc, 2, 8},           {"prep_lane", &t.prep_lane, 0, 1},
        {"host_chunk_mb", &t.host_chunk_mb, 1, 4096},
        {"host_min_groups", &t.host_min_groups, 1, 1 << 20},
        {"ring_wg", &t.ring_wg, -1, 1 << 20}, {"bsyn_wg", &t.bsyn_wg, -1, 1 << 20},
        {"psyn_wg", &t.psyn_wg, 0, 1 << 20},  {"dcol_wg", &t.dcol_wg, 0, 1 << 20},
        {"stream_wg", &t.stream_wg, -1, 1 << 20},
        {"xor_wg", &t.xor_wg, 0, 1 << 20},
    };
    for (const Opt& o : opts) {
        if (strcmp(o.n, name) != 0) continue;
        if (value < o.lo || value > o.hi || (o.p == &t.enc_rc && (value & (value - 1))) ||
            (o.p == &t.dcol_depth && value == 7) || (o.p == &t.bsyn_depth && !(value & 1)))
            return fail(-2, std::string("option value out of range: ") + name);
        *o.p = value;
        return 0;
    }
    return fail(-2, std::string("unknown option: ") + name);
}

int qfec_ctx_get_option(qfec_ctx* c, const char* name, int* value) {
    if (!c || !name || !value) return fail(-2, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    const qfec::Tune& t = c->tune;
    const std::pair<const char*, int> opts[] = {
        {"cus", t.cus}, {"xor_slots", t.xor_slots}, {"xor_waves", t.xor_waves}, {"dma", t.dma},
        {"stream", t.stream}, {"stream_ring", t.stream_ring}, {"stream_grid", t.stream_grid},
        {"const_enc", t.const_enc}, {"stream_static", t.stream_static}, {"ring_wide", t.ring_wide}, {"psyn_wide", t.psyn_wide}, {"ring_split", t.ring_split},
        {"dcol", t.dcol},
        {"dcol_grid", t.dcol_grid}, {"dcol_depth", t.dcol_depth},
        {"bsyn", t.bsyn}, {"bsyn_depth", t.bsyn_depth}, {"psyn", t.psyn},
        {"pd", t.pd}, {"flat", t.flat}, {"enc_rc", t.enc_rc}, {"prep_lane", t.prep_lane},
        {"host_chunk_mb", t.host_chunk_mb}, {"host_min_groups", t.host_min_groups},
        {"ring_wg", t.ring_wg}, {"bsyn_wg", t.bsyn_wg}, {"psyn_wg", t.psyn_wg}, {"stream_wg", t.stream_wg},
        {"dcol_wg", t.dcol_wg}, {"xor_wg", t.xor_wg},
    };
    for (const auto& o : opts)
        if (strcmp(o.first, name) == 0) { *value = o.second; return 0; }
    return fail(-2, std::string("unknown option: ") + name);
}

int qfec_cauchy_matrix(int k, int m, unsigned char* out) {
    if (!blob_ok()) return fail(-2, "embedded Cauchy tables have the wrong size");
    return cauchy_rows(k, m, out);
}

int qfec_ctx_create(int device, qfec_ctx** out) {
    if (!out) return fail(-2, "null out");
    *out = nullptr;
    int n = 0;
    QF_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(-2, "no such HIP device");
    auto c = std::make_unique<qfec_ctx>();
    c->device = device;
    c->ws_graph.keep = true;
    QF_HIP(hipSetDevice(device));
    int cus = 0;
    QF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    c->tune.cus = cus > 0 ? cus : 256;
    QF_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    QF_HIP(hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming));
    QF_HIP(hipEventCreateWithFlags(&c->ws_tmp, hipEventDisableTiming));
    *out = c.release();
    return 0;
}

void qfec_ctx_destroy(qfec_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // the last use of the workspace may be on any stream the caller used (and may have
    // destroyed since), and a graph replay may still read the graph workspace: wait for the
    // whole device rather than for a stored stream handle
    if (c->ws_used || c->ws_graph.dslots.p) (void)hipDeviceSynchronize();
    for (hipStream_t s : {c->stream, c->s_in, c->s_out})
        if (s) (void)hipStreamSynchronize(s);
    if (c->ws_ev) (void)hipEventDestroy(c->ws_ev);
    if (c->ws_tmp) (void)hipEventDestroy(c->ws_tmp);
    for (int b = 0; b < qfec_ctx::NB; ++b)
        for (hipEvent_t e : {c->ev_in[b], c->ev_done[b], c->ev_out[b]})
            if (e) (void)hipEventDestroy(e);
    for (hipStream_t s : {c->stream, c->s_in, c->s_out, c->ws_helper})
        if (s) (void)hipStreamDestroy(s);
    delete c;
}

int qfec_encode_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                      const unsigned char* d_data, unsigned char* d_parity, void* stream) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups && (!d_data || !d_parity)) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    return encode_impl(c, k, m, bb, groups, d_data, d_parity, pick(c, stream));
}

int qfec_decode_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                      const unsigned char* d_blocks, const unsigned char* d_rows_in,
                      unsigned char* d_out, unsigned char* d_rows_out, int* d_status,
                      void* stream) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups && (!d_blocks || !d_rows_in || !d_out || !d_rows_out))
        return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    return decode_impl(c, k, m, bb, groups, d_blocks, d_rows_in, d_out, d_rows_out,
                       (int32_t*)d_status, pick(c, stream));
}

int qfec_decode_batch_recovered(qfec_ctx* c, int k, int m, int bb, long long groups,
                                const unsigned char* d_blocks, const unsigned char* d_rows_in,
                                unsigned char* d_rec, unsigned char* d_rec_rows, int* d_status,
                                void* stream) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups && (!d_blocks || !d_rows_in || !d_rec || !d_rec_rows))
        return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    return decode_recovered_impl(c, k, m, bb, groups, d_blocks, d_rows_in, d_rec, d_rec_rows,
                                 (int32_t*)d_status, pick(c, stream));
}

// ---- packet protection (pp_null.hip; null_encrypter.cc:23-43, null_decrypter.cc)
int qfec_null_seal_batch(qfec_ctx* c, long long n, const unsigned char* d_ad, long long ad_stride,
                         const int* d_ad_len, int ad_len_all, const unsigned char* d_pt,
                         long long pt_stride, const int* d_pt_len, int pt_len_all,
                         unsigned char* d_out, long long out_stride, int* d_out_len,
                         void* stream) {
    if (!c) return fail(-2, "null context");
    if (n < 0 || ad_stride < 0 || pt_stride < 0 || out_stride < 0) return fail(-2, "bad n / stride");
    if (n && (!d_out || !d_out_len || (!d_ad && (d_ad_len || ad_len_all)) || (!d_pt && (d_pt_len || pt_len_all))))
        return fail(-2, "null buffer");
    if ((((uintptr_t)d_out) | (uintptr_t)out_stride) & 3) return fail(-2, "out / out_stride not 4-byte aligned");
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    QF_HIP(qfec::launch_null_seal_h(n, d_ad, ad_stride, (const int32_t*)d_ad_len, ad_len_all, d_pt,
                                  pt_stride, (const int32_t*)d_pt_len, pt_len_all, d_out,
                                  out_stride, (int32_t*)d_out_len, pick(c, stream)));
    return 0;
}

int qfec_null_open_batch(qfec_ctx* c, long long n, const unsigned char* d_pkt, long long pkt_stride,
                         const int* d_pkt_len, int pkt_len_all, const int* d_ad_len,
                         int ad_len_all, unsigned char* d_out, long long out_stride,
                         int* d_out_len, void* stream) {
    if (!c) return fail(-2, "null context");
    if (n < 0 || pkt_stride < 0 || out_stride < 0) return fail(-2, "bad n / stride");
    if (n && (!d_pkt || !d_out || !d_out_len)) return fail(-2, "null buffer");
    if ((((uintptr_t)d_out) | (uintptr_t)out_stride) & 3) return fail(-2, "out / out_stride not 4-byte aligned");
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    QF_HIP(qfec::launch_null_open_h(n, d_pkt, pkt_stride, (const int32_t*)d_pkt_len, pkt_len_all,
                                  (const int32_t*)d_ad_len, ad_len_all, d_out, out_stride,
                                  (int32_t*)d_out_len, pick(c, stream)));
    return 0;
}

int qfec_encode_seal_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                           const unsigned char* d_data, unsigned char* d_parity,
                           const unsigned char* d_hdr, long long hdr_stride, const int* d_hdr_len,
                           int hdr_len_all, unsigned char* d_pkt, long long pkt_stride,
                           int* d_pkt_len, void* stream) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups && (!d_data || !d_parity || !d_pkt || !d_pkt_len || (!d_hdr && (d_hdr_len || hdr_len_all))))
        return fail(-2, "null buffer");
    if (hdr_stride < 0 || pkt_stride < 0) return fail(-2, "bad stride");
    if ((((uintptr_t)d_pkt) | (uintptr_t)pkt_stride) & 3) return fail(-2, "pkt / pkt_stride not 4-byte aligned");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const hipStream_t st = pick(c, stream);
    // SerializeFec (quic_packet_creator.cc:935-957): parity packets from the group's encode,
    // each sealed with its packet header as the associated data; packet (g, i) = g * m + i
    if ((rc = encode_impl(c, k, m, bb, groups, d_data, d_parity, st))) return rc;
    QF_HIP(qfec::launch_null_seal_h(groups * m, d_hdr, hdr_stride, (const int32_t*)d_hdr_len,
                                  hdr_len_all, d_parity, bb, nullptr, bb, d_pkt, pkt_stride,
                                  (int32_t*)d_pkt_len, st));
    return 0;
}

// Every packet of each group, data and FEC, in one launch (quic_packet_creator.cc:733-736
// seals each data packet, :948-953 each FEC packet); packet (g, i) = g * (k + m) + i.
static int seal_groups_args(qfec_ctx* c, int k, int m, int bb, long long groups,
                            const unsigned char* d_data, const unsigned char* d_parity,
                            const unsigned char* d_hdr, long long hdr_stride, const int* d_hdr_len,
                            int hdr_len_all, const int* d_pt_len, int pt_len_all,
                            const unsigned char* d_pkt, long long pkt_stride, const int* d_pkt_len) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (k + m > 256) return fail(-2, "k + m > 256");
    if (groups && (!d_data || !d_parity || !d_pkt || !d_pkt_len || (!d_hdr && (d_hdr_len || hdr_len_all))))
        return fail(-2, "null buffer");
    if (hdr_stride < 0 || pkt_stride < 0) return fail(-2, "bad stride");
    if (!d_pt_len && (pt_len_all < 0 || pt_len_all > bb)) return fail(-2, "pt_len_all outside 0..block_bytes");
    if ((((uintptr_t)d_pkt) | (uintptr_t)pkt_stride) & 3) return fail(-2, "pkt / pkt_stride not 4-byte aligned");
    return 0;
}

int qfec_seal_groups_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                           const unsigned char* d_data, const unsigned char* d_parity,
                           const unsigned char* d_hdr, long long hdr_stride, const int* d_hdr_len,
                           int hdr_len_all, const int* d_pt_len, int pt_len_all,
                           unsigned char* d_pkt, long long pkt_stride, int* d_pkt_len, void* stream) {
    int rc = seal_groups_args(c, k, m, bb, groups, d_data, d_parity, d_hdr, hdr_stride, d_hdr_len,
                              hdr_len_all, d_pt_len, pt_len_all, d_pkt, pkt_stride, d_pkt_len);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    QF_HIP(qfec::launch_null_seal_groups(k, m, bb, groups, d_data, d_parity, d_hdr, hdr_stride,
                                         (const int32_t*)d_hdr_len, hdr_len_all,
                                         (const int32_t*)d_pt_len, pt_len_all, d_pkt, pkt_stride,
                                         (int32_t*)d_pkt_len, pick(c, stream)));
    return 0;
}

int qfec_encode_seal_groups_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                                  const unsigned char* d_data, unsigned char* d_parity,
                                  const unsigned char* d_hdr, long long hdr_stride,
                                  const int* d_hdr_len, int hdr_len_all, const int* d_pt_len,
                                  int pt_len_all, unsigned char* d_pkt, long long pkt_stride,
                                  int* d_pkt_len, void* stream) {
    int rc = seal_groups_args(c, k, m, bb, groups, d_data, d_parity, d_hdr, hdr_stride, d_hdr_len,
                              hdr_len_all, d_pt_len, pt_len_all, d_pkt, pkt_stride, d_pkt_len);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const hipStream_t st = pick(c, stream);
    if ((rc = encode_impl(c, k, m, bb, groups, d_data, d_parity, st))) return rc;
    QF_HIP(qfec::launch_null_seal_groups(k, m, bb, groups, d_data, d_parity, d_hdr, hdr_stride,
                                         (const int32_t*)d_hdr_len, hdr_len_all,
                                         (const int32_t*)d_pt_len, pt_len_all, d_pkt, pkt_stride,
                                         (int32_t*)d_pkt_len, st));
    return 0;
}

// Receiver: open every packet of each group (quic_framer.cc:657 decrypts before the group
// sees a packet), place the data plaintexts, fill the holes with opened FEC packets, decode.
int qfec_open_decode_batch(qfec_ctx* c, int k, int m, int bb, long long groups,
                           const unsigned char* d_pkt, long long pkt_stride, const int* d_pkt_len,
                           const int* d_ad_len, int ad_len_all, unsigned char* d_blocks,
                           unsigned char* d_rows, int* d_open_len, unsigned char* d_rec,
                           unsigned char* d_rec_rows, int* d_status, void* stream) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (k + m > 255) return fail(-2, "k + m > 255 (row tag 255 marks an unfilled slot)");
    if (groups && (!d_pkt || !d_pkt_len || !d_blocks || !d_rows || !d_open_len || !d_rec || !d_rec_rows))
        return fail(-2, "null buffer");
    if (pkt_stride <= 0 && groups) return fail(-2, "bad pkt_stride");
    if (!d_ad_len && ad_len_all < 0) return fail(-2, "bad ad_len_all");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const hipStream_t st = pick(c, stream);
    if ((rc = ws_begin(c, st))) return rc;
    if ((rc = open_decode_impl(c, k, m, bb, groups, d_pkt, pkt_stride, d_pkt_len, d_ad_len,
                               ad_len_all, d_blocks, d_rows, d_open_len, d_rec, d_rec_rows,
                               d_status, st)))
        return rc;
    return ws_end(c, st);
}

int qfec_decode_batch_recovered_host(qfec_ctx* c, int k, int m, int bb, long long groups,
                                     const unsigned char* h_blocks, const unsigned char* h_rows,
                                     unsigned char* h_rec, unsigned char* h_rec_rows,
                                     int* h_status) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups == 0) return 0;
    if (!h_blocks || !h_rows || !h_rec || !h_rec_rows) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const int rmax = std::min(k, m);
    const size_t blk_g = (size_t)k * bb, rec_g = (size_t)rmax * bb;
    // per group: blocks, recovered blocks, row tags, recovered rows, status (aligned)
    const size_t per = blk_g + rec_g + k + rmax + sizeof(int32_t);
    return host_pipeline(c, groups, per, [&](long long g0, long long n, uint8_t* buf,
                                             int phase) -> int {
        uint8_t* db = buf;
        uint8_t* dre = db + (size_t)n * blk_g;
        uint8_t* dr = dre + (size_t)n * rec_g;
        uint8_t* drr = dr + (size_t)n * k;
        int32_t* ds = (int32_t*)(((uintptr_t)(drr + (size_t)n * rmax) + 3) & ~(uintptr_t)3);
        if (phase == 0) {
            QF_HIP(hipMemcpyAsync(db, h_blocks + (size_t)g0 * blk_g, (size_t)n * blk_g,
                                  hipMemcpyHostToDevice, c->s_in));
            QF_HIP(hipMemcpyAsync(dr, h_rows + (size_t)g0 * k, (size_t)n * k,
                                  hipMemcpyHostToDevice, c->s_in));
        } else if (phase == 1) {
            const int r = decode_recovered_impl(c, k, m, bb, n, db, dr, dre, drr, ds, c->stream);
            if (r) return r;
        } else {
            QF_HIP(hipMemcpyAsync(h_rec + (size_t)g0 * rec_g, dre, (size_t)n * rec_g,
                                  hipMemcpyDeviceToHost, c->s_out));
            QF_HIP(hipMemcpyAsync(h_rec_rows + (size_t)g0 * rmax, drr, (size_t)n * rmax,
                                  hipMemcpyDeviceToHost, c->s_out));
            if (h_status)
                QF_HIP(hipMemcpyAsync(h_status + g0, ds, (size_t)n * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, c->s_out));
        }
        return 0;
    });
}

// Sender, host memory to host memory: data blocks and packet headers in, every sealed packet
// of each group out (the parity never leaves the device).  Chunked and pipelined as the
// other host batches: H2D of chunk i + 1 and D2H of chunk i - 1 overlap chunk i's encode and
// seal.
int qfec_encode_seal_groups_batch_host(qfec_ctx* c, int k, int m, int bb, long long groups,
                                       const unsigned char* h_data, const unsigned char* h_hdr,
                                       long long hdr_stride, const int* h_hdr_len,
                                       int hdr_len_all, const int* h_pt_len, int pt_len_all,
                                       unsigned char* h_pkt, long long pkt_stride,
                                       int* h_pkt_len) {
    const unsigned char* dummy = (const unsigned char*)16;   // non-null for the argument check
    int rc = seal_groups_args(c, k, m, bb, groups, h_data, dummy, h_hdr, hdr_stride, h_hdr_len,
                              hdr_len_all, h_pt_len, pt_len_all, h_pkt, pkt_stride, h_pkt_len);
    if (rc) return rc;
    if (groups == 0) return 0;
    if (hdr_stride <= 0 && h_hdr) return fail(-2, "host headers need a row stride > 0");
    if (pkt_stride <= 0) return fail(-2, "host packets need a row stride > 0");
    // the encode's -1 (cauchy_256.cpp:1530-1534): no packet is sealed, as on the device path
    // (the parity rows past P0 would be stale staging bytes sent with valid tags)
    if (m > 1 && k > 1 && (k + m > 256 || bb % 8 != 0))
        return fail(-1, "unsupported (k + m > 256 or block_bytes % 8 != 0)");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const long long np = k + m;                        // packets per group
    const size_t in_g = (size_t)k * bb, par_g = (size_t)m * bb;
    const size_t hdr_g = h_hdr ? (size_t)np * hdr_stride : 0;
    const size_t pkt_g = (size_t)np * pkt_stride;
    const size_t len_g = (size_t)np * sizeof(int32_t);
    const size_t per = in_g + par_g + hdr_g + pkt_g + len_g * (1 + (h_hdr_len ? 1 : 0) + (h_pt_len ? 1 : 0));
    rc = host_pipeline(c, groups, per, [&](long long g0, long long n, uint8_t* buf,
                                           int phase) -> int {
        Carve cv{buf};
        uint8_t* dd = cv.take((size_t)n * in_g);
        uint8_t* dp = cv.take((size_t)n * par_g);
        uint8_t* dh = h_hdr ? cv.take((size_t)n * hdr_g) : nullptr;
        uint8_t* dk = cv.take((size_t)n * pkt_g);
        int32_t* dkl = (int32_t*)cv.take((size_t)n * len_g);
        int32_t* dhl = h_hdr_len ? (int32_t*)cv.take((size_t)n * len_g) : nullptr;
        int32_t* dpl = h_pt_len ? (int32_t*)cv.take((size_t)n * len_g) : nullptr;
        const size_t p0 = (size_t)g0 * np, pn = (size_t)n * np;
        if (phase == 0) {
            QF_HIP(hipMemcpyAsync(dd, h_data + (size_t)g0 * in_g, (size_t)n * in_g,
                                  hipMemcpyHostToDevice, c->s_in));
            if (dh)
                QF_HIP(hipMemcpyAsync(dh, h_hdr + p0 * hdr_stride, pn * hdr_stride,
                                      hipMemcpyHostToDevice, c->s_in));
            if (dhl)
                QF_HIP(hipMemcpyAsync(dhl, h_hdr_len + p0, pn * sizeof(int32_t),
                                      hipMemcpyHostToDevice, c->s_in));
            if (dpl)
                QF_HIP(hipMemcpyAsync(dpl, h_pt_len + p0, pn * sizeof(int32_t),
                                      hipMemcpyHostToDevice, c->s_in));
        } else if (phase == 1) {
            const int r = encode_impl(c, k, m, bb, n, dd, dp, c->stream);
            if (r) return r;
            // packet rows are copied back whole: zero the staging rows first, so the bytes of
            // a row past its packet are zeros (as the device path leaves them untouched), not
            // an earlier chunk's packets
            QF_HIP(hipMemsetAsync(dk, 0, pn * pkt_stride, c->stream));
            QF_HIP(qfec::launch_null_seal_groups(k, m, bb, n, dd, dp, dh,
                                                 dh ? hdr_stride : 0, dhl, dh ? hdr_len_all : 0,
                                                 dpl, pt_len_all, dk, pkt_stride, dkl, c->stream));
        } else {
            QF_HIP(hipMemcpyAsync(h_pkt + p0 * pkt_stride, dk, pn * pkt_stride,
                                  hipMemcpyDeviceToHost, c->s_out));
            QF_HIP(hipMemcpyAsync(h_pkt_len + p0, dkl, pn * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, c->s_out));
        }
        return 0;
    }, kCarveSlack);
    return rc;
}

// Receiver, host memory to host memory: wire packets in, the recovered blocks (and, if asked,
// each packet's open length) out.  Chunked and pipelined as the other host batches.
int qfec_open_decode_batch_host(qfec_ctx* c, int k, int m, int bb, long long groups,
                                const unsigned char* h_pkt, long long pkt_stride,
                                const int* h_pkt_len, const int* h_ad_len, int ad_len_all,
                                unsigned char* h_rec, unsigned char* h_rec_rows, int* h_status,
                                int* h_open_len) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (k + m > 255) return fail(-2, "k + m > 255 (row tag 255 marks an unfilled slot)");
    if (groups == 0) return 0;
    if (!h_pkt || !h_pkt_len || !h_rec || !h_rec_rows) return fail(-2, "null buffer");
    if (pkt_stride <= 0) return fail(-2, "bad pkt_stride");
    if (!h_ad_len && ad_len_all < 0) return fail(-2, "bad ad_len_all");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const long long np = k + m;
    const int rmax = std::min(k, m);
    const size_t pkt_g = (size_t)np * pkt_stride, len_g = (size_t)np * sizeof(int32_t);
    const size_t blk_g = (size_t)k * bb, rec_g = (size_t)rmax * bb;
    const size_t per = pkt_g + len_g * (2 + (h_ad_len ? 1 : 0)) + blk_g + k + rec_g + rmax +
                       sizeof(int32_t);
    return host_pipeline(c, groups, per, [&](long long g0, long long n, uint8_t* buf,
                                             int phase) -> int {
        Carve cv{buf};
        uint8_t* dk = cv.take((size_t)n * pkt_g);
        int32_t* dkl = (int32_t*)cv.take((size_t)n * len_g);
        int32_t* dal = h_ad_len ? (int32_t*)cv.take((size_t)n * len_g) : nullptr;
        int32_t* dol = (int32_t*)cv.take((size_t)n * len_g);
        uint8_t* db = cv.take((size_t)n * blk_g);
        uint8_t* dr = cv.take((size_t)n * k);
        uint8_t* dre = cv.take((size_t)n * rec_g);
        uint8_t* drr = cv.take((size_t)n * rmax);
        int32_t* ds = (int32_t*)cv.take((size_t)n * sizeof(int32_t));
        const size_t p0 = (size_t)g0 * np, pn = (size_t)n * np;
        if (phase == 0) {
            QF_HIP(hipMemcpyAsync(dk, h_pkt + p0 * pkt_stride, pn * pkt_stride,
                                  hipMemcpyHostToDevice, c->s_in));
            QF_HIP(hipMemcpyAsync(dkl, h_pkt_len + p0, pn * sizeof(int32_t),
                                  hipMemcpyHostToDevice, c->s_in));
            if (dal)
                QF_HIP(hipMemcpyAsync(dal, h_ad_len + p0, pn * sizeof(int32_t),
                                      hipMemcpyHostToDevice, c->s_in));
        } else if (phase == 1) {
            return open_decode_impl(c, k, m, bb, n, dk, pkt_stride, dkl, dal, ad_len_all, db, dr,
                                    dol, dre, drr, ds, c->stream);
        } else {
            QF_HIP(hipMemcpyAsync(h_rec + (size_t)g0 * rec_g, dre, (size_t)n * rec_g,
                                  hipMemcpyDeviceToHost, c->s_out));
            QF_HIP(hipMemcpyAsync(h_rec_rows + (size_t)g0 * rmax, drr, (size_t)n * rmax,
                                  hipMemcpyDeviceToHost, c->s_out));
            if (h_status)
                QF_HIP(hipMemcpyAsync(h_status + g0, ds, (size_t)n * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, c->s_out));
            if (h_open_len)
                QF_HIP(hipMemcpyAsync(h_open_len + p0, dol, pn * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, c->s_out));
        }
        return 0;
    }, kCarveSlack);
}

int qfec_encode_batch_host(qfec_ctx* c, int k, int m, int bb, long long groups,
                           const unsigned char* h_data, unsigned char* h_parity) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups == 0) return 0;
    if (!h_data || !h_parity) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    // On the reference's -1 path only P0 is written (cauchy_256.cpp:1519-1534): copy back
    // only row 0 of each group so the caller's other recovery rows stay untouched.
    const bool p0_only = m > 1 && k > 1 && (k + m > 256 || bb % 8 != 0);
    const size_t in_g = (size_t)k * bb, out_g = (size_t)m * bb;
    int result = 0;
    rc = host_pipeline(c, groups, in_g + out_g, [&](long long g0, long long n, uint8_t* buf,
                                                     int phase) -> int {
        uint8_t* dd = buf;
        uint8_t* dp = buf + (size_t)n * in_g;
        if (phase == 0) {
            QF_HIP(hipMemcpyAsync(dd, h_data + (size_t)g0 * in_g, (size_t)n * in_g,
                                  hipMemcpyHostToDevice, c->s_in));
        } else if (phase == 1) {
            const int r = encode_impl(c, k, m, bb, n, dd, dp, c->stream);
            if (r < -1) return r;
            if (r) result = r;
        } else if (p0_only) {
            QF_HIP(hipMemcpy2DAsync(h_parity + (size_t)g0 * out_g, out_g, dp, out_g, bb, n,
                                    hipMemcpyDeviceToHost, c->s_out));
        } else {
            QF_HIP(hipMemcpyAsync(h_parity + (size_t)g0 * out_g, dp, (size_t)n * out_g,
                                  hipMemcpyDeviceToHost, c->s_out));
        }
        return 0;
    });
    return rc ? rc : result;
}

int qfec_decode_batch_host(qfec_ctx* c, int k, int m, int bb, long long groups,
                           unsigned char* h_blocks, unsigned char* h_rows, int* h_status) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    if (groups == 0) return 0;
    if (!h_blocks || !h_rows) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const size_t blk_g = (size_t)k * bb;
    // per group: blocks, row tags, status (4-byte aligned inside the chunk buffer)
    const size_t per = blk_g + k + sizeof(int32_t);
    return host_pipeline(c, groups, per, [&](long long g0, long long n, uint8_t* buf,
                                             int phase) -> int {
        uint8_t* db = buf;
        uint8_t* dr = db + (size_t)n * blk_g;
        int32_t* ds = (int32_t*)(((uintptr_t)(dr + (size_t)n * k) + 3) & ~(uintptr_t)3);
        if (phase == 0) {
            QF_HIP(hipMemcpyAsync(db, h_blocks + (size_t)g0 * blk_g, (size_t)n * blk_g,
                                  hipMemcpyHostToDevice, c->s_in));
            QF_HIP(hipMemcpyAsync(dr, h_rows + (size_t)g0 * k, (size_t)n * k,
                                  hipMemcpyHostToDevice, c->s_in));
        } else if (phase == 1) {
            const int r = decode_impl(c, k, m, bb, n, db, dr, db, dr, ds, c->stream);
            if (r) return r;
        } else {
            QF_HIP(hipMemcpyAsync(h_blocks + (size_t)g0 * blk_g, db, (size_t)n * blk_g,
                                  hipMemcpyDeviceToHost, c->s_out));
            QF_HIP(hipMemcpyAsync(h_rows + (size_t)g0 * k, dr, (size_t)n * k,
                                  hipMemcpyDeviceToHost, c->s_out));
            if (h_status)
                QF_HIP(hipMemcpyAsync(h_status + g0, ds, (size_t)n * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, c->s_out));
        }
        return 0;
    });
}

int qfec_synth_fill(void* d_dst, unsigned long long bytes, unsigned long long seed,
                    unsigned long long byte_offset, void* stream) {
    qfec::TimingMute mute;
    QF_HIP(qfec::launch_synth_fill((uint8_t*)d_dst, bytes, seed, byte_offset,
                                   (hipStream_t)stream));
    return 0;
}

int qfec_synth_gather(const unsigned char* d_data, const unsigned char* d_parity,
                      const short* d_src, unsigned char* d_blocks, int k, int m, int bb,
                      long long groups, void* stream) {
    qfec::TimingMute mute;
    QF_HIP(qfec::launch_synth_gather(d_data, d_parity, (const int16_t*)d_src, d_blocks, k, m, bb,
                                     groups, (hipStream_t)stream));
    return 0;
}

// ---------------------------------------------------------- single-group drop-ins
int _cauchy_256_init(int expected_version) {
    if (expected_version != CAUCHY_256_VERSION) return -1;   // cauchy_256.cpp:389-398
    qfec_ctx* c;
    return default_ctx(&c);
}

int cauchy_256_encode(int k, int m, const unsigned char* data_ptrs[], void* recovery_blocks,
                      int block_bytes) {
    qfec_ctx* c;
    int rc = default_ctx(&c);
    if (rc) return rc;
    if ((rc = check_common(c, k, m, block_bytes, 1))) return rc;
    if (!data_ptrs || !recovery_blocks) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const size_t bb = (size_t)block_bytes;
    const size_t in_bytes = (size_t)k * bb, out_bytes = (size_t)m * bb;
    QF_HIP(c->h_stage.ensure(in_bytes + out_bytes));
    QF_HIP(c->d_stage.ensure(in_bytes + out_bytes));
    uint8_t* hs = (uint8_t*)c->h_stage.p;
    for (int x = 0; x < k; ++x) memcpy(hs + x * bb, data_ptrs[x], bb);
    uint8_t* dd = (uint8_t*)c->d_stage.p;
    QF_HIP(hipMemcpyAsync(dd, hs, in_bytes, hipMemcpyHostToDevice, c->stream));
    // outputs the reference leaves untouched (the -1 paths) keep the caller's bytes
    QF_HIP(hipMemcpyAsync(dd + in_bytes, recovery_blocks, out_bytes, hipMemcpyHostToDevice,
                          c->stream));
    if (m > 1 && k > 1 && k + m <= 256 && bb % 8 == 0)   // :1554 zeroes rows 1..m-1
        QF_HIP(hipMemsetAsync(dd + in_bytes, 0, out_bytes, c->stream));
    rc = encode_impl(c, k, m, block_bytes, 1, dd, dd + in_bytes, c->stream);
    if (rc < -1) return rc;
    QF_HIP(hipMemcpyAsync(hs + in_bytes, dd + in_bytes, out_bytes, hipMemcpyDeviceToHost,
                          c->stream));
    QF_HIP(hipStreamSynchronize(c->stream));
    memcpy(recovery_blocks, hs + in_bytes, out_bytes);
    return rc;
}

int cauchy_256_decode(int k, int m, Block* blocks, int block_bytes) {
    qfec_ctx* c;
    int rc = default_ctx(&c);
    if (rc) return rc;
    if ((rc = check_common(c, k, m, block_bytes, 1))) return rc;
    if (!blocks) return fail(-2, "null buffer");
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    const size_t bb = (size_t)block_bytes;
    const size_t data_bytes = (size_t)k * bb;
    QF_HIP(c->h_stage.ensure(data_bytes + 256 + 16));
    QF_HIP(c->d_stage.ensure(data_bytes + 256 + 16));
    uint8_t* hs = (uint8_t*)c->h_stage.p;
    uint8_t* hr = hs + data_bytes;
    int32_t* hst = (int32_t*)(((uintptr_t)(hr + 256) + 3) & ~(uintptr_t)3);
    for (int x = 0; x < k; ++x) {
        memcpy(hs + x * bb, blocks[x].data, bb);
        hr[x] = blocks[x].row;
    }
    uint8_t* dd = (uint8_t*)c->d_stage.p;
    uint8_t* dr = dd + data_bytes;
    int32_t* dst = (int32_t*)(((uintptr_t)(dr + 256) + 3) & ~(uintptr_t)3);
    QF_HIP(hipMemcpyAsync(dd, hs, data_bytes + 256, hipMemcpyHostToDevice, c->stream));
    rc = decode_impl(c, k, m, block_bytes, 1, dd, dr, dd, dr, dst, c->stream);
    if (rc) return rc;
    QF_HIP(hipMemcpyAsync(hs, dd, data_bytes + k, hipMemcpyDeviceToHost, c->stream));
    QF_HIP(hipMemcpyAsync(hst, dst, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    QF_HIP(hipStreamSynchronize(c->stream));
    for (int x = 0; x < k; ++x) {
        if (blocks[x].row >= k || hr[x] != blocks[x].row)   // only recovery slots change
            memcpy(blocks[x].data, hs + x * bb, bb);
        blocks[x].row = hr[x];
    }
    return *hst;
}

int qfec_reserve(qfec_ctx* c, int k, int m, int bb, long long groups) {
    int rc = check_common(c, k, m, bb, groups);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    // both workspaces: the eager one and the one calls captured into a graph use
    for (Workspace* W : {&c->ws, &c->ws_graph}) {
        QF_HIP(W->ensure(W->dslots, (size_t)groups));   // m == 1 decode: erased slot per group
        if (m > 1 && k > 1) {
            const int rmax = std::min(k, m);
            if ((rc = decode_workspace(*W, k, rmax, decode_rc(rmax), groups))) return rc;
            if (rmax > decode_rc(rmax)) QF_HIP(W->ensure(W->dscratch, (size_t)groups * rmax * bb));
        }
    }
    if (m > 1 && k > 1 && k + m <= 256) {
        const uint8_t* t;
        if ((rc = get_enc_table(c, k, m, stream_encode_rc(k, m, bb, true, c->tune), &t))) return rc;
    }
    if (m > 1 && k > 1) {
        const uint8_t* t;
        if ((rc = get_cenc(c, k, m, &t))) return rc;
    }
    return 0;
}

}  // extern "C"
