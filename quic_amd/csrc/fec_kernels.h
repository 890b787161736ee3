// fec_kernels.h — launch interface of the gfx950 FEC kernels (internal to libquic_fec.so).
//
// Layouts (all device memory, row-major, bb = block_bytes, s = bb / 8):
//   data     [G][k][bb]   the k data blocks of each packet group
//   parity   [G][m][bb]   encode output (parity block y of group g at (g*m + y)*bb)
//   blocks   [G][k][bb]   decode input: the first k packets received, any order
//   rows     [G][k]       row tag of each received block (data 0..k-1, parity k..k+m-1)
// The bit-sliced code treats every block as 8 sub-rows of s bytes; see DESIGN.md.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qfec {

// Per-context launch configuration.  The defaults are the measured best shapes
// (DESIGN.md); qfec_ctx_set_option() changes them for one context only, so no
// environment variable can change what the product launches.
struct Tune {
    int cus = 256;            // compute units of the context's device (filled at create)
    int xor_slots = 2;        // m = 1 LDS ring: group slots per wave (2..4)
    int xor_waves = 3;        //                 waves per workgroup (1..4)
    int dma = 1;              // m = 1: LDS-DMA ring kernel (0: flat register kernel)
    int stream = 1;           // m > 1, small blocks: gf_stream (0: gf_apply)
    int stream_ring = 8;      // gf_stream: 1 KiB ring slots per wave (4..36), + 2 mirrored
    int stream_grid = 0;      // gf_stream: grid cap in workgroups (0: CUs x per-CU fit)
    int stream_static = 1;    // gf_ring: compile-time ring schedule (B/C and preset encodes)
    int ring_wide = 1;        // gf_ring preset encodes: LDS-staged 8-byte parity stores
    int ring_split = 1;       // gf_ring (10, 20) encode: two units of 10 parity rows per group
    int psyn_wide = 1;        // gf_psyn wide recovered-block stores: 1 (10, 10), 2 all
    int const_enc = 1;        // encode kernels specialised for fixed (k, m) where compiled
    int pd = 2;               // gf_apply: register pipeline depth (1..3)
    int flat = 1;             // gf_apply: lane-flat encode
    int enc_rc = 8;           // gf_apply: encode outputs per wave (2, 4, 8)
    int prep_lane = 1;        // decode prep with 4 lanes per group when it applies
    int bsyn = 1;             // (32, 4) x 1352 B decode: compiled syndrome kernel gf_bsyn
                              //   (0: the run-time gf_stream decode)
    int bsyn_depth = 3;       // gf_bsyn: blocks in flight per wave (3, 5, 7; 3: 5 waves/SIMD)
    int psyn = 1;             // QuicR presets with m >= 7 and (5, 5) at 1352 B: compiled syndrome decode
                              //   gf_psyn (0: the run-time gf_stream decode)
    int dcol = 1;             // (128, 16) x 9008 B: gf_dcol (one wave per column tile, all 16
                              //   rows; 0: gf_apply)
    int dcol_grid = 0;        // gf_dcol: grid cap in workgroups (0: CUs x per-CU fit)
    int dcol_depth = 6;       // gf_dcol: blocks in flight per wave (6 or 8; two waves per SIMD)
    // Oversubscribed grids: about this many groups (units) per wave, more workgroups than the
    // device holds at once, so the hardware hands the last ones to whichever CU frees first
    // (0: the resident persistent grid, every wave walking groups g0, g0 + W, ...; -1: the
    // measured choice)
    int ring_wg = -1;         // gf_ring encodes (-1: 1 for (32,4), (10,10), (5,5), (250,5))
    int bsyn_wg = -1;         // gf_bsyn decode (-1: 2)
    int psyn_wg = 0;          // gf_psyn decodes
    int stream_wg = -1;       // gf_stream (run-time coefficients: the (250, 5) decode, other shapes;
                              //   -1: 1 for groups of at least 64 KiB, else 0)
    int dcol_wg = 4;          // gf_dcol encode / decode (units = column tiles; D 1909 -> 2000 GiB/s
                              //   over three alternating pairs on a power-limited box)
    int xor_wg = 0;           // xor_dma (m = 1)
    int host_chunk_mb = 64;   // host-pointer batches: chunk size
    int host_min_groups = 512;  // host-pointer batches: at least this many groups per chunk
                                //   (capped at 2 GiB of staging per buffer)
};

// Records the name of a kernel a call launched (qfec_last_kernels(), per thread).
void note_kernel(const char* name);
// Records the grid (workgroups) a persistent kernel was launched with (qfec_last_grids(),
// per thread, "name=grid" entries).
void note_grid(const char* name, unsigned grid);

// Workgroups of `kern` one CU holds at once (the runtime's occupancy answer), cached per
// (kernel, threads, LDS bytes); thread-safe.
int resident_blocks(const void* kern, int threads, size_t lds);

// Kernel timing hook (qfec_set_timing_events, per thread).  While a stop event is set, each
// engine call records `start` at the start of its first kernel and `stop` at the end of
// every kernel (the last record wins), through hipExtLaunchKernel: the events bracket the
// kernels themselves, not the launch gaps around them, so they agree with rocprofv3.
struct LaunchTiming {
    hipEvent_t start = nullptr, stop = nullptr;
    bool first = true;   // the call's first kernel has not been launched yet
    bool muted = false;  // a helper call (synth) is launching: leave the events alone
};
LaunchTiming& launch_timing();

// Helper entry points (qfec_synth_*) launch under this guard, so a timing bracket armed
// for the engine's next call neither starts nor stops at their kernels.
struct TimingMute {
    TimingMute() { launch_timing().muted = true; }
    ~TimingMute() { launch_timing().muted = false; }
};

// Every kernel of the library is launched through this.
template <typename F, typename... Args>
inline void qlaunch(F kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t st,
                    Args... args) {
    LaunchTiming& t = launch_timing();
    hipEvent_t a = nullptr, b = t.muted ? nullptr : t.stop;
    if (b && t.first) {
        a = t.start;
        t.first = false;
    }
    hipExtLaunchKernelGGL(kernel, grid, block, lds, st, a, b, 0u, args...);
}

// Decode work tables written by the prep kernel and read by the apply kernel.
struct DecodeWork {
    uint8_t* coef;     // [G][nchunk][k][RCP]  bit-sliced GF(256) coefficients
    uint8_t* slots;    // [G][RMAX]            output slot (0..k-1) of recovered block j
    int32_t* nout;     // [G]                  number of recovered blocks in this group
};

// Syndrome table (decode prep in syndrome mode, read by gf_dcol's syndrome decode), one per
// group at coef + g * coef_gstride, k <= 128 and at most 16 parity rows:
namespace syn {
constexpr int kPerm = 0;     // u8[k]  stream order of the slots: the present data rows
                             //        ascending (one slot each), then the extras: recovery
                             //        blocks and repeated data rows, in slot order
constexpr int kMask = 128;   // u32[4] bit x: data row x is in the ascending part
constexpr int kNeed = 144;   // u32    bit y: parity row y was received (a syndrome row)
constexpr int kISlot = 148;  // u8[16] syndrome index i of received parity row y
constexpr int kERow = 164;   // u8[k]  row tag of extra e
constexpr int kSinv = 292;   // u8[16][16] Sinv[j][i]: recovered j = sum_i Sinv[j][i] T_i
constexpr int kRowSlot = 548;  // u8[128] slot holding data row x (255: erased / unchanged group)
constexpr int kYmap = 676;   // u8[16] parity row y_i of syndrome i (recovery blocks, array order)
constexpr int kNExt = 692;   // u32    extras to stream after the rows (0: unchanged group)
constexpr int kBytes = 696;
}  // namespace syn

// Compact syndrome table of the small-block decode (decode_prep_bsyn, read by gf_bsyn), one
// per group at tab + g * kBytes, k <= 64 and at most 4 recovered blocks:
namespace bsyn {
constexpr int kPerm = 0;     // u8[64] stream order of the slots: present data rows ascending
                             //        (first copy of each), then the extras in slot order
constexpr int kMask = 64;    // u32[2] bit x: data row x is in the ascending part
constexpr int kY = 72;       // u8[4]  parity row y_i of recovery block i
constexpr int kSinv = 76;    // u8[4][4] Sinv[j][i]: recovered j = sum_i Sinv[j][i] T_{y_i}
constexpr int kERow = 92;    // u8[64] row tag of extra e (255: no-op, unchanged group)
constexpr int kBytes = 156;
}  // namespace bsyn

// Preset syndrome table (decode_prep_psyn, read by gf_psyn), one per group at
// tab + g * kBytes, k <= 64, m <= 32, at most 16 recovered blocks:
namespace psyn {
constexpr int kPerm = 0;     // u8[64] stream order of the slots: present data rows ascending
                             //        (first copy of each), then the extras in slot order
constexpr int kMask = 64;    // u32[2] bit x: data row x is in the ascending part
constexpr int kYs = 72;      // u8[16] received parity rows, ascending (syndrome slot s)
constexpr int kERow = 88;    // u8[64] row tag of extra e (255: no-op, unchanged group)
constexpr int kCoef = 152;   // u8[16][16] g[p][i]: pivot p's coefficient for slot i
constexpr int kNeed = 408;   // u32    bit y: parity row y enters the solve (received)
constexpr int kBytes = 412;
}  // namespace psyn

// parity[g*out_gstride ..+bb) = XOR of the k blocks of group g (m == 1 encode, and the
// P0 the reference writes before rejecting invalid m > 1 parameters).
hipError_t launch_xor_encode(const uint8_t* data, uint8_t* parity, int k, int bb,
                             long long groups, long long out_gstride, hipStream_t st,
                             const Tune& t);

// m == 1 decode: XOR the k-1 other blocks into the block tagged row >= k.  eidx is a
// [G] byte workspace (erased slot per group).  compact: the recovered block of group g
// goes to out + g * bb and its data row to rows_out[g] (255 = nothing erased).
hipError_t launch_xor_decode(const uint8_t* blocks, uint8_t* out, const uint8_t* rows_in,
                             uint8_t* rows_out, int32_t* status, uint8_t* eidx, int k, int bb,
                             long long groups, hipStream_t st, const Tune& t,
                             bool compact = false);

// k <= 1 encode: copy data[0] into each of the m outputs (cauchy_256.cpp:1508-1516).
hipError_t launch_replicate(const uint8_t* data, uint8_t* parity, int m, int bb,
                            long long groups, hipStream_t st);

// k <= 1 decode in the recovered-blocks layout (rec [G][rmax][bb], rec_rows [G][rmax]).
hipError_t launch_rec_k1(const uint8_t* blocks, const uint8_t* rows_in, uint8_t* rec,
                        uint8_t* rec_rows, int32_t* status, int bb, int rmax, long long groups,
                        hipStream_t st);

// k <= 1 decode: row := 0 (cauchy_256.cpp:1257-1261).
hipError_t launch_rows_k1(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                          long long groups, hipStream_t st);

// Bit-sliced GF(256) apply.  Encode: coef is the shared [nchunk][k][RCP] table built
// from the Cauchy matrix (row 0 = ones), outputs are parity rows chunk*RC + j.
hipError_t launch_gf_encode(const uint8_t* data, uint8_t* parity, const uint8_t* coef,
                            int k, int m, int bb, long long groups, int rc, hipStream_t st,
                            const Tune& t);

// Decode prep: per group, sort blocks, invert the erasure submatrix in GF(256) and
// emit the r x k recovery coefficients (syndrome: the syn:: table instead).  cenc is the
// [m][k] encode matrix (row 0 = ones).
// rows_out == nullptr: recovered-blocks layout, rec_rows [G][rmax] gets the data row of
// recovered block j (ascending), 255 past the group's erasure count.
hipError_t launch_decode_prep(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                              const uint8_t* cenc, DecodeWork w, int k, int m, int bb,
                              int rc, int rmax, long long groups, hipStream_t st,
                              const Tune& t, uint8_t* rec_rows = nullptr,
                              bool syndrome = false);

// Decode apply: recovered block j of group g = sum_pos coef[g][..][pos][j] (x) blocks[g][pos],
// written to out[g][slots[g][j]].
hipError_t launch_gf_decode(const uint8_t* blocks, uint8_t* out, DecodeWork w, int k, int m,
                            int bb, long long groups, int rc, int rmax, hipStream_t st,
                            const Tune& t);

// In-place decode when rmax > rc: apply into scratch [G][rmax][bb], then scatter to slots.
hipError_t launch_gf_decode_scratch(const uint8_t* blocks, uint8_t* scratch, DecodeWork w,
                                   int k, int m, int bb, long long groups, int rc, int rmax,
                                   hipStream_t st, const Tune& t);
hipError_t launch_scatter_recovered(const uint8_t* scratch, uint8_t* out, DecodeWork w, int k,
                                   int bb, int rmax, long long groups, hipStream_t st);

// m = 1 LDS-ring XOR kernel (xor_dma.hip).  Requires 16-byte aligned `in`, 8-byte aligned
// `out`/stride and bb % 8 == 0; decode with rows_in != null also does the row bookkeeping.
bool xor_dma_ok(const void* in, const void* out, int k, int bb, long long ogs, const Tune& t);
// compact: recovered-blocks layout (out [G][bb], rows_out [G] = recovered data row).
hipError_t launch_xor_dma(const uint8_t* in, uint8_t* out, const uint8_t* eidx,
                          const uint8_t* rows_in, uint8_t* rows_out, int32_t* status, int k,
                          int bb, long long groups, long long out_gstride, bool decode,
                          hipStream_t st, const Tune& t, bool compact = false);

// Per-wave LDS-ring streaming kernel for bb = 1352, one output chunk (gf_stream.hip).
bool gf_stream_supported(int k, int m, int bb, int rc, bool decode, const Tune& t);
// (k, m) codes whose gf_stream encode is compiled at this block size (no coefficient table)
bool gf_stream_compiled(int k, int m, int bb);
hipError_t launch_gf_stream(const uint8_t* in, uint8_t* out, const uint8_t* coef,
                            const uint8_t* slots, const int32_t* nout, int k, int m, int bb,
                            long long groups, int rc, int rmax, long long coef_gstride,
                            long long out_gstride, bool decode, hipStream_t st,
                            const Tune& t);


// One wave per column tile computing all 16 rows (gf_dcol.hip): encode of the compiled
// (128, 16) x 9008-byte code, and its syndrome decode from the syn:: table.
bool gf_dcol_supported(int k, int m, int bb, const Tune& t);
hipError_t launch_gf_dcol_encode(const uint8_t* in, uint8_t* out, int k, int m, int bb,
                                 long long groups, long long out_gstride, hipStream_t st,
                                 const Tune& t);
hipError_t launch_gf_dcol_syndrome(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                                   const uint8_t* slots, const int32_t* nout,
                                   const uint8_t* cenc, int k, int m, int bb, long long groups,
                                   int rmax, long long tab_gstride, long long out_gstride,
                                   hipStream_t st, const Tune& t);

// Syndrome decode of the compiled (32, 4) x 1352-byte code (gf_bsyn.hip): prep (bsyn::
// table, one lane per group) and the block pass + r x r solve.
bool gf_bsyn_supported(int k, int m, int bb, int rmax, const Tune& t);
hipError_t launch_decode_prep_bsyn(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                                   const uint8_t* cenc, uint8_t* tab, uint8_t* slots,
                                   int32_t* nout, uint8_t* rec_rows, int k, int m, int bb,
                                   int rmax, long long groups, hipStream_t st);
hipError_t launch_gf_bsyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* cenc, const uint8_t* slots, const int32_t* nout, int k,
                          int m, int bb, long long groups, int rmax, long long out_gstride,
                          hipStream_t st, const Tune& t);

// Syndrome decode of the compiled QuicR preset codes with m >= 7 and (5, 5) at 1352-byte blocks
// (gf_psyn.hip): prep (psyn:: table, 16 lanes per group) and the block pass + in-place
// Gauss-Jordan replay.
bool gf_psyn_supported(int k, int m, int bb, int rmax, const Tune& t);
hipError_t launch_decode_prep_psyn(const uint8_t* rows_in, uint8_t* rows_out, int32_t* status,
                                   const uint8_t* cenc, uint8_t* tab, uint8_t* slots,
                                   int32_t* nout, uint8_t* rec_rows, int k, int m, int bb,
                                   int rmax, long long groups, hipStream_t st);
hipError_t launch_gf_psyn(const uint8_t* in, uint8_t* out, const uint8_t* tab,
                          const uint8_t* cenc, const uint8_t* slots, const int32_t* nout, int k,
                          int m, int bb, long long groups, int rmax, long long out_gstride,
                          hipStream_t st, const Tune& t);

// Synthetic workload helpers (bench / tests): splitmix64 stream and receive-set gather.
hipError_t launch_synth_fill(uint8_t* dst, unsigned long long bytes, unsigned long long seed,
                             unsigned long long byte_offset, hipStream_t st);
hipError_t launch_synth_gather(const uint8_t* data, const uint8_t* parity, const int16_t* src,
                               uint8_t* blocks, int k, int m, int bb, long long groups,
                               hipStream_t st);

// Packet protection (pp_null.hip): NullEncrypter seal / NullDecrypter open over n packets.
// Per-packet lengths come from the arrays, or from the `_all` scalar when an array is null.
// out and out_stride must be 4-byte aligned.
hipError_t launch_null_seal(long long n, const uint8_t* ad, long long ad_stride,
                            const int32_t* ad_len, int ad_all, const uint8_t* pt,
                            long long pt_stride, const int32_t* pt_len, int pt_all, uint8_t* out,
                            long long out_stride, int32_t* out_len, hipStream_t st);
hipError_t launch_null_open(long long n, const uint8_t* pkt, long long pkt_stride,
                            const int32_t* pkt_len, int pkt_all, const int32_t* ad_len,
                            int ad_all, uint8_t* out, long long out_stride, int32_t* out_len,
                            hipStream_t st);

}  // namespace qfec
