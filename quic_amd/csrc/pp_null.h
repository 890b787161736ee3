// pp_null.h — launchers of the grouped packet-protection kernels (pp_null.hip) that sit next
// to the FEC codec: all k + m packets of a group sealed in one launch, and the receiver's
// open -> group assembly that feeds the decode.  The per-packet seal / open launchers are in
// fec_kernels.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qfec {

hipError_t launch_null_seal_h(long long n, const uint8_t* ad, long long ad_stride,
                              const int32_t* ad_len, int ad_all, const uint8_t* pt,
                              long long pt_stride, const int32_t* pt_len, int pt_all,
                              uint8_t* out, long long out_stride, int32_t* out_len,
                              hipStream_t st);
hipError_t launch_null_open_h(long long n, const uint8_t* pkt, long long pkt_stride,
                              const int32_t* pkt_len, int pkt_all, const int32_t* ad_len,
                              int ad_all, uint8_t* out, long long out_stride, int32_t* out_len,
                              hipStream_t st);

// Seal packet p = g * (k + m) + i of every group: AD = hdr row p, PT = data block (g, i) for
// i < k, parity block (g, i - k) otherwise (rows of bb bytes), PT length pt_len[p] (or
// pt_all), wire packet at out + p * out_stride (quic_packet_creator.cc:733-736 seals every
// data packet, :948-953 every FEC packet).
hipError_t launch_null_seal_groups(int k, int m, int bb, long long groups, const uint8_t* data,
                                   const uint8_t* parity, const uint8_t* hdr,
                                   long long hdr_stride, const int32_t* hdr_len, int hdr_all,
                                   const int32_t* pt_len, int pt_all, uint8_t* out,
                                   long long out_stride, int32_t* out_len, hipStream_t st);

// Receiver: open packet p = g * (k + m) + i (pkt_len[p] < 0: not received).  A data packet's
// plaintext goes to blocks[g][i], zero-padded to bb; open_len[p] = plaintext bytes, or -1
// (not received, malformed, longer than bb, or tag mismatch).  Then one wave per group builds
// rows[g][*] (data row i where packet i opened, else the next opened parity packet, ascending,
// whose plaintext it copies into the hole; 255 when none is left) for the decode.
hipError_t launch_open_groups(int k, int m, int bb, long long groups, const uint8_t* pkt,
                              long long pkt_stride, const int32_t* pkt_len,
                              const int32_t* ad_len, int ad_all, uint8_t* blocks,
                              uint8_t* rows, int32_t* open_len, hipStream_t st);

// After the decode of an open batch: groups with an unfilled slot get status -3 and no
// recovered rows.
hipError_t launch_open_status(int k, int rmax, long long groups, const uint8_t* rows,
                              uint8_t* rec_rows, int32_t* status, hipStream_t st);

}  // namespace qfec
