#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE codec.

Runs only in the build container: it loads oracle/_ref/libref_cauchy.so, which
oracle/Makefile compiles from /root/reference/net/quic/core/libcat/
{cauchy_256,MemXOR,MemSwap}.cpp.  The committed outputs are pure data:
  golden.json  - case parameters, the receive patterns, return codes, the
                 decoded row fields and SHA-256 digests of every output buffer;
  golden_small.npz - full parity bytes and recovered blocks for the small cases.
Inputs are not stored: they are regenerated from the seed by
quic_amd.synth.group_data (splitmix64 stream, documented there).

Usage:  python tests/golden/gen_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from quic_amd import synth  # noqa: E402

# (name, k, m, bb, groups, r, mode, parity, shuffle, keep_full)
BATCH_CASES = [
    # BASELINE configs (scaled-down group counts)
    ("A_xor_10_1", 10, 1, 1352, 8, 1, "random", "first", False, True),
    ("B_gf_32_4_r2", 32, 4, 1352, 4, 2, "random", "random", False, True),
    ("D_jumbo_128_16_r8", 128, 16, 9008, 2, 8, "random", "random", False, False),
    # m = 1 with block_bytes not a multiple of 8 (the XOR path has no restriction)
    ("A_xor_10_1_bb1350", 10, 1, 1350, 4, 1, "random", "first", False, True),
    # erasure counts: none, all parity used, shuffled arrival order
    ("B_gf_32_4_r0", 32, 4, 1352, 2, 0, "random", "random", False, True),
    ("B_gf_32_4_r4", 32, 4, 1352, 3, 4, "random", "random", True, True),
    ("B_gf_32_4_r1_shuffled", 32, 4, 1352, 3, 1, "random", "random", True, True),
    # windowed paths in the reference (m > 4 encode, > 4 erasures decode)
    ("W_20_10_r6", 20, 10, 64, 4, 6, "random", "random", True, True),
    ("W_64_8_r8", 64, 8, 256, 2, 8, "random", "random", False, True),
    # every table regime: m = 2..6 precomputed rows, m >= 7 from X/Y vectors
    ("T_m2", 17, 2, 40, 3, 2, "random", "random", False, True),
    ("T_m3", 9, 3, 8, 3, 3, "random", "random", False, True),
    ("T_m5", 31, 5, 24, 3, 5, "random", "random", False, True),
    ("T_m6", 50, 6, 16, 2, 3, "random", "random", False, True),
    ("T_m7", 12, 7, 8, 2, 7, "random", "random", False, True),
    ("T_m16_k240", 240, 16, 8, 1, 16, "random", "random", False, True),
    # QuicR presets (quic_fec_group.cc:22-82): FEC_5_5 .. FEC_250_5
    ("P_5_5", 5, 5, 1352, 2, 5, "random", "random", False, True),
    ("P_10_10", 10, 10, 1352, 2, 7, "random", "random", False, True),
    ("P_10_15", 10, 15, 1352, 2, 10, "random", "random", False, True),
    ("P_10_20", 10, 20, 128, 2, 10, "random", "random", False, True),
    ("P_15_15", 15, 15, 256, 2, 15, "random", "random", False, True),
    ("P_250_5", 250, 5, 64, 2, 5, "random", "random", False, True),
    # k + m == 256 (largest legal)
    ("L_200_56", 200, 56, 16, 1, 40, "random", "random", False, True),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def batch_case(name, k, m, bb, G, r, mode, parity, shuffle, keep, seed, full):
    data = synth.group_data(seed, k, bb, G)
    par, rc_e = O.encode_batch(k, m, bb, data, use_ref=True)
    rows, src = synth.loss_patterns(k, m, r, G, seed + 1, mode=mode, parity=parity,
                                    shuffle=shuffle)
    recv = synth.assemble_received(data, par, src)
    out, rows_out, status = O.decode_batch(k, m, bb, recv, rows, use_ref=True)
    # sanity: every slot now holds the data block its row names
    for g in range(G):
        for i in range(k):
            assert (out[g, i] == data[g, rows_out[g, i]]).all(), (name, g, i)
    case = dict(name=name, kind="batch", k=k, m=m, bb=bb, groups=G, seed=seed,
                loss=dict(r=r, mode=mode, parity=parity, shuffle=shuffle),
                encode_rc=int(rc_e), parity_sha256=sha(par),
                rows_in=rows.tolist(), rows_out=rows_out.tolist(),
                status=status.tolist(), decoded_sha256=sha(out))
    if keep:
        full[name + "__parity"] = par
        # only the recovered slots (rows_in >= k) are stored in full
        slots = rows.astype(np.int64) >= k
        full[name + "__recovered"] = out[slots].reshape(G, -1, bb)
    return case


def single_cases(full):
    """Single-group ABI edge cases (cauchy_256.h semantics)."""
    cases = []

    def enc(name, k, m, bb, seed):
        blocks = [synth.stream_bytes(seed, i * bb, bb) for i in range(k)]
        out, rc = O.encode_ptrs(k, m, bb, blocks, use_ref=True)
        full[name + "__recovery"] = out
        cases.append(dict(name=name, kind="encode", k=k, m=m, bb=bb, seed=seed, rc=int(rc),
                          recovery_sha256=sha(out)))

    def dec(name, k, m, bb, seed, rows):
        blocks = [synth.stream_bytes(seed, i * bb, bb) for i in range(k)]
        outb, outr, rc = O.decode_blocks(k, m, bb, blocks, rows, use_ref=True)
        full[name + "__blocks"] = np.stack(outb)
        cases.append(dict(name=name, kind="decode", k=k, m=m, bb=bb, seed=seed,
                          rows_in=list(rows), rows_out=[int(x) for x in outr], rc=int(rc),
                          blocks_sha256=sha(np.stack(outb))))

    enc("E_k1_copy", 1, 3, 24, 11)                 # k <= 1: copy data[0] to every output
    enc("E_k2_m2", 2, 2, 8, 12)
    enc("E_err_k_plus_m_257", 250, 7, 16, 13)      # -1, but P0 already written
    enc("E_err_bb_not_mult8", 10, 3, 1350, 14)     # -1, but P0 already written
    enc("E_m1_bb1350", 10, 1, 1350, 15)            # m = 1 allows any block_bytes
    dec("D_k1", 1, 2, 16, 21, [1])                 # k <= 1: row := 0, data untouched
    dec("D_nothing_erased", 6, 3, 16, 22, [0, 1, 2, 3, 4, 5])
    dec("D_m1_no_erasure", 6, 1, 16, 23, [5, 4, 3, 2, 1, 0])
    dec("D_m1_parity_first", 6, 1, 16, 24, [6, 0, 1, 2, 4, 5])
    dec("D_err_bb_not_mult8", 6, 3, 12, 25, [0, 1, 2, 6, 7, 5])   # -1
    dec("D_err_k_plus_m_257", 250, 7, 8, 26, list(range(1, 250)) + [250])  # -1
    dec("D_err_but_no_erasure", 6, 3, 12, 27, [0, 1, 2, 3, 4, 5])  # 0: checked only if erased
    return cases


def main():
    if not O.ref_available():
        sys.exit("oracle/_ref/libref_cauchy.so missing: run `make -C oracle ref` first")
    full = {}
    cases = []
    for i, c in enumerate(BATCH_CASES):
        cases.append(batch_case(*c, seed=1000 + i, full=full))
    cases += single_cases(full)
    meta = dict(
        generator="tests/golden/gen_golden.py",
        reference="net/quic/core/libcat/cauchy_256.cpp (compiled by oracle/Makefile)",
        stream="quic_amd.synth.stream_bytes (splitmix64); group g block x = bytes "
               "[(g*k + x)*bb, +bb) of the stream",
        cases=cases)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), **full)
    print(f"{len(cases)} cases written")


if __name__ == "__main__":
    main()
