"""CPU: the packet-protection oracle (oracle/pp_oracle.c) against the reference's own
known-answer tests and an independent big-integer restatement.

Reference tests replayed (vectors transcribed as data):
  null_encrypter_test.cc:15-31  Encrypt("hello world!", "goodbye!") -> a06f448a...b213 || PT
  null_decrypter_test.cc        Decrypt (same vector), BadHash (tag 4611ea5f...), ShortInput
  null_encrypter_test.cc:33-45  GetMaxPlaintextSize / GetCiphertextSize: +-12 bytes
"""
import numpy as np
import pytest

KAT_AD = b"hello world!"
KAT_PT = b"goodbye!"
KAT_TAG = bytes.fromhex("a06f448a44f8183b4791b213")
BAD_TAG = bytes.fromhex("4611ea5fcf1d665bbaf0bcfd")

FNV_OFFSET = 144066263297769815596495629667062367629   # quic_utils.cc:116
FNV_PRIME = (1 << 88) + 315                             # quic_utils.cc:45-47


def fnv_py(*parts):
    h = FNV_OFFSET
    for part in parts:
        for b in part:
            h = ((h ^ b) * FNV_PRIME) % (1 << 128)
    return h


def test_encrypt_known_answer(oracle):
    assert oracle.null_seal(KAT_AD, KAT_PT) == KAT_TAG + KAT_PT


def test_decrypt_known_answer(oracle):
    pt, _ = oracle.null_open(KAT_AD, KAT_TAG + KAT_PT)
    assert pt == KAT_PT


def test_decrypt_bad_hash(oracle):
    pt, buf = oracle.null_open(KAT_AD, BAD_TAG + KAT_PT)
    assert pt is None
    # the reference copies the ciphertext to the output before checking
    assert buf[:20].tobytes() == BAD_TAG + KAT_PT


def test_decrypt_short_input(oracle):
    pt, _ = oracle.null_open(KAT_AD, BAD_TAG[:11])
    assert pt is None


def test_sizes(oracle):
    for n in (1000, 100, 10):
        assert len(oracle.null_seal(b"", bytes(n))) == n + 12
    # too small an output buffer: the reference returns false
    assert oracle.null_seal(KAT_AD, KAT_PT, max_out=19) is None
    assert oracle.null_seal(KAT_AD, KAT_PT, max_out=20) is not None


def test_fnv_matches_big_integer_restatement(oracle):
    rng = np.random.default_rng(7)
    assert oracle.fnv1a_128(b"") == FNV_OFFSET
    for n1, n2 in [(0, 1), (1, 0), (12, 8), (13, 1352), (25, 9008), (3, 5)]:
        a = rng.integers(0, 256, n1, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, n2, dtype=np.uint8).tobytes()
        assert oracle.fnv1a_128(a, b) == fnv_py(a, b)
        assert oracle.fnv1a_128(a + b) == fnv_py(a, b)


def test_tag_serialisation_and_top_bits(oracle):
    # tag = low 8 bytes LE || bytes 8..11 LE (quic_utils.cc:175-181); the decrypter ignores
    # the top 32 bits of the hash (null_decrypter.cc ComputeHash mask)
    rng = np.random.default_rng(3)
    ad = rng.integers(0, 256, 17, dtype=np.uint8).tobytes()
    pt = rng.integers(0, 256, 300, dtype=np.uint8).tobytes()
    h = fnv_py(ad, pt)
    sealed = oracle.null_seal(ad, pt)
    assert sealed[:12] == (h & ((1 << 96) - 1)).to_bytes(12, "little")
    flipped = bytearray(sealed)
    flipped[11] ^= 0x80
    assert oracle.null_open(ad, bytes(flipped))[0] is None
    flipped = bytearray(sealed)
    flipped[12 + 150] ^= 1
    assert oracle.null_open(ad, bytes(flipped))[0] is None


def test_batch_layout_and_edges(oracle):
    rng = np.random.default_rng(11)
    n, S = 40, 160
    ad = rng.integers(0, 256, (n, 24), dtype=np.uint8)
    pt = rng.integers(0, 256, (n, S), dtype=np.uint8)
    ad_len = rng.integers(0, 25, n).astype(np.int32)
    pt_len = rng.integers(0, S - 4, n).astype(np.int32)   # 24 + 12 + 155 fits in 192
    pt_len[0] = S
    ad_len[0] = 24   # 24 + 12 + 160 = 196 > out_stride: does not fit
    out, res = oracle.null_seal_batch(ad, ad_len, pt, pt_len, 192)
    assert res[0] == -1 and not out[0].any()
    for i in range(1, n):
        a, p = ad[i, :ad_len[i]].tobytes(), pt[i, :pt_len[i]].tobytes()
        wire = a + oracle.null_seal(a, p)
        assert res[i] == len(wire)
        assert out[i, :res[i]].tobytes() == wire
    # open what was sealed, tamper with some
    pkt = out.copy()
    pkt_len = np.where(res < 0, 0, res).astype(np.int32)
    pkt[5, ad_len[5] + 12 - 1] ^= 1            # tag byte
    pkt_len[6] = ad_len[6] + 11                 # short ciphertext
    opened, ores = oracle.null_open_batch(pkt, pkt_len, ad_len, 192)
    for i in range(1, n):
        if i in (5, 6):
            assert ores[i] == -1
            cl = pkt_len[i] - ad_len[i]
            assert opened[i, :cl].tobytes() == pkt[i, ad_len[i]:pkt_len[i]].tobytes()
        else:
            assert ores[i] == pt_len[i]
            assert opened[i, :pt_len[i]].tobytes() == pt[i, :pt_len[i]].tobytes()


def test_batch_rejects_lengths_beyond_stride(oracle):
    ad = np.zeros((2, 8), np.uint8)
    pt = np.zeros((2, 8), np.uint8)
    _, res = oracle.null_seal_batch(ad, np.array([9, 8], np.int32), pt,
                                    np.array([8, 9], np.int32), 64)
    assert list(res) == [-1, -1]
    _, res = oracle.null_open_batch(np.zeros((2, 32), np.uint8), np.array([33, 32], np.int32),
                                    np.array([0, 0], np.int32), 64)
    assert res[0] == -1 and res[1] == -1   # 33 > stride; 32 bytes: a bad tag


def test_fnv_chain_split_algebra():
    """The split DESIGN.md 6.2 plans for the FNV-1a chain, checked against the oracle's hash:
    h ^ d = h + delta with delta = (l ^ d) - l, l = h mod 256, the low byte evolving alone as
    l' = ((l ^ d) * 59) mod 256, so h_n = h_0 P^n + sum_i delta_i P^(n - i) (mod 2^96, the
    tag's bits).  A plain restatement on the CPU (no GPU kernel implements it)."""
    import numpy as np
    from oracle import oracle as O
    P, M96 = (1 << 88) + 315, (1 << 96) - 1
    H0 = 144066263297769815596495629667062367629            # quic_utils.cc:116-118
    rng = np.random.default_rng(5)
    for n in [0, 1, 2, 17, 1380, 1999]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        lo, deltas = H0 & 255, []
        for b in d.tolist():
            x = lo ^ b
            deltas.append(x - lo)
            lo = (x * 59) & 255
        h = H0 * pow(P, n, 1 << 96)
        for i, dl in enumerate(deltas):
            h += dl * pow(P, n - i, 1 << 96)
        assert h & M96 == O.fnv1a_128(d) & M96, n
