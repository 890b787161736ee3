"""CPU: the oracle (plain-C restatement, oracle/fec_oracle.c) against the golden
vectors produced by the reference codec itself (tests/golden/gen_golden.py), and
against the compiled reference directly when oracle/_ref is built."""
import hashlib

import numpy as np
import pytest

from quic_amd import synth


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def batch_cases(cases):
    return [c for c in cases if c["kind"] == "batch"]


def test_golden_has_all_baseline_configs(golden):
    cases, _ = golden
    names = {c["name"] for c in cases}
    for n in ("A_xor_10_1", "B_gf_32_4_r2", "D_jumbo_128_16_r8"):
        assert n in names


@pytest.mark.parametrize("idx", range(22))
def test_oracle_batch_matches_golden(golden, oracle, idx):
    cases, full = golden
    c = batch_cases(cases)[idx]
    k, m, bb, G = c["k"], c["m"], c["bb"], c["groups"]
    data = synth.group_data(c["seed"], k, bb, G)
    par, rc = oracle.encode_batch(k, m, bb, data)
    assert rc == c["encode_rc"]
    assert sha(par) == c["parity_sha256"], c["name"]
    if c["name"] + "__parity" in full:
        np.testing.assert_array_equal(par, full[c["name"] + "__parity"])
    rows = np.array(c["rows_in"], np.uint8)
    recv = synth.assemble_received(data, par, rows.astype(np.int16))
    out, rows_out, status = oracle.decode_batch(k, m, bb, recv, rows)
    assert rows_out.tolist() == c["rows_out"]
    assert status.tolist() == c["status"]
    assert sha(out) == c["decoded_sha256"], c["name"]


def test_oracle_single_cases_match_golden(golden, oracle):
    cases, full = golden
    for c in cases:
        if c["kind"] == "encode":
            k, m, bb = c["k"], c["m"], c["bb"]
            blocks = [synth.stream_bytes(c["seed"], i * bb, bb) for i in range(k)]
            out, rc = oracle.encode_ptrs(k, m, bb, blocks)
            assert rc == c["rc"], c["name"]
            assert sha(out) == c["recovery_sha256"], c["name"]
        elif c["kind"] == "decode":
            k, m, bb = c["k"], c["m"], c["bb"]
            blocks = [synth.stream_bytes(c["seed"], i * bb, bb) for i in range(k)]
            outb, outr, rc = oracle.decode_blocks(k, m, bb, blocks, c["rows_in"])
            assert rc == c["rc"], c["name"]
            assert outr == c["rows_out"], c["name"]
            assert sha(np.stack(outb)) == c["blocks_sha256"], c["name"]


def test_stream_matches_c_oracle(oracle):
    import ctypes
    for seed, off, n in [(1, 0, 64), (7, 13, 100), (2**63 + 5, 4095, 333)]:
        a = synth.stream_bytes(seed, off, n)
        b = np.zeros(n, np.uint8)
        oracle.lib().oracle_fill_stream(seed, off, b.ctypes.data_as(ctypes.c_void_p), n)
        np.testing.assert_array_equal(a, b)


def test_gf_field_is_0x187(oracle):
    # alpha^8 = x^7 + x^2 + x + 1 (cauchy_256.cpp:272); the unused Galois256 uses 0x15F
    assert oracle.gf_mul(0x80, 2) == 0x87
    for a in (1, 2, 3, 0x53, 0xFF):
        for b in (1, 7, 0x80, 0xCA):
            assert oracle.gf_div(oracle.gf_mul(a, b), b) == a


@pytest.mark.skipif("not __import__('oracle.oracle', fromlist=['x']).ref_available()")
@pytest.mark.parametrize("k,m,bb,r", [(10, 1, 1352, 1), (32, 4, 1352, 2), (29, 11, 72, 9),
                                      (7, 30, 16, 7), (100, 100, 8, 60), (3, 2, 1352, 2)])
def test_oracle_equals_compiled_reference(oracle, k, m, bb, r):
    G = 3
    data = synth.group_data(99 + k, k, bb, G)
    p_ref, rc_ref = oracle.encode_batch(k, m, bb, data, use_ref=True)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    assert rc_ref == rc_or
    np.testing.assert_array_equal(p_ref, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 5, shuffle=True)
    recv = synth.assemble_received(data, p_ref, src)
    b1, r1, s1 = oracle.decode_batch(k, m, bb, recv, rows, use_ref=True)
    b2, r2, s2 = oracle.decode_batch(k, m, bb, recv, rows)
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(s1, s2)
