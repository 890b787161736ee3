"""GPU parity: the gfx950 kernels (through the C ABI) against the golden vectors from
the reference codec and against the CPU oracle, bit-exact.  Run with -m gpu."""
import hashlib

import numpy as np
import pytest

from quic_amd import fec, synth

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def gpu_encode(engine, k, m, bb, data):
    import torch
    d = dev(data)
    p = torch.zeros((data.shape[0], m, bb), dtype=torch.uint8, device="cuda")
    rc = engine.encode(k, m, bb, d, p)
    return host(p), rc


def gpu_decode(engine, k, m, bb, blocks, rows, inplace=True):
    import torch
    b = dev(blocks)
    r = dev(rows)
    st = torch.full((blocks.shape[0],), 7, dtype=torch.int32, device="cuda")
    if inplace:
        engine.decode(k, m, bb, b, r, status=st)
        return host(b), host(r), host(st)
    out = torch.zeros_like(b)
    ro = torch.zeros_like(r)
    engine.decode(k, m, bb, b, r, out=out, rows_out=ro, status=st)
    # out-of-place: only recovered slots are written; merge for comparison
    o = host(out)
    rin = rows.astype(np.int64)
    merged = blocks.copy()
    mask = rin >= k
    merged[mask] = o[mask]
    return merged, host(ro), host(st)


# ---------------------------------------------------------------- golden vectors
def batch_case_ids(golden_cases):
    return [c["name"] for c in golden_cases if c["kind"] == "batch"]


@pytest.mark.parametrize("inplace", [True, False])
def test_golden_batch_cases(engine, golden, inplace):
    cases, full = golden
    for c in cases:
        if c["kind"] != "batch":
            continue
        k, m, bb, G = c["k"], c["m"], c["bb"], c["groups"]
        data = synth.group_data(c["seed"], k, bb, G)
        par, rc = gpu_encode(engine, k, m, bb, data)
        assert rc == c["encode_rc"], c["name"]
        assert sha(par) == c["parity_sha256"], c["name"]
        rows = np.array(c["rows_in"], np.uint8)
        recv = synth.assemble_received(data, par, rows.astype(np.int16))
        out, rows_out, status = gpu_decode(engine, k, m, bb, recv, rows, inplace=inplace)
        assert rows_out.tolist() == c["rows_out"], c["name"]
        assert status.tolist() == c["status"], c["name"]
        assert sha(out) == c["decoded_sha256"], c["name"]


def test_golden_single_group_dropins(golden):
    """cauchy_256_encode / cauchy_256_decode (the drop-in ABI) on the GPU."""
    cases, full = golden
    assert fec.cauchy_256_init() == 0
    for c in cases:
        k, m, bb = c.get("k"), c.get("m"), c.get("bb")
        if c["kind"] == "encode":
            blocks = [synth.stream_bytes(c["seed"], i * bb, bb) for i in range(k)]
            out = np.zeros(m * bb, np.uint8)
            rc = fec.cauchy_256_encode(k, m, blocks, out, bb)
            assert rc == c["rc"], c["name"]
            assert sha(out.reshape(m, bb)) == c["recovery_sha256"], c["name"]
        elif c["kind"] == "decode":
            blocks = [synth.stream_bytes(c["seed"], i * bb, bb) for i in range(k)]
            blk = fec.make_blocks(blocks, c["rows_in"])
            rc = fec.cauchy_256_decode(k, m, blk, bb)
            assert rc == c["rc"], c["name"]
            assert [blk[i].row for i in range(k)] == c["rows_out"], c["name"]
            assert sha(np.stack(blocks)) == c["blocks_sha256"], c["name"]
        elif c["kind"] == "batch" and c["groups"] * c["k"] * c["bb"] < 2_000_000:
            # the batch cases through the per-group drop-in, group 0
            k, m, bb = c["k"], c["m"], c["bb"]
            data = synth.group_data(c["seed"], k, bb, 1)[0]
            rec = np.zeros(m * bb, np.uint8)
            rc = fec.cauchy_256_encode(k, m, list(data), rec, bb)
            assert rc == c["encode_rc"]
            full_par = full.get(c["name"] + "__parity")
            if full_par is not None:
                np.testing.assert_array_equal(rec.reshape(m, bb), full_par[0])
            rows = c["rows_in"][0]
            sent = np.concatenate([data, rec.reshape(m, bb)])
            blocks = [sent[r].copy() for r in rows]
            blk = fec.make_blocks(blocks, rows)
            assert fec.cauchy_256_decode(k, m, blk, bb) == c["status"][0]
            assert [blk[i].row for i in range(k)] == c["rows_out"][0]
            for i in range(k):
                np.testing.assert_array_equal(blocks[i], data[blk[i].row])


# ----------------------------------------------------------- randomized vs oracle
CONFIGS = [
    # (k, m, bb, r, shuffle)
    (10, 1, 1352, 1, False), (10, 1, 1350, 1, True), (10, 1, 1351, 1, False), (3, 1, 7, 1, True),
    (10, 1, 1352, 0, False), (255, 1, 64, 1, False), (64, 1, 9008, 1, True),
    (32, 4, 1352, 2, False), (32, 4, 1352, 4, True), (32, 4, 1352, 1, True), (32, 4, 1352, 0, False),
    (2, 2, 8, 2, False), (5, 3, 16, 3, True), (7, 2, 24, 1, False), (9, 4, 40, 4, True),
    (17, 5, 1352, 5, True), (16, 8, 9008, 8, False), (20, 10, 64, 10, True),
    (128, 16, 1352, 8, False), (100, 20, 136, 17, True), (40, 40, 32, 33, True),
    (200, 56, 16, 40, False), (250, 5, 1352, 5, False), (10, 15, 1352, 10, True),
    (128, 16, 9008, 8, True), (128, 16, 9008, 16, False), (130, 16, 9008, 3, True),
    (8, 5, 9008, 5, False),
]


@pytest.mark.parametrize("k,m,bb,r,shuffle", CONFIGS)
def test_random_vs_oracle(engine, oracle, k, m, bb, r, shuffle):
    G = 5
    data = synth.group_data(1234 + k * 7 + m, k, bb, G)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    assert rc == rc_or
    np.testing.assert_array_equal(p_gpu, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 77 + bb, shuffle=shuffle)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    for inplace in (True, False):
        b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=inplace)
        np.testing.assert_array_equal(rr, r_or)
        np.testing.assert_array_equal(s, s_or)
        np.testing.assert_array_equal(b, b_or)


def test_unsupported_params_status(engine, oracle):
    # k + m > 256: encode writes P0 then returns -1; decode with erasures -> status -1
    k, m, bb = 250, 7, 16
    data = synth.group_data(5, k, bb, 3)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    assert rc == rc_or == -1
    np.testing.assert_array_equal(p_gpu, p_or)
    rows = np.tile(np.array(list(range(1, 250)) + [250], np.uint8), (3, 1))
    b, rr, s = gpu_decode(engine, k, m, bb, data, rows)
    b2, rr2, s2 = oracle.decode_batch(k, m, bb, data, rows)
    assert s.tolist() == s2.tolist() == [-1, -1, -1]
    np.testing.assert_array_equal(rr, rr2)
    np.testing.assert_array_equal(b, b2)
    # block_bytes % 8 != 0 with m > 1
    k, m, bb = 10, 3, 1350
    data = synth.group_data(6, k, bb, 2)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    assert rc == rc_or == -1
    np.testing.assert_array_equal(p_gpu, p_or)


def test_host_pointer_batch(engine, oracle):
    k, m, bb, G, r = 32, 4, 1352, 64, 3
    data = synth.group_data(42, k, bb, G)
    par, rc = engine.encode_host(k, m, bb, data)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    assert rc == 0
    np.testing.assert_array_equal(par, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 3, shuffle=True)
    recv = synth.assemble_received(data, par, src)
    b, rr, s = engine.decode_host(k, m, bb, recv, rows)
    b2, rr2, s2 = oracle.decode_batch(k, m, bb, recv, rows)
    np.testing.assert_array_equal(b, b2)
    np.testing.assert_array_equal(rr, rr2)
    np.testing.assert_array_equal(s, s2)


# ------------------------------------------------------ BASELINE-size properties
@pytest.mark.parametrize("k,m,bb,r", [(10, 1, 1352, 1), (32, 4, 1352, 2)])
def test_full_size_round_trip(engine, oracle, k, m, bb, r):
    """65,536 groups (BASELINE.json configs[1], [2]): device-side synthetic data,
    encode -> lose r data blocks per group -> decode; every recovered block must equal
    the original, and sampled groups must match the oracle byte for byte."""
    import torch
    G = 65536
    data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_fill(data, seed=2024)
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    assert engine.encode(k, m, bb, data, parity) == 0
    rows, src = synth.loss_patterns(k, m, r, G, 11, shuffle=False)
    rows_d, src_d = dev(rows), dev(src)
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_gather(data, parity, src_d, blocks, k, m, bb)
    out = torch.zeros_like(blocks)
    rows_out = torch.zeros_like(rows_d)
    status = torch.full((G,), 9, dtype=torch.int32, device="cuda")
    engine.decode(k, m, bb, blocks, rows_d, out=out, rows_out=rows_out, status=status)
    torch.cuda.synchronize()
    assert int(status.abs().max()) == 0
    # recovered slots: rows_in >= k; their data must be data[g][rows_out]
    rin = rows_d.long()
    slot_mask = rin >= k
    ro = rows_out.long()
    assert bool((ro[slot_mask] < k).all())
    g_idx = torch.arange(G, device="cuda")[:, None].expand(G, k)[slot_mask]
    recovered = out[slot_mask]
    original = data[g_idx, ro[slot_mask]]
    assert torch.equal(recovered, original)
    # the synthetic stream is the documented splitmix64 stream
    np.testing.assert_array_equal(host(data[5]).ravel(),
                                  synth.stream_bytes(2024, 5 * k * bb, k * bb))
    # sampled groups vs the oracle
    sample = [0, 1, 777, G - 1]
    d_np = host(data[sample])
    p_or, _ = oracle.encode_batch(k, m, bb, d_np)
    np.testing.assert_array_equal(host(parity[sample]), p_or)


# ------------------------------------------------- recovered-blocks layout (receiver)
def expected_recovered(k, m, bb, rows_in, b_or, r_or, s_or):
    """Recovered blocks in the order cauchy_256_decode assigns erased rows: the i-th
    recovery slot (array order, row >= k) gets the i-th smallest erased row
    (cauchy_256.cpp:570-574); m = 1 uses only the first such slot (:486-540)."""
    G = rows_in.shape[0]
    rmax = min(k, m)
    rec = np.zeros((G, rmax, bb), np.uint8)
    rec_rows = np.full((G, rmax), 255, np.uint8)
    for g in range(G):
        if s_or[g] != 0:
            continue
        if k <= 1:
            if rows_in[g][0] != 0:
                rec_rows[g][0] = 0
                rec[g][0] = b_or[g][0]
            continue
        slots = [i for i in range(k) if rows_in[g][i] >= k]
        if m == 1:
            slots = slots[:1]
        j = 0
        for sl in slots:
            if r_or[g][sl] < k and r_or[g][sl] != rows_in[g][sl]:
                rec_rows[g][j] = r_or[g][sl]
                rec[g][j] = b_or[g][sl]
                j += 1
    return rec, rec_rows


@pytest.mark.parametrize("k,m,bb,r,shuffle", [
    (10, 1, 1352, 1, False), (10, 1, 1352, 0, False), (10, 1, 1350, 1, True),
    (32, 4, 1352, 2, True), (32, 4, 1352, 4, False), (8, 4, 64, 3, True),
    (16, 8, 9008, 8, False), (128, 16, 1352, 11, True), (4, 4, 64, 0, False),
    (20, 10, 64, 10, True),
])
def test_decode_recovered_vs_oracle(engine, oracle, k, m, bb, r, shuffle):
    import torch
    G = 6
    data = synth.group_data(4321 + k + m, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    rows, src = synth.loss_patterns(k, m, r, G, 55 + bb, shuffle=shuffle)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rmax = min(k, m)
    b = dev(recv)
    rw = dev(rows)
    rec = torch.zeros((G, rmax, bb), dtype=torch.uint8, device="cuda")
    rec_rows = torch.zeros((G, rmax), dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 7, dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, b, rw, rec, rec_rows, status=st)
    np.testing.assert_array_equal(host(st), s_or)
    got_rows = host(rec_rows)
    np.testing.assert_array_equal(got_rows, exp_rows)
    got = host(rec)
    mask = exp_rows != 255
    np.testing.assert_array_equal(got[mask], exp[mask])
    # recovered blocks are the original data rows
    for g in range(G):
        for j in range(rmax):
            if got_rows[g][j] != 255:
                np.testing.assert_array_equal(got[g][j], data[g][got_rows[g][j]])
    # inputs untouched
    np.testing.assert_array_equal(host(b), recv)
    np.testing.assert_array_equal(host(rw), rows)


def test_decode_recovered_k1_and_unsupported(engine, oracle):
    import torch
    # k = 1: a parity block is a copy of data row 0
    k, m, bb, G = 1, 3, 64, 4
    data = synth.group_data(9, k, bb, G)
    rows = np.array([[0], [1], [3], [2]], np.uint8)
    rec = torch.zeros((G, 1, bb), dtype=torch.uint8, device="cuda")
    rr = torch.zeros((G, 1), dtype=torch.uint8, device="cuda")
    engine.decode_recovered(k, m, bb, dev(data), dev(rows), rec, rr)
    assert host(rr)[:, 0].tolist() == [255, 0, 0, 0]
    np.testing.assert_array_equal(host(rec)[1:, 0], data[1:, 0])
    # k + m > 256: status -1, nothing recovered
    k, m, bb, G = 250, 7, 16, 2
    data = synth.group_data(5, k, bb, G)
    rows = np.tile(np.array(list(range(1, 250)) + [250], np.uint8), (G, 1))
    rec = torch.zeros((G, 7, bb), dtype=torch.uint8, device="cuda")
    rr = torch.zeros((G, 7), dtype=torch.uint8, device="cuda")
    st = torch.zeros((G,), dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, dev(data), dev(rows), rec, rr, status=st)
    assert host(st).tolist() == [-1, -1]
    assert (host(rr) == 255).all()


def test_decode_recovered_host(engine, oracle):
    import torch
    k, m, bb, G, r = 32, 4, 1352, 40, 3
    data = synth.group_data(77, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    rows, src = synth.loss_patterns(k, m, r, G, 8, shuffle=True)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rec = torch.zeros((G, 4, bb), dtype=torch.uint8)
    rr = torch.zeros((G, 4), dtype=torch.uint8)
    st = torch.zeros((G,), dtype=torch.int32)
    fec.decode_recovered_host_into(engine, k, m, bb, torch.from_numpy(recv),
                                   torch.from_numpy(rows), rec, rr, st)
    np.testing.assert_array_equal(rr.numpy(), exp_rows)
    mask = exp_rows != 255
    np.testing.assert_array_equal(rec.numpy()[mask], exp[mask])
    assert st.abs().max() == 0


@pytest.mark.parametrize("k,m,r", [(32, 4, 3), (10, 10, 7)])
def test_host_pipeline_many_chunks(tuned_engine, oracle, k, m, r):
    """Host-pointer batches cut into more chunks than the NB = 3 rotating staging buffers
    (host_chunk_mb = 1, host_min_groups = 1: 1 MiB chunks): every buffer is reused, so the
    H2D / kernel / D2H event chain must order each reuse after the previous chunk's
    copy-out.  Encode, in-place decode and recovered-blocks decode against the oracle."""
    import torch
    engine = tuned_engine
    engine.set_option("host_chunk_mb", 1)
    engine.set_option("host_min_groups", 1)
    bb = 1352
    G = 4 * ((3 << 20) // (2 * k * bb)) + 5       # more than 4 x NB chunks for every call
    data = synth.group_data(900 + k, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    par, rc = engine.encode_host(k, m, bb, data)
    assert rc == 0
    np.testing.assert_array_equal(par, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 31 + k, shuffle=True)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    b, rr, s = engine.decode_host(k, m, bb, recv, rows)
    np.testing.assert_array_equal(s, s_or)
    np.testing.assert_array_equal(rr, r_or)
    np.testing.assert_array_equal(b, b_or)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rmax = min(k, m)
    rec = torch.zeros((G, rmax, bb), dtype=torch.uint8)
    rec_rows = torch.zeros((G, rmax), dtype=torch.uint8)
    st = torch.full((G,), 7, dtype=torch.int32)
    fec.decode_recovered_host_into(engine, k, m, bb, torch.from_numpy(recv),
                                   torch.from_numpy(rows), rec, rec_rows, st)
    np.testing.assert_array_equal(rec_rows.numpy(), exp_rows)
    mask = exp_rows != 255
    np.testing.assert_array_equal(rec.numpy()[mask], exp[mask])
    assert st.abs().max() == 0


# ------------------------------------------- gf_stream ring (many groups per wave)
@pytest.fixture
def tuned_engine():
    """A fresh engine (own context) for tests that change launch options."""
    from quic_amd.fec import FecEngine
    eng = FecEngine(0)
    yield eng
    eng.close()


@pytest.mark.parametrize("ring", [4, 7, 10])
@pytest.mark.parametrize("k,m,r", [(32, 4, 2), (32, 3, 3), (250, 5, 5), (32, 8, 6)])
def test_stream_ring_many_groups_per_wave(tuned_engine, oracle, ring, k, m, r):
    """One workgroup (4 waves) walks every group, so each wave streams several groups
    through its LDS ring back to back (the ring wraps inside blocks and across groups);
    every third group has no loss (decode skips it but its pieces stay in the stream)."""
    import torch
    engine = tuned_engine
    engine.set_option("stream_grid", 1)
    engine.set_option("stream_ring", ring)
    bb, G = 1352, 23
    data = synth.group_data(900 + k + m + ring, k, bb, G)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    assert rc == rc_or == 0
    np.testing.assert_array_equal(p_gpu, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 31 + ring, shuffle=True)
    rows[::3] = np.arange(k, dtype=rows.dtype)
    src[::3] = np.arange(k, dtype=src.dtype)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    for inplace in (True, False):
        b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=inplace)
        np.testing.assert_array_equal(s, s_or)
        np.testing.assert_array_equal(rr, r_or)
        np.testing.assert_array_equal(b, b_or)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rmax = min(k, m)
    rec = torch.zeros((G, rmax, bb), dtype=torch.uint8, device="cuda")
    rec_rows = torch.zeros((G, rmax), dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 7, dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, dev(recv), dev(rows), rec, rec_rows, status=st)
    np.testing.assert_array_equal(host(st), s_or)
    np.testing.assert_array_equal(host(rec_rows), exp_rows)
    got = host(rec)
    mask = exp_rows != 255
    np.testing.assert_array_equal(got[mask], exp[mask])


@pytest.mark.parametrize("ring", [4, 5])
@pytest.mark.parametrize("bb", [2040, 1544, 2048])
def test_stream_ring_too_small_for_block(tuned_engine, oracle, ring, bb):
    """A ring must hold blocks x and x + 1 from block x's head piece: up to
    (1024 - gcd(bb, 1024) + 2 bb + 1023) / 1024 slots (5 for bb = 2040 or 1544, 4 for
    2048).  With a smaller ring the library does not launch gf_stream (it would read a
    slot whose piece was never issued); the result stays bit-exact either way."""
    engine = tuned_engine
    engine.set_option("stream_grid", 1)
    engine.set_option("stream_ring", ring)
    k, m, r, G = 8, 4, 3, 9
    data = synth.group_data(bb + ring, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    streamed = "gf_stream" in fec.last_kernels()
    assert streamed == (bb == 2048 or ring >= 5)
    assert rc == 0
    np.testing.assert_array_equal(p_gpu, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 5 + bb, shuffle=True)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=True)
    assert ("gf_stream" in fec.last_kernels()) == streamed
    np.testing.assert_array_equal(s, s_or)
    np.testing.assert_array_equal(rr, r_or)
    np.testing.assert_array_equal(b, b_or)


# ------------------------------------------------- non-default launch options
OPTION_SETS = [
    {"xor_slots": 3, "xor_waves": 3}, {"xor_slots": 4, "xor_waves": 2}, {"xor_waves": 1},
    {"dma": 0}, {"stream": 0}, {"stream": 0, "pd": 1}, {"stream": 0, "pd": 3},
    {"stream": 0, "flat": 0}, {"enc_rc": 4}, {"enc_rc": 2}, {"prep_lane": 0},
    {"stream_ring": 36}, {"host_chunk_mb": 1, "host_min_groups": 1}, {"const_enc": 0},
    {"stream_static": 0}, {"bsyn": 0}, {"bsyn_depth": 5}, {"bsyn_depth": 7}, {"ring_split": 0},
    {"dcol": 0}, {"dcol_depth": 8},
    {"psyn": 0},
    {"ring_wg": 0, "bsyn_wg": 0, "dcol_wg": 0, "stream_wg": 0},
    {"ring_wg": 3, "bsyn_wg": 5, "psyn_wg": 2, "dcol_wg": 1, "xor_wg": 3, "stream_wg": 2},
]


# measured-and-rejected variants and timing probes are not options of the product ABI
# (DESIGN.md section 3.7): qfec_ctx_set_option refuses them with -2
REMOVED_OPTIONS = ["psyn_ablate", "enc_split", "wide_st", "stream_rc16", "dcol_rows", "dcol_cache",
                   "psyn_jump", "psyn_pf", "psyn_depth", "ring_nt", "dec_nt", "stream_jump", "pp_hash",
                   "bsyn_ring"]


@pytest.mark.parametrize("name", REMOVED_OPTIONS)
def test_removed_options_refused(engine, name):
    with pytest.raises(fec.FecError) as e:
        engine.set_option(name, 1)
    assert e.value.rc == -2


@pytest.mark.parametrize("opts", OPTION_SETS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_options_parity(tuned_engine, oracle, opts):
    """Every launch option the library accepts produces the oracle's bytes."""
    engine = tuned_engine
    for name, v in opts.items():
        engine.set_option(name, v)
        assert engine.get_option(name) == v
    for (k, m, bb, r) in [(10, 1, 1352, 1), (32, 4, 1352, 2), (16, 8, 9008, 5), (17, 6, 136, 6),
                          (128, 16, 9008, 8)]:
        G = 7
        data = synth.group_data(555 + k + m, k, bb, G)
        p_or, rc_or = oracle.encode_batch(k, m, bb, data)
        p_gpu, rc = gpu_encode(engine, k, m, bb, data)
        assert rc == rc_or
        np.testing.assert_array_equal(p_gpu, p_or)
        rows, src = synth.loss_patterns(k, m, r, G, 99 + k, shuffle=True)
        recv = synth.assemble_received(data, p_or, src)
        b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
        b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=True)
        np.testing.assert_array_equal(s, s_or)
        np.testing.assert_array_equal(rr, r_or)
        np.testing.assert_array_equal(b, b_or)
        if "host_chunk_mb" in opts:
            b2, rr2, s2 = engine.decode_host(k, m, bb, recv, rows)
            np.testing.assert_array_equal(b2, b_or)


def test_option_errors(tuned_engine):
    with pytest.raises(fec.FecError):
        tuned_engine.set_option("no_such_option", 1)
    with pytest.raises(fec.FecError):
        tuned_engine.set_option("enc_rc", 3)
    with pytest.raises(fec.FecError):
        tuned_engine.set_option("stream_ring", 99)
    assert tuned_engine.get_option("cus") > 0


def test_last_kernels_reports_launches(tuned_engine):
    """The library names the kernels it launched (bench.py reports these)."""
    import torch
    engine = tuned_engine
    for (k, m, bb, enc, dec) in [
            (10, 1, 1352, "xor_dma_kernel<encode>", "xor_dma_kernel<decode,recovered>"),
            (32, 4, 1352, "gf_ring_kernel<encode,k32m4>", "gf_bsyn_kernel<decode,k32m4>"),
            (32, 3, 1352, "gf_stream_kernel<encode>", "gf_stream_kernel<decode>"),
            (16, 4, 1352, "gf_stream_kernel<encode>", "gf_stream_kernel<decode>")]:
        G = 8
        data = torch.from_numpy(synth.group_data(3, k, bb, G)).cuda()
        parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
        engine.encode(k, m, bb, data, parity)
        assert fec.last_kernels() == enc
        rows, src = synth.loss_patterns(k, m, min(k, m), G, 5)
        rmax = min(k, m)
        rec = torch.zeros((G, rmax, bb), dtype=torch.uint8, device="cuda")
        rr = torch.zeros((G, rmax), dtype=torch.uint8, device="cuda")
        engine.decode_recovered(k, m, bb, data, dev(rows), rec, rr)
        assert fec.last_kernels().endswith(dec)
    engine.set_option("stream", 0)
    data = torch.zeros((4, 32, 1352), dtype=torch.uint8, device="cuda")
    parity = torch.zeros((4, 4, 1352), dtype=torch.uint8, device="cuda")
    engine.encode(32, 4, 1352, data, parity)
    assert fec.last_kernels().startswith("gf_apply_kernel<encode")
    torch.cuda.synchronize()


# ------------------------------------------------- concurrency: streams and contexts
def _case(k, m, bb, r, G, seed):
    data = synth.group_data(seed, k, bb, G)
    rows, src = synth.loss_patterns(k, m, r, G, seed + 1, shuffle=True)
    return data, rows, src


def test_two_contexts_two_streams(oracle):
    """Two contexts on device 0, each on its own stream, running A- and B-shaped batches
    at the same time; both bit-exact vs the oracle (contexts share no state)."""
    import torch
    from quic_amd.fec import FecEngine
    e1, e2 = FecEngine(0), FecEngine(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cases = [(e1, s1, (10, 1, 1352, 1, 512, 71)), (e2, s2, (32, 4, 1352, 2, 256, 72))]
    outs = []
    for eng, st, (k, m, bb, r, G, seed) in cases:
        data, rows, src = _case(k, m, bb, r, G, seed)
        with torch.cuda.stream(st):
            d = dev(data)
            p = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
            rec = torch.zeros((G, min(k, m), bb), dtype=torch.uint8, device="cuda")
            rr = torch.zeros((G, min(k, m)), dtype=torch.uint8, device="cuda")
            b = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
            sd = dev(src)
            rw = dev(rows)
        outs.append((eng, st, k, m, bb, r, G, data, rows, src, d, p, rec, rr, b, sd, rw))
    torch.cuda.synchronize()
    for _ in range(3):   # interleave the enqueues of the two contexts
        for (eng, st, k, m, bb, r, G, data, rows, src, d, p, rec, rr, b, sd, rw) in outs:
            with torch.cuda.stream(st):
                assert eng.encode(k, m, bb, d, p, stream=st.cuda_stream) == 0
                fec.synth_gather(d, p, sd, b, k, m, bb, stream=st.cuda_stream)
                eng.decode_recovered(k, m, bb, b, rw, rec, rr, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for (eng, st, k, m, bb, r, G, data, rows, src, d, p, rec, rr, b, sd, rw) in outs:
        p_or, _ = oracle.encode_batch(k, m, bb, data)
        np.testing.assert_array_equal(host(p), p_or)
        recv = synth.assemble_received(data, p_or, src)
        b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
        exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
        np.testing.assert_array_equal(host(rr), exp_rows)
        mask = exp_rows != 255
        np.testing.assert_array_equal(host(rec)[mask], exp[mask])
    e1.close()
    e2.close()


def test_one_context_two_streams_decode(tuned_engine, oracle):
    """Two decodes of one context enqueued on two streams back to back share the decode
    workspace; the library orders the second behind the first, so both are exact."""
    import torch
    engine = tuned_engine
    k, m, bb = 32, 4, 1352
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    runs = []
    for i, (r, G) in enumerate([(4, 4096), (1, 4096)]):
        data, rows, src = _case(k, m, bb, r, G, 300 + i)
        p_or, _ = oracle.encode_batch(k, m, bb, data)
        recv = synth.assemble_received(data, p_or, src)
        rec = torch.zeros((G, 4, bb), dtype=torch.uint8, device="cuda")
        rr = torch.zeros((G, 4), dtype=torch.uint8, device="cuda")
        runs.append((recv, rows, dev(recv), dev(rows), rec, rr))
    torch.cuda.synchronize()
    for (recv, rows, b, rw, rec, rr), st in zip(runs, (s1, s2)):
        engine.decode_recovered(k, m, bb, b, rw, rec, rr, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for (recv, rows, b, rw, rec, rr) in runs:
        b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
        exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
        np.testing.assert_array_equal(host(rr), exp_rows)
        mask = exp_rows != 255
        np.testing.assert_array_equal(host(rec)[mask], exp[mask])


# ------------------------------------------------- config C: one GPU's shard
def test_config_c_shard_round_trip(engine, oracle):
    """BASELINE.json configs[3]: 1,048,576 groups of (32 + 4) x 1350 B split over 8 GPUs;
    one GPU's shard is 131,072 groups (rank 3's range of the global stream here).  Encode,
    lose 2 data blocks per group, decode in the recovered-blocks layout: every recovered
    block equals its original; sampled groups match the oracle byte for byte."""
    import torch
    from quic_amd import shard
    k, m, bb, r = 32, 4, 1352, 2
    g0, G = shard.strong_range(1048576, 8, 3)
    assert G == 131072
    data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_fill(data, seed=77, byte_offset=shard.data_byte_offset(g0, k, bb))
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    assert engine.encode(k, m, bb, data, parity) == 0
    rows, src = synth.loss_patterns(k, m, r, G, shard.loss_seed(77, 3))
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_gather(data, parity, dev(src), blocks, k, m, bb)
    rec = torch.zeros((G, 4, bb), dtype=torch.uint8, device="cuda")
    rr = torch.zeros((G, 4), dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 9, dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, blocks, dev(rows), rec, rr, status=st)
    torch.cuda.synchronize()
    assert int(st.abs().max()) == 0
    got = rr != 255
    assert bool((got.sum(dim=1) == r).all())
    g_idx = torch.arange(G, device="cuda")[:, None].expand(G, 4)[got]
    assert torch.equal(rec[got], data[g_idx, rr.long()[got]])
    # the shard is the global stream at its offset
    np.testing.assert_array_equal(host(data[1]).ravel(),
                                  synth.stream_bytes(77, (g0 + 1) * k * bb, k * bb))
    sample = [0, 4097, G - 1]
    p_or, _ = oracle.encode_batch(k, m, bb, host(data[sample]))
    np.testing.assert_array_equal(host(parity[sample]), p_or)
    del data, parity, blocks, rec
    torch.cuda.empty_cache()


# ------------------------------------------------- config D at its production size
def test_config_d_full_size_round_trip(engine, oracle):
    """BASELINE.json configs[4]: 65,536 groups of (128 + 16) x 9000 B (bb 9008), 8 data
    blocks lost per group and a random 8-subset of the parity rows received, decoded in the
    recovered-blocks layout (the bench default; 165 GB resident).  At this size every
    workgroup of the default grid streams 256 groups x 128 blocks through its 32-bit
    counters and the re-read tail.  Every recovered block equals its original; sampled
    groups match the oracle byte for byte, parity and recovered blocks."""
    import torch
    k, m, bb, r, G = 128, 16, 9008, 8, 65536
    data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_fill(data, seed=4242)
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    assert engine.encode(k, m, bb, data, parity) == 0
    assert "gf_dcol" in fec.last_kernels()
    rows, src = synth.loss_patterns(k, m, r, G, 99)
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_gather(data, parity, dev(src), blocks, k, m, bb)
    rec = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    rr = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 9, dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, blocks, dev(rows), rec, rr, status=st)
    kern = fec.last_kernels()
    torch.cuda.synchronize()
    assert "gf_dcol_kernel<decode" in kern, kern
    assert int(st.abs().max()) == 0
    got = rr != 255
    assert bool((got.sum(dim=1) == r).all())
    # compare in slices of groups (the gathered originals are 4.7 GB)
    for a in range(0, G, 8192):
        sl = slice(a, a + 8192)
        g_got = got[sl]
        g_idx = torch.arange(a, a + 8192, device="cuda")[:, None].expand(8192, m)[g_got]
        assert torch.equal(rec[sl][g_got], data[g_idx, rr[sl].long()[g_got]]), a
    sample = [0, 255, 256, 40961, G - 1]   # first/last groups of a workgroup's stream
    d_np = host(data[sample])
    p_or, _ = oracle.encode_batch(k, m, bb, d_np)
    np.testing.assert_array_equal(host(parity[sample]), p_or)
    recv = synth.assemble_received(d_np, p_or, src[sample])
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows[sample])
    exp, exp_rows = expected_recovered(k, m, bb, rows[sample], b_or, r_or, s_or)
    np.testing.assert_array_equal(host(rr[sample]), exp_rows)
    mask = exp_rows != 255
    np.testing.assert_array_equal(host(rec[sample])[mask], exp[mask])
    del data, parity, blocks, rec
    torch.cuda.empty_cache()


# ------------------------------------------------- gf_stream at other block sizes
@pytest.mark.parametrize("bb", [1344, 1000, 520, 136, 2048, 8, 1352])
@pytest.mark.parametrize("k,m,r", [(32, 4, 2), (10, 3, 3), (6, 8, 5), (5, 5, 4), (15, 12, 11)])
def test_stream_any_small_block(engine, oracle, bb, k, m, r):
    """Groups whose padded blocks are at most 2 KiB (quic_fec_group.cc:344-352 pads to the
    group's longest packet) run the streaming kernel, not gf_apply; bit-exact vs the
    oracle, encode and both decode layouts."""
    import torch
    G = 9   # odd k with bb % 16 == 8: every other group starts 8 bytes off 16
    data = synth.group_data(bb + 17 * k + m, k, bb, G)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    assert fec.last_kernels().startswith(("gf_stream_kernel<encode", "gf_ring_kernel<encode"))
    assert rc == rc_or == 0
    np.testing.assert_array_equal(p_gpu, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 3 + bb, shuffle=True)
    recv = synth.assemble_received(data, p_or, src)
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=True)
    dec = ("gf_bsyn_kernel<decode" if (k, m, bb) == (32, 4, 1352) else
           "gf_psyn_kernel<decode" if (k, m, bb) == (5, 5, 1352) else "gf_stream_kernel<decode")
    assert dec in fec.last_kernels()
    np.testing.assert_array_equal(s, s_or)
    np.testing.assert_array_equal(rr, r_or)
    np.testing.assert_array_equal(b, b_or)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rmax = min(k, m)
    rec = torch.zeros((G, rmax, bb), dtype=torch.uint8, device="cuda")
    rec_rows = torch.zeros((G, rmax), dtype=torch.uint8, device="cuda")
    engine.decode_recovered(k, m, bb, dev(recv), dev(rows), rec, rec_rows)
    assert dec in fec.last_kernels()
    np.testing.assert_array_equal(host(rec_rows), exp_rows)
    mask = exp_rows != 255
    np.testing.assert_array_equal(host(rec)[mask], exp[mask])


# ------------------------------------------------- the reference's FEC presets
PRESETS = [(5, 5), (10, 10), (10, 15), (10, 20), (15, 15), (250, 5)]   # quic_fec_group.cc:22-82


PSYN = {(10, 10), (10, 15), (10, 20), (15, 15), (5, 5)}   # gf_psyn's compiled syndrome decode
RING_ENC = {(5, 5), (10, 10), (10, 15), (10, 20), (15, 15), (250, 5)}   # gf_ring's schedule


@pytest.mark.parametrize("opts", [{}, {"stream_grid": 1}, {"psyn": 0},
                                  {"psyn": 0, "stream_grid": 1}, {"stream_static": 0},
                                  {"ring_wide": 0}, {"ring_wide": 0, "stream_grid": 1},
                                  {"psyn_wide": 2}, {"psyn_wide": 0, "stream_grid": 1}],
                         ids=["default", "grid1", "runtime", "runtime_grid1", "no_ring",
                              "ring_plain", "ring_plain_grid1", "psyn_wide_all", "psyn_plain_grid1"])
@pytest.mark.parametrize("k,m", PRESETS)
def test_reference_presets_stream(tuned_engine, oracle, k, m, opts):
    """QuicR's negotiated configurations with 1350-byte payloads (bb = 1352): odd k puts every
    other group 8 bytes off a 16-byte boundary, m > 8 and more than 8 losses cut the run-time
    decode's outputs into chunks.  Encodes run gf_ring's static schedule for every preset
    (gf_stream with stream_static = 0; odd k streams every other group 8 bytes into its
    16-byte aligned stream);
    decodes run gf_psyn
    (compiled syndromes + Gauss-Jordan) for the m >= 7 presets and gf_stream for the others,
    never gf_apply; with psyn = 0, the run-time gf_stream decode (nibble-jump products) for
    every preset.  The (5, 5) encode writes its parity through LDS-staged wide stores.  Bit-exact vs the oracle in every decode layout, with as many losses as
    the code allows (min(k, m)), with half of them and with one; grid 1: one workgroup
    streams every unit."""
    engine = tuned_engine
    for name, v in opts.items():
        engine.set_option(name, v)
    bb, G = 1352, 11
    data = synth.group_data(9000 + k + m, k, bb, G)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    enc = ("gf_ring_kernel<encode" if (k, m) in RING_ENC and opts.get("stream_static", 1)
           else "gf_stream_kernel<encode")
    assert fec.last_kernels().startswith(enc), fec.last_kernels()
    assert rc == rc_or == 0
    np.testing.assert_array_equal(p_gpu, p_or)
    dec = ("gf_psyn_kernel<decode" if (k, m) in PSYN and opts.get("psyn", 1)
           else "gf_stream_kernel<decode")
    for r in sorted({min(k, m), min(k, m) // 2, 1}):
        rows, src = synth.loss_patterns(k, m, r, G, 31 + r, shuffle=True)
        recv = synth.assemble_received(data, p_or, src)
        s_or = check_decodes(engine, oracle, k, m, bb, recv, rows, dec)
        assert (s_or == 0).all()
        assert "gf_apply" not in fec.last_kernels()


@pytest.mark.parametrize("wide", [0, 2])
@pytest.mark.parametrize("grid", [1, 2, 0])
@pytest.mark.parametrize("k,m", sorted(PSYN))
def test_psyn_decode_patterns(tuned_engine, oracle, k, m, grid, wide):
    """The preset decode (gf_psyn: syndromes of every parity row with the compiled code,
    Gauss-Jordan replayed on the data) on hand-built receive sets: no loss, 1 .. min(k, m)
    losses with first / scattered / last parity rows in any arrival order (blocks streamed
    from any slot, odd slots of odd-k groups 8 bytes off a 16-byte boundary), a repeated
    data row (an extra block with run-time coefficients), malformed sets (a repeated parity
    row: singular; a row tag past k + m: status -3, group unchanged); the grid capped so a
    wave streams many groups back to back (the next group's blocks are prefetched across
    the previous group's stores, up to 16 x 2 x min(k, m) of them)."""
    engine = tuned_engine
    engine.set_option("stream_grid", grid)
    engine.set_option("psyn_wide", wide)
    bb = 1352
    rmax = min(k, m)
    rng = np.random.default_rng(500 + 7 * k + m + grid)
    G = 26
    data = synth.group_data(1901 + k + m + grid, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)

    def lose(lost, par):
        keep = [x for x in range(k) if x not in set(lost)]
        return keep + [k + y for y in par]
    base = [
        list(range(k)),
        lose([0], [0]), lose([k - 1], [m - 1]), lose([3], [m // 2]),
        lose(list(range(rmax)), list(range(rmax))),
        lose(list(range(k - rmax, k)), list(range(m - rmax, m))),
        lose(sorted(rng.choice(k, rmax, replace=False)), sorted(rng.choice(m, rmax, replace=False))),
        lose([1, 4], [m - 1, 0]),
    ]
    dup = list(range(k))                      # row a + 1 twice, row a missing, parity row 2
    a, b = (5, 7) if k >= 8 else (1, 3)
    dup[a] = a + 1
    dup[b] = k + 2
    sets = base + [dup]
    while len(sets) < G - 2:
        r = int(rng.integers(0, rmax + 1))
        sets.append(lose(sorted(rng.choice(k, r, replace=False)),
                         sorted(rng.choice(m, r, replace=False))))
    rows = np.zeros((G, k), np.uint8)
    src = np.zeros((G, k), np.int16)
    for g, st in enumerate(sets):
        st = np.array(st)
        if g % 2:
            st = st[rng.permutation(k)]
        rows[g] = st
        src[g] = st
    recv = synth.assemble_received(data[:G - 2], p_or[:G - 2], src[:G - 2])
    ok_rows = rows[:G - 2]
    s_or = check_decodes(engine, oracle, k, m, bb, recv, ok_rows, "gf_psyn_kernel<decode")
    assert (s_or == 0).all()
    # malformed: a repeated parity row (singular), a row tag past k + m
    bad = np.stack([np.array(lose([2, 3], [1, 1])), np.array(lose([4], [0]))]).astype(np.uint8)
    bad[1, -1] = k + m + 3
    bsrc = np.where(bad < k + m, bad, 0).astype(np.int16)
    brecv = synth.assemble_received(data[:2], p_or[:2], bsrc)
    b, rr, st = gpu_decode(engine, k, m, bb, brecv, bad, inplace=True)
    assert st.tolist() == [-3, -3]
    np.testing.assert_array_equal(rr, bad)
    np.testing.assert_array_equal(b, brecv)


def test_psyn_grid_per_code(oracle):
    """QuicR switches presets at run time (quic_connection.cc:822-966), so one context decodes
    several codes.  Each code's gf_psyn grid is its own kernel's occupancy answer: decoding
    (10, 20) first must not fix the grid of a later (10, 10) decode (one cache per kernel)."""
    import torch
    bb, G = 1352, 65536

    def grid_of(eng, k, m):
        rows, src = synth.loss_patterns(k, m, 1, 4, 17, shuffle=False)
        rows = np.repeat(rows[:1], G, axis=0)
        blocks = torch.zeros((G, k, bb), dtype=torch.uint8, device="cuda")
        d_rows = torch.from_numpy(rows).cuda()
        rec = torch.empty((G, min(k, m), bb), dtype=torch.uint8, device="cuda")
        rec_rows = torch.empty((G, min(k, m)), dtype=torch.uint8, device="cuda")
        st = torch.empty((G,), dtype=torch.int32, device="cuda")
        eng.decode_recovered(k, m, bb, blocks, d_rows, rec, rec_rows, st)
        torch.cuda.synchronize()
        assert "gf_psyn_kernel" in fec.last_kernels()
        return fec.last_grids()["gf_psyn_kernel"]

    fresh = {}
    for km in [(10, 10), (10, 20), (15, 15)]:
        e = fec.FecEngine(0)
        fresh[km] = grid_of(e, *km)
        e.close()
    e = fec.FecEngine(0)
    for km in [(10, 20), (10, 10), (15, 15), (10, 10)]:
        assert grid_of(e, *km) == fresh[km], km
    e.close()
    # the codes do differ in occupancy, so the check has teeth
    assert fresh[(10, 10)] != fresh[(10, 20)]


def test_workspace_eager_capture_other_stream():
    """The decode workspace is one per context: an eager decode on stream A, then
    a graph capture begun on A, then an eager decode on stream B.  B's prep must not overwrite
    the tables A's eager decode is still reading: ws_end records an event after every eager
    decode and ws_begin on B waits for it, whatever A does meanwhile.  Both decodes are
    checked by their property (every lost data block restored)."""
    import torch
    k, m, bb = 32, 4, 1352
    eng = fec.FecEngine(0)
    ga, gb = 65536, 8192
    eng.reserve(k, m, bb, ga)

    def setup(G, lost, par, seed):
        gen = torch.Generator(device="cuda").manual_seed(seed)
        data = torch.randint(0, 256, (G, k, bb), dtype=torch.uint8, device="cuda", generator=gen)
        parity = torch.empty((G, m, bb), dtype=torch.uint8, device="cuda")
        eng.encode(k, m, bb, data, parity)
        recv = data.clone()
        rows = torch.arange(k, dtype=torch.uint8, device="cuda").repeat(G, 1)
        for x, y in zip(lost, par):
            recv[:, x] = parity[:, y]
            rows[:, x] = k + y
        rec = torch.full((G, m, bb), 0x5A, dtype=torch.uint8, device="cuda")
        rr = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
        st = torch.full((G,), 7, dtype=torch.int32, device="cuda")
        return data, recv, rows, rec, rr, st

    A = setup(ga, [0, 1], [0, 1], 1)
    B = setup(gb, [5, 9, 30], [3, 2, 1], 2)
    C = setup(16, [2], [0], 3)                 # captured, never replayed
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    eng.decode_recovered(k, m, bb, A[1], A[2], A[3], A[4], A[5], stream=sa.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sa):
        eng.decode_recovered(k, m, bb, C[1], C[2], C[3], C[4], C[5], stream=sa.cuda_stream)
        eng.decode_recovered(k, m, bb, B[1], B[2], B[3], B[4], B[5], stream=sb.cuda_stream)
    torch.cuda.synchronize()
    for (data, recv, rows, rec, rr, st), lost in ((A, [0, 1]), (B, [5, 9, 30])):
        assert bool((st == 0).all())
        srt = sorted(lost)
        assert bool((rr[:, :len(srt)] == torch.tensor(srt, dtype=torch.uint8, device="cuda")).all())
        for j, x in enumerate(srt):
            assert torch.equal(rec[:, j], data[:, x]), (x, j)
    eng.close()


def test_graph_replay_then_eager_other_stream():
    """A decode captured into a graph on stream A and replayed there, then an eager decode of
    the same context on stream B: the eager call's prep must not overwrite the
    tables the replay still reads.  Captured calls use the context's graph workspace, so the
    two never share tables.  The replay is checked after B's decode has been enqueued."""
    import torch
    k, m, bb = 32, 4, 1352
    eng = fec.FecEngine(0)
    ga, gb = 65536, 65536
    eng.reserve(k, m, bb, ga)

    def setup(G, lost, par, seed):
        gen = torch.Generator(device="cuda").manual_seed(seed)
        data = torch.randint(0, 256, (G, k, bb), dtype=torch.uint8, device="cuda", generator=gen)
        parity = torch.empty((G, m, bb), dtype=torch.uint8, device="cuda")
        eng.encode(k, m, bb, data, parity)
        recv = data.clone()
        rows = torch.arange(k, dtype=torch.uint8, device="cuda").repeat(G, 1)
        for x, y in zip(lost, par):
            recv[:, x] = parity[:, y]
            rows[:, x] = k + y
        rec = torch.full((G, m, bb), 0x5A, dtype=torch.uint8, device="cuda")
        rr = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
        st = torch.full((G,), 7, dtype=torch.int32, device="cuda")
        return data, recv, rows, rec, rr, st

    A = setup(ga, [0, 1, 7, 20], [0, 1, 2, 3], 11)
    B = setup(gb, [5], [2], 12)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sa):
        eng.decode_recovered(k, m, bb, A[1], A[2], A[3], A[4], A[5], stream=sa.cuda_stream)
    torch.cuda.synchronize()
    A[3].fill_(0x5A)
    A[5].fill_(7)
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        g.replay()
    eng.decode_recovered(k, m, bb, B[1], B[2], B[3], B[4], B[5], stream=sb.cuda_stream)
    torch.cuda.synchronize()
    for (data, recv, rows, rec, rr, st), lost in ((A, [0, 1, 7, 20]), (B, [5])):
        assert bool((st == 0).all())
        srt = sorted(lost)
        assert bool((rr[:, :len(srt)] == torch.tensor(srt, dtype=torch.uint8, device="cuda")).all())
        for j, x in enumerate(srt):
            assert torch.equal(rec[:, j], data[:, x]), (x, j)
    eng.close()


# ------------------------------------------------- gf_bsyn (compiled (32, 4) decode, B/C)
@pytest.mark.parametrize("depth", [3, 5, 7])
@pytest.mark.parametrize("grid", [1, 2, 0])
def test_bsyn_decode_patterns(tuned_engine, oracle, depth, grid):
    """Configs B/C's decode (syndromes of every parity row with the compiled (32, 4) code, then
    the r x r solve, gf_bsyn_kernel) on hand-built receive sets: no loss, 1-4 losses with
    first / scattered / last parity rows, shuffled arrival (blocks streamed from any slot,
    odd slots 8 bytes off a 16-byte boundary), a repeated data row (an extra with run-time
    coefficients), malformed sets (status -3, group unchanged); the grid capped so a wave
    streams many groups back to back (the next group's blocks are prefetched across the
    previous group's stores)."""
    engine = tuned_engine
    engine.set_option("stream_grid", grid)
    engine.set_option("bsyn_depth", depth)
    k, m, bb = 32, 4, 1352
    rng = np.random.default_rng(300 + depth + grid)
    G = 24
    data = synth.group_data(901 + depth + grid, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)

    def lose(lost, par):
        keep = [x for x in range(k) if x not in set(lost)]
        return keep + [k + y for y in par]
    base = [
        list(range(k)),
        lose([5], [0]), lose([0], [3]), lose([31], [2]),
        lose([3, 4], [0, 1]), lose([0, 31], [2, 3]), lose([7, 19], [1, 3]),
        lose([1, 2, 3], [0, 1, 2]), lose([8, 16, 24], [1, 2, 3]),
        lose([0, 1, 2, 3], [0, 1, 2, 3]), lose([28, 29, 30, 31], [0, 1, 2, 3]),
        lose(sorted(rng.choice(k, 4, replace=False)), [0, 1, 2, 3]),
    ]
    dup = list(range(k))                      # row 6 twice, row 5 missing, parity row 2
    dup[5] = 6
    dup[20] = k + 2
    sets = base + [dup]
    while len(sets) < G - 2:
        r = int(rng.integers(0, 5))
        sets.append(lose(sorted(rng.choice(k, r, replace=False)), sorted(rng.choice(m, r, replace=False))))
    bad1 = lose([3, 4], [1, 1])               # the same parity row twice: singular
    bad2 = lose([10], [1])
    bad2[-1] = 200                            # row tag past k + m
    sets += [bad1, bad2]
    rows = np.zeros((G, k), np.uint8)
    src = np.zeros((G, k), np.int16)
    for g, s in enumerate(sets):
        s = np.array(s)
        if g % 2:
            s = s[rng.permutation(k)]
        rows[g] = s
        src[g] = np.where(s < k + m, s, 0)
    recv = synth.assemble_received(data, p_or, src)
    ok = np.arange(G) < G - 2
    s_or = check_decodes(engine, oracle, k, m, bb, recv[ok], rows[ok],
                         "gf_bsyn_kernel<decode,k32m4>")
    assert (s_or == 0).all()
    b, rr, st = gpu_decode(engine, k, m, bb, recv[~ok], rows[~ok], inplace=True)
    assert st.tolist() == [-3, -3]
    np.testing.assert_array_equal(rr, rows[~ok])
    np.testing.assert_array_equal(b, recv[~ok])


# ------------------------------------------------- gf_dcol (9008-byte blocks, config D)
D_KERNELS = {1: ("gf_dcol_kernel<encode,k128m16", "gf_dcol_kernel<decode,k128m16"),
             0: ("gf_apply_kernel<encode", "gf_apply_kernel<decode")}


D_VARIANTS = [{"dcol": 1}, {"dcol": 1, "dcol_depth": 8}, {"dcol": 0}]


@pytest.mark.parametrize("opts", D_VARIANTS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
@pytest.mark.parametrize("grid", [1, 3, 0])
@pytest.mark.parametrize("k,m,r", [(128, 16, 8), (128, 16, 13), (40, 16, 16), (16, 6, 4)])
def test_tile_many_groups_per_workgroup(tuned_engine, oracle, grid, k, m, r, opts):
    """Config D's kernels with the grid capped so one workgroup streams several groups back
    to back (the DMA prefetch crosses group / unit boundaries and the previous group's stores
    sit in the vmcnt count); every third group has no loss.  dcol = 1: gf_dcol (one wave
    per column tile, units of (group, tile)) at ring depths 6 and 8; dcol = 0: the gf_apply
    fallback."""
    engine = tuned_engine
    for name, v in opts.items():
        engine.set_option(name, v)
    dcol = opts["dcol"]
    engine.set_option("dcol_grid", grid)
    bb, G = 9008, 7
    data = synth.group_data(4000 + k + m + grid, k, bb, G)
    p_or, rc_or = oracle.encode_batch(k, m, bb, data)
    p_gpu, rc = gpu_encode(engine, k, m, bb, data)
    if (k, m) == (128, 16):
        assert fec.last_kernels().startswith(D_KERNELS[dcol][0])
    assert rc == rc_or == 0
    np.testing.assert_array_equal(p_gpu, p_or)
    rows, src = synth.loss_patterns(k, m, r, G, 71 + grid, shuffle=True)
    rows[::3] = np.arange(k, dtype=rows.dtype)
    src[::3] = np.arange(k, dtype=src.dtype)
    recv = synth.assemble_received(data, p_or, src)
    dec_kernel = D_KERNELS[dcol][1] if (k, m) == (128, 16) else "gf_apply_kernel<decode"
    check_decodes(engine, oracle, k, m, bb, recv, rows, dec_kernel)


def check_decodes(engine, oracle, k, m, bb, recv, rows, dec_kernel):
    """Both in-place layouts and the recovered-blocks layout against the oracle."""
    import torch
    G = recv.shape[0]
    b_or, r_or, s_or = oracle.decode_batch(k, m, bb, recv, rows)
    for inplace in (True, False):
        b, rr, s = gpu_decode(engine, k, m, bb, recv, rows, inplace=inplace)
        assert dec_kernel in fec.last_kernels()
        np.testing.assert_array_equal(s, s_or)
        np.testing.assert_array_equal(rr, r_or)
        np.testing.assert_array_equal(b, b_or)
    exp, exp_rows = expected_recovered(k, m, bb, rows, b_or, r_or, s_or)
    rmax = min(k, m)
    rec = torch.zeros((G, rmax, bb), dtype=torch.uint8, device="cuda")
    rec_rows = torch.zeros((G, rmax), dtype=torch.uint8, device="cuda")
    st = torch.full((G,), 7, dtype=torch.int32, device="cuda")
    engine.decode_recovered(k, m, bb, dev(recv), dev(rows), rec, rec_rows, status=st)
    assert dec_kernel in fec.last_kernels()
    np.testing.assert_array_equal(host(st), s_or)
    np.testing.assert_array_equal(host(rec_rows), exp_rows)
    mask = exp_rows != 255
    np.testing.assert_array_equal(host(rec)[mask], exp[mask])
    return s_or


@pytest.mark.parametrize("opts", [{"dcol": 1}, {"dcol": 1, "dcol_depth": 8}, {"dcol": 0}],
                         ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
@pytest.mark.parametrize("grid", [1, 3, 0])
def test_syndrome_decode_patterns(tuned_engine, oracle, grid, opts):
    """Config D's decode (syndromes of the compiled (128, 16) code, then the r x r solve,
    gf_dcol_kernel; dcol = 0: the gf_apply fallback) on hand-built receive sets: no loss, 16 losses, single and scattered
    parity rows, more than 8 losses (two syndrome exchange rounds), a repeated data row (an
    extra block with run-time coefficients); shuffled arrival; the grid capped so groups
    share workgroups.  Malformed sets (a repeated parity row: singular; a row tag past
    k + m) are where the reference's result is not defined (its elimination runs on a
    singular bit matrix / reads past its Cauchy matrix): status -3, group left unchanged."""
    engine = tuned_engine
    for name, v in opts.items():
        engine.set_option(name, v)
    dcol = opts["dcol"]
    engine.set_option("dcol_grid", grid)
    k, m, bb = 128, 16, 9008
    rng = np.random.default_rng(90 + grid)
    data = synth.group_data(777 + grid, k, bb, 10)
    p_or, _ = oracle.encode_batch(k, m, bb, data)

    def lose(lost, par):
        keep = [x for x in range(k) if x not in set(lost)]
        return keep + [k + y for y in par]
    sets = [
        list(range(k)),                                                  # no loss
        lose(sorted(rng.choice(k, 16, replace=False)), list(range(16))),  # 16 losses
        lose([77], [15]),                                                # one, last parity row
        lose([0, 9, 64, 100, 127], [1, 3, 9, 12, 14]),                   # scattered rows
        lose(list(range(8)), list(range(8))),                            # the bench's pattern
        lose(sorted(rng.choice(k, 9, replace=False)), [0, 2, 4, 5, 6, 8, 10, 13, 15]),
    ]
    dup_data = list(range(k))                 # row 6 twice, row 5 missing, parity row 2
    dup_data[5] = 6
    dup_data[40] = k + 2
    sets.append(dup_data)
    dup_par = lose([3, 4], [3, 3])            # the same parity row twice: singular
    sets.append(dup_par)
    bad = lose([10], [1])
    bad[-1] = 200                             # row tag past k + m
    sets.append(bad)
    sets.append(lose(sorted(rng.choice(k, 12, replace=False)), sorted(rng.choice(m, 12, replace=False))))
    rows = np.zeros((10, k), np.uint8)
    src = np.zeros((10, k), np.int16)
    for g, s in enumerate(sets):
        s = np.array(s)
        if g % 2:
            s = s[rng.permutation(k)]
        rows[g] = s
        src[g] = np.where(s < k + m, s, 0)
    recv = synth.assemble_received(data, p_or, src)
    ok = np.array([g not in (7, 8) for g in range(10)])
    s_or = check_decodes(engine, oracle, k, m, bb, recv[ok], rows[ok], D_KERNELS[dcol][1])
    assert (s_or == 0).all()
    bad = ~ok
    b, rr, st = gpu_decode(engine, k, m, bb, recv[bad], rows[bad], inplace=True)
    assert st.tolist() == [-3, -3]
    np.testing.assert_array_equal(rr, rows[bad])
    np.testing.assert_array_equal(b, recv[bad])
