"""GPU: packet protection next to the FEC path (pp_null.hip) through the C ABI, bit-exact
against the oracle (oracle/pp_oracle.c, itself pinned by null_encrypter_test.cc and
null_decrypter_test.cc in tests/test_pp_oracle.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KAT_AD = b"hello world!"
KAT_PT = b"goodbye!"
KAT_TAG = bytes.fromhex("a06f448a44f8183b4791b213")


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture
def pp_engine(engine):
    """The engine (one FNV-1a-128 chain: six 22-bit limbs; the 64-bit-halves form was removed
    in r05)."""
    yield engine


def test_known_answer_through_gpu(pp_engine):
    engine = pp_engine
    import torch
    ad = _dev(np.frombuffer(KAT_AD, np.uint8).reshape(1, -1))
    pt = _dev(np.frombuffer(KAT_PT, np.uint8).reshape(1, -1))
    out = torch.zeros((1, 64), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.null_seal(ad, 12, pt, 8, out, out_len)
    n = int(_host(out_len)[0])
    assert n == 32
    assert _host(out)[0, :n].tobytes() == KAT_AD + KAT_TAG + KAT_PT
    plain = torch.zeros((1, 64), dtype=torch.uint8, device="cuda")
    plen = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.null_open(out, n, 12, plain, plen)
    assert int(_host(plen)[0]) == 8
    assert _host(plain)[0, :8].tobytes() == KAT_PT


@pytest.mark.parametrize("n,S,AS", [(1, 64, 16), (63, 200, 21), (300, 1352, 19),
                                    (517, 1400, 33), (70, 9008, 16)])
def test_seal_open_random_vs_oracle(pp_engine, oracle, n, S, AS):
    import torch
    engine = pp_engine
    rng = np.random.default_rng(n * 7 + S)
    ad = rng.integers(0, 256, (n, AS), dtype=np.uint8)
    pt = rng.integers(0, 256, (n, S), dtype=np.uint8)
    ad_len = rng.integers(0, AS + 1, n).astype(np.int32)
    pt_len = rng.integers(0, S + 1, n).astype(np.int32)
    pt_len[: min(n, 3)] = S                    # full-size packets
    ad_len[: min(n, 2)] = AS
    out_stride = (AS + 12 + S) // 4 * 4        # the largest packets may not fit
    exp, eres = oracle.null_seal_batch(ad, ad_len, pt, pt_len, out_stride)
    out = torch.zeros((n, out_stride), dtype=torch.uint8, device="cuda")
    out_len = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    engine.null_seal(_dev(ad), _dev(ad_len), _dev(pt), _dev(pt_len), out, out_len)
    got, gres = _host(out), _host(out_len)
    assert np.array_equal(gres, eres)
    assert np.array_equal(got, exp)

    # open: tamper with some packets, cut some short
    pkt = exp.copy()
    pkt_len = np.where(eres < 0, ad_len, eres).astype(np.int32)
    bad = rng.choice(n, size=max(1, n // 5), replace=False)
    for i in bad:
        if eres[i] >= 0:
            pos = ad_len[i] + rng.integers(0, pkt_len[i] - ad_len[i])
            pkt[i, pos] ^= 1 << int(rng.integers(0, 8))
    short = rng.choice(n, size=max(1, n // 10), replace=False)
    pkt_len[short] = ad_len[short] + rng.integers(0, 12, len(short)).astype(np.int32)
    o_stride = ((S + 12 + 3) // 4) * 4
    exp_o, eres_o = oracle.null_open_batch(pkt, pkt_len, ad_len, o_stride)
    out_o = torch.zeros((n, o_stride), dtype=torch.uint8, device="cuda")
    len_o = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    engine.null_open(_dev(pkt), _dev(pkt_len), _dev(ad_len), out_o, len_o)
    assert np.array_equal(_host(len_o), eres_o)
    assert np.array_equal(_host(out_o), exp_o)
    assert (eres_o[bad[eres[bad] >= 0]] == -1).all()


def test_unaligned_inputs(engine, oracle):
    # AD and plaintext rows at odd offsets (strides not multiples of 4)
    import torch
    rng = np.random.default_rng(5)
    n, AS, S = 130, 13, 1351
    ad = rng.integers(0, 256, (n, AS), dtype=np.uint8)
    pt = rng.integers(0, 256, (n, S), dtype=np.uint8)
    exp, eres = oracle.null_seal_batch(ad, np.full(n, AS, np.int32), pt,
                                       np.full(n, S, np.int32), 1380)
    out = torch.zeros((n, 1380), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.null_seal(_dev(ad), AS, _dev(pt), S, out, out_len)
    assert np.array_equal(_host(out_len), eres)
    assert np.array_equal(_host(out), exp)


@pytest.mark.parametrize("k,m,G", [(10, 1, 37), (32, 4, 19), (5, 5, 8)])
def test_encode_seal_vs_oracle(engine, oracle, k, m, G):
    import torch
    bb = 1352
    rng = np.random.default_rng(k * 100 + m)
    data = rng.integers(0, 256, (G, k, bb), dtype=np.uint8)
    hdr = rng.integers(0, 256, (G * m, 20), dtype=np.uint8)
    hdr_len = rng.integers(9, 21, G * m).astype(np.int32)
    parity_exp, rc = oracle.encode_batch(k, m, bb, data)
    assert rc == 0
    exp, eres = oracle.null_seal_batch(hdr, hdr_len, parity_exp.reshape(G * m, bb),
                                       np.full(G * m, bb, np.int32), 1400)
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    pkt = torch.zeros((G * m, 1400), dtype=torch.uint8, device="cuda")
    pkt_len = torch.zeros(G * m, dtype=torch.int32, device="cuda")
    engine.encode_seal(k, m, bb, _dev(data), parity, _dev(hdr), _dev(hdr_len), pkt, pkt_len)
    assert np.array_equal(_host(parity), parity_exp)
    assert np.array_equal(_host(pkt_len), eres)
    assert np.array_equal(_host(pkt), exp)


def test_full_size_round_trip(engine):
    """BASELINE config A's 65,536 FEC packets: seal, open, every packet accepted and equal
    to its parity block; one flipped bit per packet in a second copy, every one rejected."""
    import torch
    from quic_amd import fec
    G, k, bb = 65536, 10, 1352
    data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_fill(data, seed=99)
    parity = torch.empty((G, 1, bb), dtype=torch.uint8, device="cuda")
    hdr = torch.arange(G * 16, dtype=torch.int32, device="cuda").to(torch.uint8).view(G, 16)
    pkt = torch.zeros((G, 1380), dtype=torch.uint8, device="cuda")
    pkt_len = torch.zeros(G, dtype=torch.int32, device="cuda")
    engine.encode_seal(k, 1, bb, data, parity, hdr, 16, pkt, pkt_len)
    plain = torch.zeros((G, bb + 12), dtype=torch.uint8, device="cuda")   # holds the ciphertext
    plen = torch.zeros(G, dtype=torch.int32, device="cuda")
    engine.null_open(pkt, pkt_len, 16, plain, plen)
    torch.cuda.synchronize()
    assert bool((pkt_len == 16 + 12 + bb).all())
    assert bool((plen == bb).all())
    assert torch.equal(plain[:, :bb], parity.view(G, bb))
    pos = 16 + torch.randint(0, 12 + bb, (G,), device="cuda")
    bad = pkt.clone()
    rows = torch.arange(G, device="cuda")
    bad[rows, pos] ^= 1
    engine.null_open(bad, pkt_len, 16, plain, plen)
    torch.cuda.synchronize()
    assert bool((plen == -1).all())


def test_lengths_beyond_row_stride_rejected(engine, oracle):
    # a length larger than its row's stride would read the next row (past the buffer for
    # the last one): rejected with -1 and nothing written, in the oracle and on the GPU
    import torch
    rng = np.random.default_rng(9)
    n, AS, S = 6, 16, 64
    ad = rng.integers(0, 256, (n, AS), dtype=np.uint8)
    pt = rng.integers(0, 256, (n, S), dtype=np.uint8)
    ad_len = np.array([16, 17, 0, 16, 3, 16], np.int32)
    pt_len = np.array([64, 10, 65, 0, 64, 1000], np.int32)
    exp, eres = oracle.null_seal_batch(ad, ad_len, pt, pt_len, 2048)
    assert list(eres < 0) == [False, True, True, False, False, True]
    out = torch.zeros((n, 2048), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.null_seal(_dev(ad), _dev(ad_len), _dev(pt), _dev(pt_len), out, out_len)
    assert np.array_equal(_host(out_len), eres)
    assert np.array_equal(_host(out), exp)
    pkt = exp[:, :128].copy()
    pkt_len = np.array([92, 129, 40, 28, 200, 12], np.int32)   # 129, 200 > stride 128
    adl = np.array([16, 16, 0, 16, 3, 12], np.int32)
    exp_o, eres_o = oracle.null_open_batch(pkt, pkt_len, adl, 256)
    assert eres_o[1] == -1 and eres_o[4] == -1 and not exp_o[1].any() and not exp_o[4].any()
    out_o = torch.zeros((n, 256), dtype=torch.uint8, device="cuda")
    len_o = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.null_open(_dev(pkt), _dev(pkt_len), _dev(adl), out_o, len_o)
    assert np.array_equal(_host(len_o), eres_o)
    assert np.array_equal(_host(out_o), exp_o)


# ---------------------------------------------------------------- grouped forms
def _group_packets(oracle, k, m, bb, G, rng, hmax=20):
    """Data blocks whose payloads are zero-padded to bb, their parity, per-packet headers
    and plaintext lengths, and the oracle's wire packets for packet p = g*(k+m)+i."""
    per = k + m
    n = G * per
    data = rng.integers(0, 256, (G, k, bb), dtype=np.uint8)
    pt_len = np.full((G, per), bb, np.int32)
    pt_len[:, :k] = rng.integers(max(0, bb - 300), bb + 1, (G, k))
    for g in range(G):
        for i in range(k):
            data[g, i, pt_len[g, i]:] = 0          # a data block is its payload, zero-padded
    parity, rc = oracle.encode_batch(k, m, bb, data)
    assert rc == 0
    rows_pt = np.concatenate([data, parity], axis=1).reshape(n, bb)
    hdr = rng.integers(0, 256, (n, hmax), dtype=np.uint8)
    hdr_len = rng.integers(9, hmax + 1, n).astype(np.int32)
    stride = (hmax + 12 + bb + 3) // 4 * 4
    pkt, plen = oracle.null_seal_batch(hdr, hdr_len, rows_pt, pt_len.reshape(n), stride)
    assert (plen >= 0).all()
    return data, parity, pt_len.reshape(n), hdr, hdr_len, pkt, plen


@pytest.mark.parametrize("k,m,G,encode", [(10, 1, 37, True), (5, 5, 21, False),
                                          (32, 4, 9, True), (10, 20, 6, False)])
def test_seal_groups_vs_oracle(pp_engine, oracle, k, m, G, encode):
    """Every data and FEC packet of each group in one launch, bit-exact with the oracle's
    per-packet NullEncrypter (quic_packet_creator.cc:733-736, :948-953)."""
    import torch
    engine = pp_engine
    bb = 1352
    rng = np.random.default_rng(k * 1000 + m * 10 + G)
    data, parity, pt_len, hdr, hdr_len, exp, eres = _group_packets(oracle, k, m, bb, G, rng)
    n = G * (k + m)
    d_par = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda") if encode else _dev(parity)
    pkt = torch.zeros((n, exp.shape[1]), dtype=torch.uint8, device="cuda")
    pkt_len = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    engine.seal_groups(k, m, bb, _dev(data), d_par, _dev(hdr), _dev(hdr_len), _dev(pt_len),
                       pkt, pkt_len, encode=encode)
    assert np.array_equal(_host(d_par), parity)
    assert np.array_equal(_host(pkt_len), eres)
    assert np.array_equal(_host(pkt), exp)


def _expected_open_decode(oracle, k, m, bb, G, pkt, pkt_len, hdr_len):
    """open_len, blocks, rows as qfec_open_decode_batch documents them, from the oracle's
    NullDecrypter; then the oracle decode of the groups that have k opened packets."""
    from tests.test_gpu_parity import expected_recovered
    per = k + m
    n = G * per
    o_stride = (bb + 12 + 3) // 4 * 4 + 64
    rcv = pkt_len >= 0
    plain, res = oracle.null_open_batch(pkt, np.where(rcv, pkt_len, hdr_len), hdr_len, o_stride)
    open_len = np.where(rcv & (res <= bb), res, -1).astype(np.int32)
    blocks = np.zeros((G, k, bb), np.uint8)
    rows = np.full((G, k), 255, np.uint8)
    for g in range(G):
        ol = open_len[g * per:(g + 1) * per]
        avail = [j for j in range(m) if ol[k + j] >= 0]
        h = 0
        for i in range(k):
            p = g * per + i
            if ol[i] >= 0:
                rows[g, i] = i
                blocks[g, i, :ol[i]] = plain[p, :ol[i]]
            elif h < len(avail):
                j = avail[h]
                h += 1
                rows[g, i] = k + j
                q = g * per + k + j
                blocks[g, i, :ol[k + j]] = plain[q, :ol[k + j]]
    ok = (rows != 255).all(axis=1)
    rec = np.zeros((G, min(k, m), bb), np.uint8)
    rec_rows = np.full((G, min(k, m)), 255, np.uint8)
    status = np.full(G, -3, np.int32)
    if ok.any():
        b_or, r_or, s_or = oracle.decode_batch(k, m, bb, blocks[ok], rows[ok])
        r_ok, rr_ok = expected_recovered(k, m, bb, rows[ok], b_or, r_or, s_or)
        rec[ok], rec_rows[ok], status[ok] = r_ok, rr_ok, s_or
    return open_len, blocks, rows, ok, rec, rec_rows, status


@pytest.mark.parametrize("k,m,G,bb", [(10, 1, 40, 1352), (5, 5, 30, 1352), (32, 4, 12, 1352),
                                      (10, 20, 9, 1352), (8, 1, 16, 1350)])
def test_open_decode_vs_oracle(pp_engine, oracle, k, m, G, bb):
    """Receiver batch: open (NullDecrypter) every packet of each group, place the data
    plaintexts, fill the holes with opened FEC packets, decode -- against the oracle's open
    and decode.  Lost packets, tampered packets (rejected by the tag) and one group that
    cannot be recovered."""
    import torch
    engine = pp_engine
    rng = np.random.default_rng(k * 77 + m + G)
    per, n = k + m, G * (k + m)
    data, parity, pt_len, hdr, hdr_len, pkt, plen = _group_packets(oracle, k, m, bb, G, rng)
    pkt_len = plen.copy()
    q = 0.4 * m / per                                   # about 0.4 m erasures per group
    lost = rng.random(n) < 0.7 * q
    pkt_len[lost] = -1
    bad = np.flatnonzero(~lost & (rng.random(n) < 0.3 * q))
    bad = bad if len(bad) else np.array([n - 1])
    for p in bad:
        pkt[p, hdr_len[p] + int(rng.integers(0, 12 + pt_len[p]))] ^= 1 << int(rng.integers(0, 8))
    pkt_len[0] = -1                                     # group 0: a data packet lost and
    pkt_len[k:per] = -1                                 # no FEC packet left to replace it
    open_len, blocks, rows, ok, rec, rec_rows, status = _expected_open_decode(
        oracle, k, m, bb, G, pkt, pkt_len, hdr_len)
    assert not ok[0] and ok.sum() >= G // 3
    d_blocks = torch.zeros((G, k, bb), dtype=torch.uint8, device="cuda")
    d_rows = torch.zeros((G, k), dtype=torch.uint8, device="cuda")
    d_ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_rec = torch.zeros((G, min(k, m), bb), dtype=torch.uint8, device="cuda")
    d_rr = torch.zeros((G, min(k, m)), dtype=torch.uint8, device="cuda")
    d_st = torch.full((G,), 99, dtype=torch.int32, device="cuda")
    engine.open_decode(k, m, bb, _dev(pkt), _dev(pkt_len), _dev(hdr_len), d_blocks, d_rows, d_ol,
                       d_rec, d_rr, d_st)
    assert np.array_equal(_host(d_ol), open_len)
    assert np.array_equal(_host(d_rows), rows)
    gb = _host(d_blocks)
    filled = rows != 255
    assert np.array_equal(gb[filled], blocks[filled])
    assert np.array_equal(_host(d_st), status)
    assert np.array_equal(_host(d_rr)[ok], rec_rows[ok])
    got_rec = _host(d_rec)
    used = rec_rows != 255
    assert np.array_equal(got_rec[used], rec[used])
    # the recovered blocks are the lost data blocks
    for g in np.flatnonzero(ok):
        for j in range(min(k, m)):
            if rec_rows[g, j] != 255:
                assert np.array_equal(got_rec[g, j], data[g, rec_rows[g, j]])


@pytest.mark.parametrize("chunk", [0, 1], ids=["one_chunk", "many_chunks"])
@pytest.mark.parametrize("k,m,G", [(10, 1, 40), (5, 5, 30), (32, 4, 12), (10, 20, 9)])
def test_host_protected_paths_vs_oracle(oracle, k, m, G, chunk):
    """The sender's and the receiver's per-packet paths from host memory to host memory
    (qfec_encode_seal_groups_batch_host, qfec_open_decode_batch_host), bit-exact with the
    oracle's NullEncrypter / NullDecrypter and decode; many_chunks: one group per pipelined
    chunk (host_chunk_mb = host_min_groups = 1), so H2D, kernels and D2H of successive
    chunks overlap across the staging buffers."""
    import torch
    from quic_amd import fec
    eng = fec.FecEngine(0)
    if chunk:
        eng.set_option("host_chunk_mb", 1)
        eng.set_option("host_min_groups", 1)
    bb = 1352
    rng = np.random.default_rng(k * 31 + m + G + chunk)
    per, n = k + m, G * (k + m)
    data, parity, pt_len, hdr, hdr_len, exp, eres = _group_packets(oracle, k, m, bb, G, rng)
    # sender: data + headers in host memory -> every sealed packet in host memory
    h_pkt = torch.zeros((n, exp.shape[1]), dtype=torch.uint8).pin_memory()
    h_len = torch.full((n,), 7, dtype=torch.int32).pin_memory()
    rc = fec.encode_seal_groups_host_into(eng, k, m, bb, torch.from_numpy(data).pin_memory(),
                                          torch.from_numpy(hdr).pin_memory(),
                                          torch.from_numpy(hdr_len), torch.from_numpy(pt_len),
                                          h_pkt, h_len)
    assert rc == 0
    assert np.array_equal(h_len.numpy(), eres)
    # whole rows: the bytes past a packet are zero (the staging rows are zeroed before the
    # seal), as in the oracle's rows, not an earlier chunk's packets
    assert np.array_equal(h_pkt.numpy(), exp)
    # receiver: lost and tampered packets, one unrecoverable group
    pkt, pkt_len = exp.copy(), eres.copy()
    lost = rng.random(n) < 0.3 * m / per
    pkt_len[lost] = -1
    for p in np.flatnonzero(~lost & (rng.random(n) < 0.1 * m / per))[:3]:
        pkt[p, hdr_len[p] + 3] ^= 0x10
    pkt_len[0] = -1
    pkt_len[k:per] = -1
    open_len, blocks, rows, ok, rec, rec_rows, status = _expected_open_decode(
        oracle, k, m, bb, G, pkt, pkt_len, hdr_len)
    rmax = min(k, m)
    h_rec = torch.zeros((G, rmax, bb), dtype=torch.uint8).pin_memory()
    h_rr = torch.zeros((G, rmax), dtype=torch.uint8).pin_memory()
    h_st = torch.full((G,), 99, dtype=torch.int32).pin_memory()
    h_ol = torch.zeros(n, dtype=torch.int32).pin_memory()
    fec.open_decode_host_into(eng, k, m, bb, torch.from_numpy(pkt).pin_memory(),
                              torch.from_numpy(pkt_len).pin_memory(), torch.from_numpy(hdr_len),
                              h_rec, h_rr, h_st, h_ol)
    assert np.array_equal(h_ol.numpy(), open_len)
    assert np.array_equal(h_st.numpy(), status)
    assert np.array_equal(h_rr.numpy()[ok], rec_rows[ok])
    used = rec_rows != 255
    assert np.array_equal(h_rec.numpy()[used], rec[used])
    eng.close()


def test_open_decode_full_size_a_shape(engine):
    """BASELINE config A's shape, 65,536 groups of (10 + 1) x 1352 B: every packet of every
    group sealed in one launch after the encode, one random packet per group lost, then
    open -> place -> decode: each group's lost data block comes back (a round trip, no
    oracle at this size)."""
    import torch
    from quic_amd import fec
    G, k, m, bb, hl = 65536, 10, 1, 1352, 16
    per, n = k + m, 65536 * 11
    data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    fec.synth_fill(data, seed=5)
    parity = torch.empty((G, m, bb), dtype=torch.uint8, device="cuda")
    hdr = torch.arange(n * hl, dtype=torch.int32, device="cuda").to(torch.uint8).view(n, hl)
    stride = (hl + 12 + bb + 3) // 4 * 4
    pkt = torch.empty((n, stride), dtype=torch.uint8, device="cuda")
    pkt_len = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.seal_groups(k, m, bb, data, parity, hdr, hl, bb, pkt, pkt_len, encode=True)
    torch.cuda.synchronize()
    assert bool((pkt_len == hl + 12 + bb).all())
    lose = torch.randint(0, per, (G,), device="cuda")
    rcv_len = pkt_len.clone().view(G, per)
    rcv_len[torch.arange(G, device="cuda"), lose] = -1
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
    rows = torch.empty((G, k), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    rec = torch.empty((G, 1, bb), dtype=torch.uint8, device="cuda")
    rr = torch.empty((G, 1), dtype=torch.uint8, device="cuda")
    st = torch.empty(G, dtype=torch.int32, device="cuda")
    engine.open_decode(k, m, bb, pkt, rcv_len.view(n), hl, blocks, rows, ol, rec, rr, st)
    torch.cuda.synchronize()
    assert bool((st == 0).all())
    assert bool(((ol.view(G, per) == bb) | (rcv_len < 0)).all())
    lost_data = lose < k
    assert bool((rr[:, 0][lost_data] == lose[lost_data].to(torch.uint8)).all())
    assert bool((rr[:, 0][~lost_data] == 255).all())
    gi = torch.nonzero(lost_data).flatten()
    assert torch.equal(rec[gi, 0], data[gi, lose[gi]])


def test_grouped_argument_limits(engine):
    """k + m = 256 is a valid seal shape but not an open -> decode one (row tag 255 marks an
    unfilled slot); a plaintext length above block_bytes is rejected; both with -2."""
    import torch
    from quic_amd.fec import FecError
    G, k, m, bb = 1, 250, 6, 64
    n = G * (k + m)
    pkt = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    plen = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    blocks = torch.zeros((G, k, bb), dtype=torch.uint8, device="cuda")
    rows = torch.zeros((G, k), dtype=torch.uint8, device="cuda")
    ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    rec = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    rr = torch.zeros((G, m), dtype=torch.uint8, device="cuda")
    with pytest.raises(FecError):
        engine.open_decode(k, m, bb, pkt, plen, 16, blocks, rows, ol, rec, rr)
    data = torch.zeros((G, 4, bb), dtype=torch.uint8, device="cuda")
    par = torch.zeros((G, 2, bb), dtype=torch.uint8, device="cuda")
    hdr = torch.zeros((6, 16), dtype=torch.uint8, device="cuda")
    out = torch.zeros((6, 128), dtype=torch.uint8, device="cuda")
    olen = torch.zeros(6, dtype=torch.int32, device="cuda")
    with pytest.raises(FecError):
        engine.seal_groups(4, 2, bb, data, par, hdr, 16, bb + 1, out, olen)
    torch.cuda.synchronize()


def test_host_seal_unsupported_shape_writes_nothing(oracle):
    """qfec_encode_seal_groups_batch_host where the encode returns -1 (m > 1 and
    block_bytes % 8 != 0, cauchy_256.cpp:1530-1534): -1 and no packet written, as on the
    device path (the parity rows past P0 would otherwise be stale staging bytes sent with
    valid tags)."""
    import torch
    from quic_amd import fec
    eng = fec.FecEngine(0)
    k, m, bb, G = 5, 3, 1350, 4
    n = G * (k + m)
    data = torch.randint(0, 256, (G, k, bb), dtype=torch.uint8)
    pkt = torch.full((n, 1400), 0xA5, dtype=torch.uint8)
    plen = torch.full((n,), 7, dtype=torch.int32)
    rc = fec.encode_seal_groups_host_into(eng, k, m, bb, data, None, 0, bb, pkt, plen)
    assert rc == -1
    assert bool((pkt == 0xA5).all()) and bool((plen == 7).all())
    eng.close()
