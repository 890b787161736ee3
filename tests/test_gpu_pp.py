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


def test_known_answer_through_gpu(engine):
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
def test_seal_open_random_vs_oracle(engine, oracle, n, S, AS):
    import torch
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
