"""QuicFecGroup counterpart (quic_amd.fec_group over include/quic_fec_group.h).

CPU: host-only logic (presets, overrides, prefix quirk, block_bytes, receive-set
bookkeeping).  GPU: full sender -> loss -> receiver flows and the batching front end,
checked against tests/ref_framing.py (the reference framing over the oracle codec)."""
import random

import numpy as np
import pytest

from quic_amd import fec_group as F
from tests import ref_framing as R


@pytest.fixture(autouse=True)
def _reset_overrides():
    F.set_fec_overrides(0, 0)
    yield
    F.set_fec_overrides(0, 0)


def test_presets_match_reference_tables():
    # quic_fec_group.cc:22-82
    assert [F.k_from_conf(c) for c in range(7)] == [0, 5, 10, 10, 10, 15, 250]
    assert [F.m_from_conf(c) for c in range(7)] == [0, 5, 10, 15, 20, 15, 5]
    F.set_fec_overrides(32, 4)
    assert F.k_from_conf(F.FEC_5_5) == 32 and F.m_from_conf(F.FEC_5_5) == 4
    g = F.QuicFecGroup(1000, F.FEC_10_20)
    assert g.GroupTotalSize() == 36 and g.GroupReduntancySize() == 4


@pytest.mark.parametrize("pnlen", [1, 2, 4, 6])
@pytest.mark.parametrize("n", [0, 1, 1350, 0x3FFF])
def test_prefix_quirk(pnlen, n):
    payload = bytes((i * 7) & 0xFF for i in range(n))
    assert F.prefix_payload(payload, pnlen) == R.prefix(payload, pnlen)
    # 4-byte packet numbers read back as 0, 6-byte as 2 (Appendix A, item 2)
    hdr = int.from_bytes(F.prefix_payload(payload, pnlen)[:2], "little")
    assert hdr >> 14 == {1: 1, 2: 2, 4: 0, 6: 2}[pnlen]
    assert hdr & 0x3FFF == n


def test_prefix_rejects_oversize():
    with pytest.raises(ValueError):
        F.prefix_payload(b"\0" * 0x4000, 1)


def test_block_bytes_rounding():
    assert F.block_bytes(1352) == 1352 and F.block_bytes(1350) == 1352
    assert F.block_bytes(9002) == 9008 and F.block_bytes(1) == 8


def test_receive_bookkeeping():
    g = F.QuicFecGroup(100, F.FEC_5_5)
    assert not g.CanRevive()
    assert g.UpdateReceivedList(2, 100, 1, b"a", False)
    assert not g.UpdateReceivedList(2, 100, 1, b"a", False)      # duplicate
    assert not g.UpdateReceivedList(2, 99, 1, b"a", False)       # before the group
    assert g.UpdateFec(1, 106, 1, b"x" * 8)
    assert g.EffectiveEncryptionLevel() == 1
    for pn in (101, 103):
        g.UpdateReceivedList(2, pn, 1, b"b", False)
    assert g.NumReceivedPackets() == 4 and not g.CanRevive()
    g.UpdateReceivedList(2, 104, 1, b"c", False)
    assert g.CanRevive()


def test_is_waiting_for_packet_before():
    rnd = random.Random(5)
    for _ in range(200):
        base = rnd.randrange(1, 50)
        g = F.QuicFecGroup(base, F.FEC_10_10)
        got = set()
        for pn in rnd.sample(range(base, base + 20), rnd.randrange(0, 12)):
            g.UpdateReceivedList(2, pn, 1, b"p", False)
            got.add(pn)
        for num in range(base - 2, base + 25):
            assert g.IsWaitingForPacketBefore(num) == R.is_waiting_for_packet_before(base, got, num)


# ---------------------------------------------------------------------------- GPU
def make_group(rnd, k, m, base, lens=None):
    sent = []
    for i in range(k):
        n = lens[i] if lens else rnd.choice([1350, 1350, 1350, rnd.randrange(1, 1351)])
        sent.append((base + i, bytes(rnd.getrandbits(8) for _ in range(n)),
                     rnd.choice([1, 2, 4, 6])))
    return sent


@pytest.mark.gpu
@pytest.mark.parametrize("conf,ov", [(F.FEC_5_5, None), (F.FEC_10_10, None), (F.FEC_10_20, None),
                                     (F.FEC_15_15, None), (None, (10, 1)), (None, (32, 4))])
def test_group_round_trip_vs_reference(oracle, conf, ov):
    rnd = random.Random(hash((conf, ov)) & 0xFFFF)
    if ov:
        F.set_fec_overrides(*ov)
        conf = F.FEC_5_5
    k, m = F.k_from_conf(conf), F.m_from_conf(conf)
    for trial in range(6):
        base = 1000 + 100 * trial
        sent = make_group(rnd, k, m, base)
        s = F.QuicFecGroup(base, conf)
        for pn, p, pl in sent:
            s.UpdateSentList(2, pn, pl, p)
        par, st = s.getRedundancyPackets()
        ref_par, ref_rc = R.redundancy(oracle, k, m, base, sent)
        assert st == ref_rc == 0
        assert par == ref_par
        # receiver: lose up to m packets (data or parity), shuffled arrival, a duplicate
        wire = [(pn, p, pl, False) for pn, p, pl in sent] + [(pn, d, pl, True) for pn, d, pl in par]
        lost = set(rnd.sample(range(len(wire)), rnd.randrange(0, m + 1)))
        arrived = [w for i, w in enumerate(wire) if i not in lost]
        rnd.shuffle(arrived)
        if arrived:
            arrived.append(arrived[0])
        r = F.QuicFecGroup(base, conf)
        stored = []
        for pn, p, pl, is_fec in arrived:
            if r.UpdateReceivedList(2, pn, pl, p, is_fec):
                stored.append((pn, p if is_fec else R.prefix(p, pl)))
        rev, rst = r.getRevivedPackets()
        ref_rev, ref_rst = R.revive(oracle, k, m, base, stored)
        assert (rev, rst) == (ref_rev, ref_rst)
        lost_data = {wire[i][0] for i in lost if wire[i][0] < base + k}
        if r.CanRevive():
            assert {pn for pn, _, _ in rev} == lost_data
            by_pn = {pn: (p, pl) for pn, p, pl in sent}
            for pn, payload, pl in rev:
                assert payload == by_pn[pn][0]
                assert pl == {1: 1, 2: 2, 4: 0, 6: 2}[by_pn[pn][1]]
        # a second call returns nothing (missing packets were marked received, :249)
        assert r.getRevivedPackets()[0] == []


@pytest.mark.gpu
def test_batch_front_end_matches_per_group(engine, oracle):
    F.set_fec_overrides(32, 4)
    k, m = 32, 4
    rnd = random.Random(9)
    groups, sends = [], []
    batch = F.FecBatch(engine, max_groups=1000, max_delay_us=10**9)
    for gi in range(40):
        base = 10000 + gi * 64
        sent = make_group(rnd, k, m, base, lens=[1350] * k if gi % 2 else None)
        s = F.QuicFecGroup(base, F.FEC_5_5)
        for pn, p, pl in sent:
            s.UpdateSentList(2, pn, pl, p)
        assert batch.add_encode(s) == 0
        groups.append(s)
        sends.append(sent)
    assert batch.pending() == 40
    assert batch.flush() == 40 and batch.pending() == 0
    receivers = []
    for gi, (s, sent) in enumerate(zip(groups, sends)):
        base = 10000 + gi * 64
        par, st = s.getRedundancyPackets()
        assert st == 0
        assert par == R.redundancy(oracle, k, m, base, sent)[0]
        r = F.QuicFecGroup(base, F.FEC_5_5)
        drop = set(rnd.sample(range(k), 2))
        for i, (pn, p, pl) in enumerate(sent):
            if i not in drop:
                r.UpdateReceivedList(2, pn, pl, p, False)
        for pn, d, pl in par:
            r.UpdateFec(2, pn, pl, d)
        assert r.CanRevive()
        assert batch.add_decode(r) == 0
        receivers.append((r, sent, drop))
    assert batch.flush() == 40
    for r, sent, drop in receivers:
        rev, st = r.getRevivedPackets()
        assert st == 0
        assert sorted(pn for pn, _, _ in rev) == sorted(sent[i][0] for i in drop)
        for pn, payload, _ in rev:
            assert payload == sent[pn - sent[0][0]][1]


@pytest.mark.gpu
def test_batch_flushes_on_count_and_timeout(engine):
    F.set_fec_overrides(10, 1)
    rnd = random.Random(3)
    batch = F.FecBatch(engine, max_groups=4, max_delay_us=0)
    gs = []
    for gi in range(4):
        s = F.QuicFecGroup(gi * 20, F.FEC_5_5)
        for pn, p, pl in make_group(rnd, 10, 1, gi * 20, lens=[1350] * 10):
            s.UpdateSentList(2, pn, pl, p)
        r = batch.add_encode(s)
        gs.append(s)
        assert r == (4 if gi == 3 else 0)      # the 4th add fills the bucket
    assert batch.pending() == 0
    s = F.QuicFecGroup(500, F.FEC_5_5)
    for pn, p, pl in make_group(rnd, 10, 1, 500, lens=[1350] * 10):
        s.UpdateSentList(2, pn, pl, p)
    batch.add_encode(s)
    assert batch.poll() == 1 and batch.pending() == 0   # timeout 0 -> flushed on poll
    for g in gs + [s]:
        assert g.getRedundancyPackets()[1] == 0


# ------------------------------------------ the C++ class with the reference's method names
def test_cxx_class_header_compiles():
    """include/quic_fec_group.hpp (qfec::QuicFecGroup, the reference's method names over the
    C ABI) compiles with plain g++ against the public headers only."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "tools", "group_cxx", "group_roundtrip.cpp")
    p = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only",
                        "-I" + os.path.join(root, "include"), src],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("conf,losses", [(F.FEC_5_5, 5), (F.FEC_10_10, 4), (F.FEC_10_20, 10),
                                         (F.FEC_15_15, 7), (F.FEC_250_5, 5), (F.FEC_10_15, 1)])
def test_cxx_class_round_trip(conf, losses):
    """qfec::QuicFecGroup used like the reference's creator / connection: UpdateSentList x k,
    getRedundancyPackets, then a receiver with `losses` data packets dropped takes parity
    packets until CanRevive() and getRevivedPackets() returns each lost packet intact
    (tools/group_cxx/group_roundtrip.cpp, codec on the GPU)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = os.path.join(root, "quic_amd", "bin", "group_roundtrip")
    if not os.path.exists(tool):
        subprocess.run(["make", "-C", root, "tools"], check=True, capture_output=True)
    for seed in (1, 2):
        p = subprocess.run([tool, str(conf), str(losses), str(seed)], capture_output=True,
                           text=True, timeout=120, cwd=root)
        assert p.returncode == 0, p.stderr
        assert p.stdout.split() == ["ok", str(losses)]
