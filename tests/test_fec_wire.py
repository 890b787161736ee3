"""QuicR FEC wire format (include/quic_fec_group.h qfec_wire_*, quic_amd/csrc/fec_wire.cpp)
against the restatement of quic_framer.cc in tests/ref_framing.py.

CPU: the private-flags byte / FEC group offset writer and parser over every flag and
configuration combination and the edge offsets, their error returns, header sizes, FEC
packet assembly.  GPU: a whole group through the wire (sender QuicFecGroup -> FEC packets
with their private headers -> loss -> parse -> receiver QuicFecGroup -> revived payloads).
The reference holds no framer vectors for FEC, so this parity is against the restatement
only (parity unpinned against the reference itself)."""
import itertools
import random

import pytest

from quic_amd import fec_group as F
from tests import ref_framing as R


@pytest.mark.parametrize("version", [33, 34, 36])
def test_write_private_matches_restatement(version):
    rnd = random.Random(version)
    for entropy, fec_flag, in_group in itertools.product([0, 1], repeat=3):
        for conf in range(7):
            for pn, grp in [(1, 1), (300, 46), (300, 300), (2**40, 2**40 - 254), (10, 0),
                            (rnd.randrange(1, 2**48), None)]:
                if grp is None:
                    grp = pn - rnd.randrange(0, min(pn, 255))
                ref = R.write_private(pn, grp, entropy, fec_flag, in_group, conf, version)
                got = F.write_private(pn, grp, entropy, fec_flag, bool(in_group), conf, version)
                assert got == ref, (entropy, fec_flag, in_group, conf, pn, grp)


def test_write_private_rejects_like_the_dchecks():
    with pytest.raises(ValueError):
        F.write_private(100, fec_group=101, in_fec_group=True)        # group after packet
    with pytest.raises(ValueError):
        F.write_private(1000, fec_group=1000 - 255, in_fec_group=True)  # offset >= 255
    assert F.write_private(1000, fec_group=1000 - 254, in_fec_group=True)[1] == 254
    # not in a group: fec_group is not looked at
    assert F.write_private(5, fec_group=99, in_fec_group=False) == b"\x00"


def test_read_private_matches_restatement_exhaustively():
    for flags in range(256):
        for off in [0, 1, 7, 254, 255]:
            for pn in [1, 7, 8, 255, 256, 1000]:
                data = bytes([flags, off, 0xAB])
                ref = R.read_private(data, pn)
                try:
                    got = F.read_private(data, pn)
                except ValueError as e:
                    got = str(e)
                assert got == ref, (flags, off, pn)


def test_read_private_errors():
    with pytest.raises(ValueError, match="Unable to read private flags"):
        F.read_private(b"", 10)
    with pytest.raises(ValueError, match="offset"):
        F.read_private(bytes([R.FLAG_FEC_GROUP]), 10)
    with pytest.raises(ValueError, match="less than the packet number"):
        F.read_private(bytes([R.FLAG_FEC_GROUP, 10]), 10)


@pytest.mark.parametrize("version", [34, 36])
def test_round_trip_all_configurations(version):
    for conf in range(32):   # 5 bits on the wire
        for fec_flag in (False, True):
            b = F.write_private(1234, 1200, entropy_flag=True, fec_flag=fec_flag,
                                fec_configuration=conf, quic_version=version)
            f, n = F.read_private(b + b"payload", 1234)
            assert n == len(b) == 2
            assert f == {"packet_number": 1234, "fec_group": 1200, "entropy_flag": True,
                         "fec_flag": fec_flag, "in_fec_group": True, "fec_configuration": conf}


def test_header_size_matches_restatement():
    for cid, ver, path, nonce, pnlen, grp in itertools.product(
            [0, 8], [0, 1], [0, 1], [0, 1], [1, 2, 4, 6], [0, 1]):
        assert F.header_size(cid, ver, path, nonce, pnlen, grp) == \
            R.header_size(cid, ver, path, nonce, pnlen, grp)
    # GetStartOfFecProtectedData for an 8-byte connection id, 6-byte packet number
    assert F.header_size(8, False, False, False, 6, True) == 17


def test_fec_packet_is_header_then_redundancy():
    hdr = bytes(range(17))
    red = bytes((i * 13) & 0xFF for i in range(1352))
    pkt = F.fec_packet(hdr, red)
    assert pkt == hdr + red and len(pkt) == 17 + 1352
    assert F.fec_packet(b"", b"") == b""


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(10, 1), (32, 4), (5, 5)])
def test_group_through_the_wire(k, m):
    """Sender group -> data and FEC packets with their private headers (the public
    header reduced to the packet number, out of scope) -> seeded loss -> receiver parses
    each private header, routes FEC packets by fec_flag and their group by the offset ->
    revived payloads equal the lost ones."""
    F.set_fec_overrides(k, m)
    try:
        rnd = random.Random(k * 100 + m)
        base, conf = 4000, F.FEC_5_5
        sent = [(base + i, bytes(rnd.getrandbits(8) for _ in range(1350)), 2) for i in range(k)]
        s = F.QuicFecGroup(base, conf)
        for pn, p, pl in sent:
            s.UpdateSentList(2, pn, pl, p)
        par, st = s.getRedundancyPackets()
        assert st == 0 and len(par) == m
        wire = []
        for pn, p, pl in sent:
            wire.append((pn, F.write_private(pn, base, fec_configuration=conf) + p))
        for pn, red, pl in par:
            hdr = F.write_private(pn, base, fec_flag=True, fec_configuration=conf)
            wire.append((pn, F.fec_packet(hdr, red)))
        lost = set(rnd.sample(range(k), min(m, k)))
        r = F.QuicFecGroup(base, conf)
        for i, (pn, pkt) in enumerate(wire):
            if i in lost:
                continue
            f, n = F.read_private(pkt, pn)
            assert f["in_fec_group"] and f["fec_group"] == base
            assert f["fec_configuration"] == conf
            r.UpdateReceivedList(2, pn, 2, pkt[n:], f["fec_flag"])
        assert r.CanRevive()
        rev, rst = r.getRevivedPackets()
        assert rst == 0
        by_pn = {pn: p for pn, p, _ in sent}
        assert {pn for pn, _, _ in rev} == {sent[i][0] for i in lost}
        for pn, payload, _ in rev:
            assert payload == by_pn[pn]
    finally:
        F.set_fec_overrides(0, 0)
