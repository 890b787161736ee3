"""Test-side restatement of the reference's group framing (net/quic/core/quic_fec_group.cc)
over the CPU oracle codec.  TEST INFRASTRUCTURE: the checker for quic_amd.fec_group."""
import struct

import numpy as np


def prefix(payload, pnlen):
    """appendLenToPayload, quic_fec_group.cc:109-121 (16-bit truncation kept)."""
    ext = (len(payload) | (pnlen << 14)) & 0xFFFF
    return struct.pack("<H", ext) + bytes(payload)


def redundancy(oracle, k, m, group_min, sent):
    """getRedundancyPackets, :338-389.  sent = [(pn, payload, pnlen)] in send order.
    Returns ([(pn, data, pnlen)] in the reference's list order, rc)."""
    pre = [prefix(p, pl) for _, p, pl in sent]
    bb = max(len(x) for x in pre)
    bb += (-bb) % 8
    blocks = [np.frombuffer(x + b"\0" * (bb - len(x)), np.uint8) for x in pre]
    rec, rc = oracle.encode_ptrs(k, m, bb, blocks)
    out = []
    for i in range(m):
        e = m - i - 1
        out.append((group_min + k + e, rec[e].tobytes(), 1))
    return out, rc


def revive(oracle, k, m, group_min, received):
    """getRevivedPackets, :234-297.  received = [(pn, stored_bytes)] in arrival order,
    data packets already prefixed.  Returns ([(pn, payload, pnlen)], rc)."""
    got = {pn for pn, _ in received}
    if len(got) < k:
        return [], 0
    missing = [pn for pn in range(group_min, group_min + k) if pn not in got]
    if not missing:
        return [], 0
    bb = max(len(d) for _, d in received)
    first = received[:k]
    blocks = [np.frombuffer(d + b"\0" * (bb - len(d)), np.uint8) for _, d in first]
    rows = [(pn - group_min) & 0xFF for pn, _ in first]
    outb, outr, rc = oracle.decode_blocks(k, m, bb, blocks, rows)
    res = []
    for pn in missing:
        idx = [i for i, r in enumerate(outr) if r == ((pn - group_min) & 0xFF)]
        if not idx:
            break
        blk = outb[idx[0]].tobytes()
        (ln,) = struct.unpack("<H", blk[:2])
        pnl = ln >> 14
        ln &= 0x3FFF
        res.append((pn, blk[2:2 + min(ln, bb - 2)], pnl))
    return res, rc


def is_waiting_for_packet_before(group_min, received_set, num):
    """IsWaitingForPacketBefore, :300-325."""
    if group_min >= num:
        return False
    rs = sorted(received_set)
    if (rs[-1] + 1 < num) if rs else (group_min < num):
        return True
    target = group_min
    for pn in rs:
        if target != pn:
            return True
        target += 1
        if target >= num:
            return False
    return False


# ------------------------------------------------------------------ FEC wire format
# Restated from net/quic/core/quic_framer.cc; flag bits from quic_protocol.h:411-427.
# The reference's own tests hold no FEC framer vectors: parity of the
# wire format is pinned to this restatement only ("parity unpinned" against the reference).
FLAG_ENTROPY, FLAG_FEC_GROUP, FLAG_FEC, FLAG_FEC_CONFIG = 1, 2, 4, 0x1F << 3


def write_private(pn, fec_group, entropy, fec_flag, in_group, conf, version):
    """AppendPacketHeader, private part (quic_framer.cc:850-893); None where the
    reference DCHECKs (:873-874)."""
    flags = 0
    if entropy:
        flags |= FLAG_ENTROPY
    if in_group:
        flags |= FLAG_FEC_GROUP
        flags |= (conf << 3)
    if fec_flag:
        flags |= FLAG_FEC
    flags &= 0xFF                                   # uint8_t private_flags
    out = bytes([flags])
    if in_group:
        if not (fec_group <= pn and pn - fec_group < 255):
            return None
        out += bytes([(pn - fec_group) & 0xFF])
    if version <= 33:                               # :885-891
        out += bytes([flags])
    return out


def read_private(data, pn):
    """ProcessAuthenticatedHeader (quic_framer.cc:1219-1256): (fields, consumed) or an
    error string."""
    if len(data) < 1:
        return "Unable to read private flags."
    flags = data[0]
    f = {"packet_number": pn, "fec_group": 0, "entropy_flag": bool(flags & FLAG_ENTROPY),
         "fec_flag": bool(flags & FLAG_FEC), "in_fec_group": False, "fec_configuration": 0}
    if not flags & FLAG_FEC_GROUP:
        return f, 1
    if len(data) < 2:
        return "Unable to read first fec protected packet offset."
    off = data[1]
    if off >= pn:
        return "First fec protected packet offset must be less than the packet number."
    f.update(in_fec_group=True, fec_group=pn - off,
             fec_configuration=(flags & FLAG_FEC_CONFIG) >> 3)
    return f, 2


def header_size(cid_len, version, path_id, nonce, pnlen, in_group):
    """GetPacketHeaderSize (quic_protocol.cc:74-88), constants quic_protocol.h:150-160,263."""
    return (1 + cid_len + (4 if version else 0) + (1 if path_id else 0) + pnlen +
            (32 if nonce else 0) + (1 if in_group else 0) + 1)
