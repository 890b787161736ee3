"""Python mirror of QuicFecGroup (net/quic/core/quic_fec_group.h:36-109) over the C ABI
in include/quic_fec_group.h; the codec behind it is the GPU engine.

Packets are (packet_number, data: bytes, packet_number_len) tuples, the fields of the
reference's ParityPacket (quic_fec_group.h:26-34).
"""
import ctypes

from ._lib import FecError, load

FEC_OFF, FEC_5_5, FEC_10_10, FEC_10_15, FEC_10_20, FEC_15_15, FEC_250_5 = range(7)
ENCRYPTION_NONE, ENCRYPTION_INITIAL, ENCRYPTION_FORWARD_SECURE = 0, 1, 2
PACKET_1BYTE_PACKET_NUMBER, PACKET_2BYTE_PACKET_NUMBER = 1, 2
PACKET_4BYTE_PACKET_NUMBER, PACKET_6BYTE_PACKET_NUMBER = 4, 6

_c = ctypes
_u8p = _c.POINTER(_c.c_uint8)
_SIG = {
    "qfec_set_fec_overrides": (None, [_c.c_size_t, _c.c_size_t]),
    "qfec_k_from_conf": (_c.c_size_t, [_c.c_int]),
    "qfec_m_from_conf": (_c.c_size_t, [_c.c_int]),
    "qfec_prefix_payload": (_c.c_long, [_c.c_char_p, _c.c_size_t, _c.c_int, _c.c_void_p]),
    "qfec_block_bytes": (_c.c_int, [_c.c_size_t]),
    "qfec_group_new": (_c.c_void_p, [_c.c_ulonglong, _c.c_int]),
    "qfec_group_free": (None, [_c.c_void_p]),
    "qfec_group_new_with_codec": (_c.c_void_p, [_c.c_ulonglong, _c.c_int, _c.c_void_p,
                                                _c.c_void_p]),
    "qfec_group_update_sent": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_ulonglong, _c.c_int,
                                          _c.c_char_p, _c.c_size_t]),
    "qfec_group_update_received": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_ulonglong, _c.c_int,
                                              _c.c_char_p, _c.c_size_t, _c.c_int]),
    "qfec_group_update_fec": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_ulonglong, _c.c_int,
                                         _c.c_char_p, _c.c_size_t]),
    "qfec_group_can_revive": (_c.c_int, [_c.c_void_p]),
    "qfec_group_is_waiting_for_packet_before": (_c.c_int, [_c.c_void_p, _c.c_ulonglong]),
    "qfec_group_num_received": (_c.c_size_t, [_c.c_void_p]),
    "qfec_group_num_sent": (_c.c_size_t, [_c.c_void_p]),
    "qfec_group_effective_encryption_level": (_c.c_int, [_c.c_void_p]),
    "qfec_group_number": (_c.c_ulonglong, [_c.c_void_p]),
    "qfec_group_total_size": (_c.c_size_t, [_c.c_void_p]),
    "qfec_group_redundancy_size": (_c.c_size_t, [_c.c_void_p]),
    "qfec_group_redundancy": (_c.c_void_p, [_c.c_void_p, _c.POINTER(_c.c_int)]),
    "qfec_group_revived": (_c.c_void_p, [_c.c_void_p, _c.POINTER(_c.c_int)]),
    "qfec_packets_count": (_c.c_size_t, [_c.c_void_p]),
    "qfec_packets_get": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.POINTER(_c.c_ulonglong),
                                    _c.POINTER(_u8p), _c.POINTER(_c.c_size_t),
                                    _c.POINTER(_c.c_int)]),
    "qfec_packets_free": (None, [_c.c_void_p]),
    "qfec_batch_new": (_c.c_void_p, [_c.c_void_p, _c.c_size_t, _c.c_uint]),
    "qfec_batch_free": (None, [_c.c_void_p]),
    "qfec_batch_add_encode": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "qfec_batch_add_decode": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "qfec_batch_poll": (_c.c_int, [_c.c_void_p]),
    "qfec_batch_flush": (_c.c_int, [_c.c_void_p]),
    "qfec_batch_pending": (_c.c_size_t, [_c.c_void_p]),
    "qfec_wire_write_private": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_void_p, _c.c_size_t]),
    "qfec_wire_read_private": (_c.c_int, [_c.c_char_p, _c.c_size_t, _c.c_void_p]),
    "qfec_wire_header_size": (_c.c_size_t, [_c.c_int] * 6),
    "qfec_wire_fec_packet": (_c.c_long, [_c.c_char_p, _c.c_size_t, _c.c_char_p, _c.c_size_t,
                                         _c.c_void_p, _c.c_size_t]),
}
_lib = None


def lib():
    global _lib
    if _lib is None:
        L = load()
        for n, (res, args) in _SIG.items():
            f = getattr(L, n)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def set_fec_overrides(k=0, m=0):
    """kDefaultMaxPacketsPerFecGroup / kDefaultRecoveryBlocksCount (0 = presets)."""
    lib().qfec_set_fec_overrides(k, m)


def k_from_conf(conf):
    return lib().qfec_k_from_conf(conf)


def m_from_conf(conf):
    return lib().qfec_m_from_conf(conf)


def prefix_payload(payload, packet_number_len):
    out = _c.create_string_buffer(len(payload) + 2)
    n = lib().qfec_prefix_payload(bytes(payload), len(payload), packet_number_len, out)
    if n < 0:
        raise ValueError("payload longer than 0x3fff bytes")
    return out.raw[:n]


def block_bytes(max_prefixed_len):
    return lib().qfec_block_bytes(max_prefixed_len)


def _packets(handle):
    L = lib()
    out = []
    try:
        for i in range(L.qfec_packets_count(handle)):
            pn = _c.c_ulonglong()
            data = _u8p()
            n = _c.c_size_t()
            pl = _c.c_int()
            L.qfec_packets_get(handle, i, _c.byref(pn), _c.byref(data), _c.byref(n),
                               _c.byref(pl))
            out.append((pn.value, _c.string_at(data, n.value), pl.value))
    finally:
        L.qfec_packets_free(handle)
    return out


class QuicFecGroup:
    def __init__(self, fec_group_number, fec_configuration):
        self._L = lib()
        self._h = self._L.qfec_group_new(fec_group_number, fec_configuration)
        self.fec_configuration = fec_configuration

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._L.qfec_group_free(h)

    def UpdateSentList(self, encryption_level, packet_number, packet_number_len, payload):
        return bool(self._L.qfec_group_update_sent(self._h, encryption_level, packet_number,
                                                   packet_number_len, bytes(payload),
                                                   len(payload)))

    def UpdateReceivedList(self, encryption_level, packet_number, packet_number_len, payload,
                           is_fec_data):
        return bool(self._L.qfec_group_update_received(self._h, encryption_level, packet_number,
                                                       packet_number_len, bytes(payload),
                                                       len(payload), int(is_fec_data)))

    def UpdateFec(self, encryption_level, packet_number, packet_number_len, redundancy):
        return bool(self._L.qfec_group_update_fec(self._h, encryption_level, packet_number,
                                                  packet_number_len, bytes(redundancy),
                                                  len(redundancy)))

    def CanRevive(self):
        return bool(self._L.qfec_group_can_revive(self._h))

    def IsWaitingForPacketBefore(self, num):
        return bool(self._L.qfec_group_is_waiting_for_packet_before(self._h, num))

    def NumReceivedPackets(self):
        return self._L.qfec_group_num_received(self._h)

    def NumSentPackets(self):
        return self._L.qfec_group_num_sent(self._h)

    def EffectiveEncryptionLevel(self):
        return self._L.qfec_group_effective_encryption_level(self._h)

    def FecGroupNumber(self):
        return self._L.qfec_group_number(self._h)

    def GroupTotalSize(self):
        return self._L.qfec_group_total_size(self._h)

    def GroupReduntancySize(self):
        return self._L.qfec_group_redundancy_size(self._h)

    def getRedundancyPackets(self, check=True):
        st = _c.c_int()
        pk = _packets(self._L.qfec_group_redundancy(self._h, _c.byref(st)))
        if check and st.value < -1:
            raise FecError(st.value, "getRedundancyPackets")
        return pk if not check else pk, st.value

    def getRevivedPackets(self):
        st = _c.c_int()
        pk = _packets(self._L.qfec_group_revived(self._h, _c.byref(st)))
        return pk, st.value


class FecBatch:
    """Batching front end: one batched GPU launch for many queued groups."""

    def __init__(self, engine, max_groups=4096, max_delay_us=1000):
        self._L = lib()
        self._h = self._L.qfec_batch_new(engine._h, max_groups, max_delay_us)
        if not self._h:
            raise ValueError("bad batch parameters")
        self._keep = []

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._L.qfec_batch_free(h)

    def add_encode(self, group):
        self._keep.append(group)
        return self._L.qfec_batch_add_encode(self._h, group._h)

    def add_decode(self, group):
        self._keep.append(group)
        return self._L.qfec_batch_add_decode(self._h, group._h)

    def poll(self):
        return self._L.qfec_batch_poll(self._h)

    def flush(self):
        r = self._L.qfec_batch_flush(self._h)
        if self.pending() == 0:
            self._keep.clear()
        return r

    def pending(self):
        return self._L.qfec_batch_pending(self._h)


# ---------------------------------------------------------------- FEC wire format
class PrivateHeader(_c.Structure):
    """qfec_private_header: the FEC fields of a QuicPacketHeader (quic_protocol.h:850-860)."""
    _fields_ = [("packet_number", _c.c_ulonglong), ("fec_group", _c.c_ulonglong),
                ("entropy_flag", _c.c_int), ("fec_flag", _c.c_int),
                ("in_fec_group", _c.c_int), ("fec_configuration", _c.c_int)]


def write_private(packet_number, fec_group=0, entropy_flag=False, fec_flag=False,
                  in_fec_group=None, fec_configuration=FEC_OFF, quic_version=36):
    """Private flags byte (+ FEC group offset) as AppendPacketHeader writes it
    (quic_framer.cc:850-893).  in_fec_group defaults to fec_group != 0, as
    QuicPacketCreator::FillPacketHeader sets it (quic_packet_creator.cc:784-788)."""
    if in_fec_group is None:
        in_fec_group = fec_group != 0
    h = PrivateHeader(packet_number, fec_group, int(bool(entropy_flag)), int(bool(fec_flag)),
                      int(bool(in_fec_group)), fec_configuration)
    buf = (_c.c_uint8 * 4)()
    n = lib().qfec_wire_write_private(_c.byref(h), quic_version, buf, 4)
    if n < 0:
        raise ValueError(f"qfec_wire_write_private: {n}")
    return bytes(buf[:n])


def read_private(data, packet_number):
    """ProcessAuthenticatedHeader (quic_framer.cc:1219-1256): returns (fields dict, bytes
    consumed); raises ValueError with the reference's error text on a bad header."""
    h = PrivateHeader(packet_number, 0, 0, 0, 0, 0)
    n = lib().qfec_wire_read_private(bytes(data), len(data), _c.byref(h))
    if n < 0:
        raise ValueError({-1: "Unable to read private flags.",
                          -2: "Unable to read first fec protected packet offset.",
                          -3: "First fec protected packet offset must be less than the "
                              "packet number."}[n])
    return ({"packet_number": h.packet_number, "fec_group": h.fec_group,
             "entropy_flag": bool(h.entropy_flag), "fec_flag": bool(h.fec_flag),
             "in_fec_group": bool(h.in_fec_group),
             "fec_configuration": h.fec_configuration}, n)


def header_size(connection_id_length, include_version, include_path_id, include_nonce,
                packet_number_length, in_fec_group):
    """GetPacketHeaderSize (quic_protocol.cc:74-88)."""
    return lib().qfec_wire_header_size(connection_id_length, int(include_version),
                                       int(include_path_id), int(include_nonce),
                                       packet_number_length, int(in_fec_group))


def fec_packet(header, redundancy):
    """BuildFecPacket's body (quic_framer.cc:469-494): header bytes + parity block."""
    n = len(header) + len(redundancy)
    buf = (_c.c_uint8 * max(n, 1))()
    r = lib().qfec_wire_fec_packet(bytes(header), len(header), bytes(redundancy),
                                   len(redundancy), buf, n)
    if r < 0:
        raise ValueError(f"qfec_wire_fec_packet: {r}")
    return bytes(buf[:r])
