"""Python front-end of the MI355X FEC engine (ctypes over libquic_fec.so).

Mirrors the reference codec interface (net/quic/core/libcat/cauchy_256.h):
`cauchy_256_init`, `cauchy_256_encode`, `cauchy_256_decode`, `Block`, with the same
argument meaning, return codes and in-place decode semantics, plus the batched
engine (`FecEngine`) that the GPU path is built for.  Every byte of parity or
recovered data is computed by the gfx950 kernels; nothing here computes on the CPU.

Device buffers are torch tensors (uint8, contiguous, on a ROCm device): torch is
used only for memory and streams.
"""
import ctypes

import numpy as np

from ._lib import Block, FecError, load

CAUCHY_256_VERSION = 2
_u8p = ctypes.POINTER(ctypes.c_uint8)


# ----------------------------------------------------------------- reference ABI
def _cauchy_256_init(expected_version):
    """cauchy_256.h:47.  0 on success, -1 on a version mismatch (what the reference
    code returns), negative on GPU bring-up failure."""
    return load()._cauchy_256_init(expected_version)


def cauchy_256_init():
    return _cauchy_256_init(CAUCHY_256_VERSION)


def _as_u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(_u8p)


def cauchy_256_encode(k, m, data_ptrs, recovery_blocks, block_bytes):
    """cauchy_256.h:78.  data_ptrs: sequence of k uint8 arrays (block_bytes each);
    recovery_blocks: writable uint8 array of m*block_bytes bytes (filled in place).
    Returns the reference's return code."""
    keep = [_as_u8(d) for d in data_ptrs]
    arr = (_u8p * max(len(keep), 1))(*[p for _, p in keep])
    if not (isinstance(recovery_blocks, np.ndarray) and recovery_blocks.dtype == np.uint8
            and recovery_blocks.flags.c_contiguous):
        raise TypeError("recovery_blocks must be a C-contiguous uint8 numpy array")
    return load().cauchy_256_encode(k, m, arr, recovery_blocks.ctypes.data_as(ctypes.c_void_p),
                                    block_bytes)


def make_blocks(arrays, rows):
    """Build a `Block[]` over caller-owned uint8 arrays (decoded in place)."""
    blocks = (Block * max(len(arrays), 1))()
    for i, (a, r) in enumerate(zip(arrays, rows)):
        if not (isinstance(a, np.ndarray) and a.dtype == np.uint8 and a.flags.c_contiguous):
            raise TypeError("blocks must be C-contiguous uint8 numpy arrays")
        blocks[i].data = a.ctypes.data_as(_u8p)
        blocks[i].row = int(r)
    return blocks


def cauchy_256_decode(k, m, blocks, block_bytes):
    """cauchy_256.h:103.  `blocks` is a Block array from make_blocks(); data and row
    fields are updated in place.  Returns the reference's return code."""
    return load().cauchy_256_decode(k, m, blocks, block_bytes)


def cauchy_matrix(k, m):
    """Rows 1..m-1 of the Cauchy matrix the reference uses, (m-1) x k."""
    out = np.zeros((m - 1, k), np.uint8)
    rc = load().qfec_cauchy_matrix(k, m, out.ctypes.data_as(ctypes.c_void_p))
    if rc:
        raise ValueError(f"no Cauchy matrix for k={k} m={m}")
    return out


# ------------------------------------------------------------------ batch engine
def _dptr(t):
    if t is None:
        return None
    import torch
    if not isinstance(t, torch.Tensor):
        raise TypeError("device buffers must be torch tensors")
    if not t.is_cuda or t.dtype not in (torch.uint8, torch.int8, torch.int16, torch.int32):
        raise TypeError("device buffers must be integer tensors on a ROCm device")
    if not t.is_contiguous():
        raise ValueError("device buffers must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream, like):
    if stream is not None:
        return ctypes.c_void_p(int(stream))
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(like.device).cuda_stream)


class FecEngine:
    """One per GPU: owns a qfec_ctx (coefficient tables, decode workspace, staging)."""

    def __init__(self, device=0):
        self.lib = load()
        self.device = device
        h = ctypes.c_void_p()
        rc = self.lib.qfec_ctx_create(device, ctypes.byref(h))
        if rc:
            raise FecError(rc, "qfec_ctx_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self.lib.qfec_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name, value):
        """Launch-shape option of this engine's context (qfec_ctx_set_option)."""
        rc = self.lib.qfec_ctx_set_option(self._h, name.encode(), int(value))
        if rc:
            raise FecError(rc, f"qfec_ctx_set_option({name})")

    def get_option(self, name):
        v = ctypes.c_int()
        rc = self.lib.qfec_ctx_get_option(self._h, name.encode(), ctypes.byref(v))
        if rc:
            raise FecError(rc, f"qfec_ctx_get_option({name})")
        return v.value

    def reserve(self, k, m, block_bytes, groups):
        rc = self.lib.qfec_reserve(self._h, k, m, block_bytes, groups)
        if rc:
            raise FecError(rc, "qfec_reserve")

    # device-resident batch calls (enqueue only)
    def encode(self, k, m, block_bytes, data, parity, stream=None):
        """data [G][k][bb] -> parity [G][m][bb] (torch uint8 on the device).  Returns
        0 or -1 (the reference's unsupported-parameter code)."""
        G = data.shape[0]
        rc = self.lib.qfec_encode_batch(self._h, k, m, block_bytes, G, _dptr(data),
                                        _dptr(parity), _stream(stream, data))
        if rc < -1:
            raise FecError(rc, "qfec_encode_batch")
        return rc

    def decode(self, k, m, block_bytes, blocks, rows_in, out=None, rows_out=None, status=None,
               stream=None):
        """blocks [G][k][bb], rows_in [G][k] uint8.  out defaults to blocks (in place),
        rows_out to rows_in.  status: optional int32 [G]."""
        G = blocks.shape[0]
        out = blocks if out is None else out
        rows_out = rows_in if rows_out is None else rows_out
        rc = self.lib.qfec_decode_batch(self._h, k, m, block_bytes, G, _dptr(blocks),
                                        _dptr(rows_in), _dptr(out), _dptr(rows_out),
                                        _dptr(status), _stream(stream, blocks))
        if rc:
            raise FecError(rc, "qfec_decode_batch")
        return rc

    def decode_recovered(self, k, m, block_bytes, blocks, rows_in, rec, rec_rows, status=None,
                         stream=None):
        """Recovered-blocks layout: rec [G][min(k,m)][bb], rec_rows [G][min(k,m)] uint8
        (data row of each recovered block, ascending; 255 = unused).  blocks / rows_in are
        not modified."""
        G = blocks.shape[0]
        rc = self.lib.qfec_decode_batch_recovered(self._h, k, m, block_bytes, G, _dptr(blocks),
                                                  _dptr(rows_in), _dptr(rec), _dptr(rec_rows),
                                                  _dptr(status), _stream(stream, blocks))
        if rc:
            raise FecError(rc, "qfec_decode_batch_recovered")
        return rc

    # packet protection next to the codec (NullEncrypter / NullDecrypter, pp_null.hip)
    @staticmethod
    def _lens(lens):
        """(array pointer, scalar) for a per-packet length argument: an int32 device
        tensor, or an int meaning the same length for every packet."""
        if isinstance(lens, int):
            return None, lens
        return _dptr(lens), 0

    def null_seal(self, ad, ad_len, pt, pt_len, out, out_len, stream=None):
        """NullEncrypter::EncryptPacket over n packets: ad [n][ad_stride], pt [n][pt_stride]
        -> out [n][out_stride] = AD || tag12 || PT; out_len int32 [n] (-1: does not fit).
        ad_len / pt_len: int32 [n] tensors or ints (null_encrypter.cc:23-43)."""
        n = out.shape[0]
        a, a_all = self._lens(ad_len)
        p, p_all = self._lens(pt_len)
        rc = self.lib.qfec_null_seal_batch(self._h, n, _dptr(ad), ad.stride(0) if n else 0, a,
                                           a_all, _dptr(pt), pt.stride(0) if n else 0, p, p_all,
                                           _dptr(out), out.stride(0), _dptr(out_len),
                                           _stream(stream, out))
        if rc:
            raise FecError(rc, "qfec_null_seal_batch")

    def null_open(self, pkt, pkt_len, ad_len, out, out_len, stream=None):
        """NullDecrypter::DecryptPacket over n wire packets pkt [n][pkt_stride] (first ad_len
        bytes = associated data) -> plaintext in out [n][out_stride], out_len int32 [n]
        (-1: rejected)."""
        n = pkt.shape[0]
        p, p_all = self._lens(pkt_len)
        a, a_all = self._lens(ad_len)
        rc = self.lib.qfec_null_open_batch(self._h, n, _dptr(pkt), pkt.stride(0), p, p_all, a,
                                           a_all, _dptr(out), out.stride(0), _dptr(out_len),
                                           _stream(stream, pkt))
        if rc:
            raise FecError(rc, "qfec_null_open_batch")

    def encode_seal(self, k, m, block_bytes, data, parity, hdr, hdr_len, pkt, pkt_len,
                    stream=None):
        """SerializeFec on the device: encode data [G][k][bb] into parity [G][m][bb], then
        seal FEC packet g*m+i = hdr[g*m+i][:hdr_len] || tag12 || parity[g][i] into
        pkt [G*m][pkt_stride]; pkt_len int32 [G*m]."""
        G = data.shape[0]
        h, h_all = self._lens(hdr_len)
        rc = self.lib.qfec_encode_seal_batch(self._h, k, m, block_bytes, G, _dptr(data),
                                             _dptr(parity), _dptr(hdr), hdr.stride(0), h, h_all,
                                             _dptr(pkt), pkt.stride(0), _dptr(pkt_len),
                                             _stream(stream, data))
        if rc:
            raise FecError(rc, "qfec_encode_seal_batch")

    def seal_groups(self, k, m, block_bytes, data, parity, hdr, hdr_len, pt_len, pkt, pkt_len,
                    encode=False, stream=None):
        """Seal every packet of each group in one launch: packet p = g*(k+m)+i =
        hdr[p][:hdr_len] || tag12 || (data[g][i] if i < k else parity[g][i-k])[:pt_len] into
        pkt [G*(k+m)][pkt_stride]; pkt_len int32 [G*(k+m)].  encode=True first encodes data
        into parity (qfec_encode_seal_groups_batch)."""
        G = data.shape[0]
        h, h_all = self._lens(hdr_len)
        p, p_all = self._lens(pt_len)
        fn = self.lib.qfec_encode_seal_groups_batch if encode else self.lib.qfec_seal_groups_batch
        rc = fn(self._h, k, m, block_bytes, G, _dptr(data), _dptr(parity), _dptr(hdr),
                hdr.stride(0), h, h_all, p, p_all, _dptr(pkt), pkt.stride(0), _dptr(pkt_len),
                _stream(stream, data))
        if rc:
            raise FecError(rc, "qfec_encode_seal_groups_batch" if encode else "qfec_seal_groups_batch")

    def open_decode(self, k, m, block_bytes, pkt, pkt_len, ad_len, blocks, rows, open_len, rec,
                    rec_rows, status=None, stream=None):
        """Receiver: open every wire packet pkt [G*(k+m)][stride] (pkt_len int32, < 0 = not
        received), place the plaintexts into blocks [G][k][bb] / rows [G][k], then the
        recovered-layout decode into rec / rec_rows / status.  open_len int32 [G*(k+m)]."""
        G = blocks.shape[0]
        a, a_all = self._lens(ad_len)
        rc = self.lib.qfec_open_decode_batch(self._h, k, m, block_bytes, G, _dptr(pkt),
                                             pkt.stride(0), _dptr(pkt_len), a, a_all,
                                             _dptr(blocks), _dptr(rows), _dptr(open_len),
                                             _dptr(rec), _dptr(rec_rows), _dptr(status),
                                             _stream(stream, pkt))
        if rc:
            raise FecError(rc, "qfec_open_decode_batch")

    # host-pointer batch calls (synchronous; include H2D/D2H)
    def encode_host(self, k, m, block_bytes, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        G = data.shape[0]
        parity = np.zeros((G, m, block_bytes), np.uint8)
        rc = self.lib.qfec_encode_batch_host(self._h, k, m, block_bytes, G,
                                             data.ctypes.data_as(ctypes.c_void_p),
                                             parity.ctypes.data_as(ctypes.c_void_p))
        if rc < -1:
            raise FecError(rc, "qfec_encode_batch_host")
        return parity, rc

    def decode_host(self, k, m, block_bytes, blocks, rows):
        blocks = np.array(blocks, dtype=np.uint8, order="C", copy=True)
        rows = np.array(rows, dtype=np.uint8, order="C", copy=True)
        G = blocks.shape[0]
        status = np.zeros(G, np.int32)
        rc = self.lib.qfec_decode_batch_host(self._h, k, m, block_bytes, G,
                                             blocks.ctypes.data_as(ctypes.c_void_p),
                                             rows.ctypes.data_as(ctypes.c_void_p),
                                             status.ctypes.data_as(ctypes.c_void_p))
        if rc:
            raise FecError(rc, "qfec_decode_batch_host")
        return blocks, rows, status


def last_kernels():
    """Kernels the calling thread's last engine call launched (qfec_last_kernels)."""
    v = load().qfec_last_kernels()
    return v.decode() if v else ""


def last_grids():
    """{kernel: workgroups} of the persistent kernels the calling thread's last engine call
    launched (qfec_last_grids)."""
    v = load().qfec_last_grids()
    out = {}
    for item in (v.decode() if v else "").split():
        name, _, grid = item.partition("=")
        out[name] = int(grid)
    return out


def _hptr(t):
    import torch
    if not isinstance(t, torch.Tensor) or t.is_cuda or not t.is_contiguous():
        raise TypeError("host buffers must be contiguous CPU tensors (pinned for full speed)")
    return ctypes.c_void_p(t.data_ptr())


def _hcheck(t, name, dtype, shape):
    """A host buffer argument: a contiguous CPU tensor of `dtype` and exactly `shape` (None in
    `shape`: any extent, > 0).  The library copies whole rows into and out of it, so a short
    buffer would be overrun and a wrong dtype misread: ValueError / TypeError instead."""
    import torch
    if not isinstance(t, torch.Tensor) or t.is_cuda or not t.is_contiguous():
        raise TypeError(f"{name}: host buffers must be contiguous CPU tensors "
                        "(pinned for full speed)")
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if t.dim() != len(shape) or any(want is not None and got != want
                                    for got, want in zip(t.shape, shape)) \
            or any(got <= 0 for got, want in zip(t.shape, shape) if want is None):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")


def _hcheck_lens(lens, name, n):
    """A per-packet length argument: an int (the same for every packet) or int32 [n]."""
    import torch
    if not isinstance(lens, int):
        _hcheck(lens, name, torch.int32, (n,))


def encode_host_into(engine, k, m, block_bytes, data_h, parity_h):
    """Host-pointer encode on caller-owned CPU tensors (pinned memory recommended):
    H2D, kernels and D2H pipelined in chunks inside the library.  Returns 0 / -1."""
    import torch
    G = data_h.shape[0]
    _hcheck(data_h, "data", torch.uint8, (G, k, block_bytes))
    _hcheck(parity_h, "parity", torch.uint8, (G, m, block_bytes))
    rc = engine.lib.qfec_encode_batch_host(engine._h, k, m, block_bytes, data_h.shape[0],
                                           _hptr(data_h), _hptr(parity_h))
    if rc < -1:
        raise FecError(rc, "qfec_encode_batch_host")
    return rc


def decode_host_into(engine, k, m, block_bytes, blocks_h, rows_h, status_h=None):
    """Host-pointer in-place decode on caller-owned CPU tensors (cauchy_256_decode
    semantics per group)."""
    import torch
    G = blocks_h.shape[0]
    _hcheck(blocks_h, "blocks", torch.uint8, (G, k, block_bytes))
    _hcheck(rows_h, "rows", torch.uint8, (G, k))
    if status_h is not None:
        _hcheck(status_h, "status", torch.int32, (G,))
    rc = engine.lib.qfec_decode_batch_host(engine._h, k, m, block_bytes, blocks_h.shape[0],
                                           _hptr(blocks_h), _hptr(rows_h),
                                           None if status_h is None else _hptr(status_h))
    if rc:
        raise FecError(rc, "qfec_decode_batch_host")
    return rc


def _hlens(lens):
    """(host array pointer, scalar) for a per-packet length argument of a host call: an int32
    CPU tensor, or an int meaning the same length for every packet."""
    if isinstance(lens, int):
        return None, lens
    return _hptr(lens), 0


def encode_seal_groups_host_into(engine, k, m, block_bytes, data_h, hdr_h, hdr_len, pt_len,
                                 pkt_h, pkt_len_h):
    """Sender, host to host (qfec_encode_seal_groups_batch_host): data [G][k][bb] and
    headers hdr [G*(k+m)][hdr_stride] (or None) -> every packet sealed into pkt
    [G*(k+m)][pkt_stride], pkt_len int32 [G*(k+m)].  Returns 0 / -1."""
    import torch
    G = data_h.shape[0]
    n = G * (k + m)
    _hcheck(data_h, "data", torch.uint8, (G, k, block_bytes))
    if hdr_h is not None:
        _hcheck(hdr_h, "hdr", torch.uint8, (n, None))
    _hcheck_lens(hdr_len, "hdr_len", n)
    _hcheck_lens(pt_len, "pt_len", n)
    _hcheck(pkt_h, "pkt", torch.uint8, (n, None))
    _hcheck(pkt_len_h, "pkt_len", torch.int32, (n,))
    h, h_all = _hlens(hdr_len)
    p, p_all = _hlens(pt_len)
    rc = engine.lib.qfec_encode_seal_groups_batch_host(
        engine._h, k, m, block_bytes, data_h.shape[0], _hptr(data_h),
        None if hdr_h is None else _hptr(hdr_h), 0 if hdr_h is None else hdr_h.stride(0), h,
        h_all, p, p_all, _hptr(pkt_h), pkt_h.stride(0), _hptr(pkt_len_h))
    if rc < -1:
        raise FecError(rc, "qfec_encode_seal_groups_batch_host")
    return rc


def open_decode_host_into(engine, k, m, block_bytes, pkt_h, pkt_len_h, ad_len, rec_h,
                          rec_rows_h, status_h=None, open_len_h=None):
    """Receiver, host to host (qfec_open_decode_batch_host): wire packets pkt
    [G*(k+m)][stride], pkt_len int32 (< 0: not received) -> rec [G][min(k,m)][bb],
    rec_rows, status [G], open_len [G*(k+m)]."""
    import torch
    G = rec_h.shape[0]
    n, rmax = G * (k + m), min(k, m)
    _hcheck(pkt_h, "pkt", torch.uint8, (n, None))
    _hcheck(pkt_len_h, "pkt_len", torch.int32, (n,))
    _hcheck_lens(ad_len, "ad_len", n)
    _hcheck(rec_h, "rec", torch.uint8, (G, rmax, block_bytes))
    _hcheck(rec_rows_h, "rec_rows", torch.uint8, (G, rmax))
    if status_h is not None:
        _hcheck(status_h, "status", torch.int32, (G,))
    if open_len_h is not None:
        _hcheck(open_len_h, "open_len", torch.int32, (n,))
    a, a_all = _hlens(ad_len)
    rc = engine.lib.qfec_open_decode_batch_host(
        engine._h, k, m, block_bytes, rec_h.shape[0], _hptr(pkt_h), pkt_h.stride(0),
        _hptr(pkt_len_h), a, a_all, _hptr(rec_h), _hptr(rec_rows_h),
        None if status_h is None else _hptr(status_h),
        None if open_len_h is None else _hptr(open_len_h))
    if rc:
        raise FecError(rc, "qfec_open_decode_batch_host")
    return rc


def decode_recovered_host_into(engine, k, m, block_bytes, blocks_h, rows_h, rec_h, rec_rows_h,
                               status_h=None):
    """Host-pointer decode returning only the recovered blocks (CPU tensors)."""
    import torch
    G, rmax = blocks_h.shape[0], min(k, m)
    _hcheck(blocks_h, "blocks", torch.uint8, (G, k, block_bytes))
    _hcheck(rows_h, "rows", torch.uint8, (G, k))
    _hcheck(rec_h, "rec", torch.uint8, (G, rmax, block_bytes))
    _hcheck(rec_rows_h, "rec_rows", torch.uint8, (G, rmax))
    if status_h is not None:
        _hcheck(status_h, "status", torch.int32, (G,))
    rc = engine.lib.qfec_decode_batch_recovered_host(
        engine._h, k, m, block_bytes, blocks_h.shape[0], _hptr(blocks_h), _hptr(rows_h),
        _hptr(rec_h), _hptr(rec_rows_h), None if status_h is None else _hptr(status_h))
    if rc:
        raise FecError(rc, "qfec_decode_batch_recovered_host")
    return rc


def synth_fill(t, seed, byte_offset=0, stream=None):
    """Fill a device tensor with the seeded splitmix64 stream (quic_amd.synth)."""
    rc = load().qfec_synth_fill(_dptr(t), t.numel() * t.element_size(), seed, byte_offset,
                                _stream(stream, t))
    if rc:
        raise FecError(rc, "qfec_synth_fill")


def synth_gather(data, parity, src, blocks, k, m, block_bytes, stream=None):
    """blocks[g][i] = sent block src[g][i] of group g (device-side receive-set build)."""
    rc = load().qfec_synth_gather(_dptr(data), _dptr(parity), _dptr(src), _dptr(blocks), k, m,
                                  block_bytes, data.shape[0], _stream(stream, data))
    if rc:
        raise FecError(rc, "qfec_synth_gather")
