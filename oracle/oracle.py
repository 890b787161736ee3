"""ctypes front-end for the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Loads oracle/liboracle_fec.so (the plain-C restatement in fec_oracle.c) and,
when present, oracle/_ref/libref_cauchy.so (the reference codec compiled from
/root/reference by oracle/Makefile).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use this module; the product path never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ORACLE_SO = os.path.join(HERE, "liboracle_fec.so")
REF_SO = os.path.join(HERE, "_ref", "libref_cauchy.so")
TABLES = os.path.join(ROOT, "quic_amd", "data", "cauchy_256_tables.bin")

_u8p = ctypes.POINTER(ctypes.c_uint8)


class OracleBlock(ctypes.Structure):
    _fields_ = [("data", _u8p), ("row", ctypes.c_uint8)]


_lib = None
_ref = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_init.argtypes = [ctypes.c_char_p]
        L.oracle_gf_mul.restype = ctypes.c_uint8
        L.oracle_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_gf_div.restype = ctypes.c_uint8
        L.oracle_gf_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_cauchy_matrix.argtypes = [ctypes.c_int, ctypes.c_int, _u8p]
        L.oracle_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_u8p),
                                    ctypes.c_void_p, ctypes.c_int]
        L.oracle_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(OracleBlock),
                                    ctypes.c_int]
        L.oracle_encode_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_longlong, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int]
        L.oracle_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_longlong, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_run_encode_batch.argtypes = [ctypes.c_void_p] + L.oracle_encode_batch.argtypes
        L.oracle_run_decode_batch.argtypes = [ctypes.c_void_p] + L.oracle_decode_batch.argtypes
        L.oracle_fill_stream.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_uint64]
        L.oracle_now.restype = ctypes.c_double
        rc = L.oracle_init(TABLES.encode())
        if rc != 0:
            raise RuntimeError(f"oracle_init({TABLES}) failed: {rc}")
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(REF_SO)


def ref():
    """The compiled reference codec (cauchy_256 ABI), or None if not built."""
    global _ref
    if _ref is None and ref_available():
        R = ctypes.CDLL(REF_SO)
        R._cauchy_256_init.argtypes = [ctypes.c_int]
        R.cauchy_256_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_u8p),
                                        ctypes.c_void_p, ctypes.c_int]
        R.cauchy_256_decode.argtypes = [ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(OracleBlock), ctypes.c_int]
        if R._cauchy_256_init(2) != 0:
            raise RuntimeError("reference _cauchy_256_init(2) failed")
        _ref = R
    return _ref


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gf_mul(x, y):
    return lib().oracle_gf_mul(x, y)


def gf_div(x, y):
    return lib().oracle_gf_div(x, y)


def cauchy_matrix(k, m):
    out = np.zeros((max(m - 1, 1), k), np.uint8)
    rc = lib().oracle_cauchy_matrix(k, m, out.ctypes.data_as(_u8p))
    if rc:
        raise ValueError(f"no Cauchy matrix for k={k} m={m}")
    return out


def encode_batch(k, m, bb, data, threads=1, use_ref=False):
    """data: uint8 [G][k][bb] -> (parity [G][m][bb], rc)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    G = data.shape[0]
    parity = np.zeros((G, m, bb), np.uint8)
    L = lib()
    if use_ref:
        fn = ctypes.cast(ref().cauchy_256_encode, ctypes.c_void_p)
        rc = L.oracle_run_encode_batch(fn, k, m, bb, G, _ptr(data), _ptr(parity), threads)
    else:
        rc = L.oracle_encode_batch(k, m, bb, G, _ptr(data), _ptr(parity), threads)
    return parity, rc


def decode_batch(k, m, bb, blocks, rows, threads=1, use_ref=False):
    """In-place semantics on copies: returns (blocks', rows', status[G])."""
    blocks = np.array(blocks, dtype=np.uint8, order="C", copy=True)
    rows = np.array(rows, dtype=np.uint8, order="C", copy=True)
    G = blocks.shape[0]
    status = np.zeros(G, np.int32)
    L = lib()
    if use_ref:
        fn = ctypes.cast(ref().cauchy_256_decode, ctypes.c_void_p)
        L.oracle_run_decode_batch(fn, k, m, bb, G, _ptr(blocks), _ptr(rows), _ptr(status),
                                  threads)
    else:
        L.oracle_decode_batch(k, m, bb, G, _ptr(blocks), _ptr(rows), _ptr(status), threads)
    return blocks, rows, status


def encode_into(k, m, bb, data, parity, threads=1, use_ref=False):
    """Encode data [G][k][bb] into the caller's parity [G][m][bb] (no copies; for timing)."""
    L = lib()
    G = data.shape[0]
    if use_ref:
        fn = ctypes.cast(ref().cauchy_256_encode, ctypes.c_void_p)
        return L.oracle_run_encode_batch(fn, k, m, bb, G, _ptr(data), _ptr(parity), threads)
    return L.oracle_encode_batch(k, m, bb, G, _ptr(data), _ptr(parity), threads)


def decode_inplace(k, m, bb, blocks, rows, status, threads=1, use_ref=False):
    """Decode the caller's blocks [G][k][bb] / rows [G][k] in place (no copies; for
    timing).  status: int32 [G]."""
    L = lib()
    G = blocks.shape[0]
    if use_ref:
        fn = ctypes.cast(ref().cauchy_256_decode, ctypes.c_void_p)
        L.oracle_run_decode_batch(fn, k, m, bb, G, _ptr(blocks), _ptr(rows), _ptr(status),
                                  threads)
    else:
        L.oracle_decode_batch(k, m, bb, G, _ptr(blocks), _ptr(rows), _ptr(status), threads)


def encode_ptrs(k, m, bb, blocks, use_ref=False):
    """Single-group call through the cauchy_256 ABI with a pointer array
    (blocks: list of k uint8 arrays of bb bytes).  Returns (recovery [m][bb], rc)."""
    arrs = [np.ascontiguousarray(b, dtype=np.uint8) for b in blocks]
    ptrs = (_u8p * max(len(arrs), 1))(*[a.ctypes.data_as(_u8p) for a in arrs])
    out = np.zeros((m, bb), np.uint8)
    f = ref().cauchy_256_encode if use_ref else lib().oracle_encode
    rc = f(k, m, ptrs, _ptr(out), bb)
    return out, rc


def decode_blocks(k, m, bb, blocks, rows, use_ref=False):
    """Single-group decode through the cauchy_256 ABI.  Returns (blocks', rows', rc)."""
    arrs = [np.array(b, dtype=np.uint8, copy=True) for b in blocks]
    blk = (OracleBlock * max(len(arrs), 1))()
    for i, a in enumerate(arrs):
        blk[i].data = a.ctypes.data_as(_u8p)
        blk[i].row = int(rows[i])
    f = ref().cauchy_256_decode if use_ref else lib().oracle_decode
    rc = f(k, m, blk, bb)
    return arrs, [blk[i].row for i in range(len(arrs))], rc


def now():
    return lib().oracle_now()
