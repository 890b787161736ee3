"""Loader for libquic_fec.so (the HIP extension).  Fails loudly when it is missing.

The product path has no CPU fallback: if the shared library was not built (run
`make lib` or `python -c "import __graft_entry__ as g; g.build()"`), importing the
engine raises instead of silently computing on the host.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libquic_fec.so")
# A/B experiments on one GPU box: QFEC_LIB_PATH names another build of the same library
LIB_PATH = os.environ.get("QFEC_LIB_PATH", LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)


class Block(ctypes.Structure):
    """cauchy_256.h:52-55 `Block { unsigned char *data; unsigned char row; }`."""
    _fields_ = [("data", _u8p), ("row", ctypes.c_uint8)]


# name -> (restype, argtypes); every symbol include/quic_fec.h declares
SIGNATURES = {
    "_cauchy_256_init": (ctypes.c_int, [ctypes.c_int]),
    "cauchy_256_encode": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_u8p),
                                         ctypes.c_void_p, ctypes.c_int]),
    "cauchy_256_decode": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Block),
                                         ctypes.c_int]),
    "qfec_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "qfec_ctx_destroy": (None, [ctypes.c_void_p]),
    "qfec_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_longlong]),
    "qfec_encode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_decode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_encode_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    "qfec_decode_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_decode_batch_recovered": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int, ctypes.c_longlong,
                                                   ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_decode_batch_recovered_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                                        ctypes.c_int, ctypes.c_int,
                                                        ctypes.c_longlong, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_null_seal_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_null_open_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "qfec_encode_seal_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_seal_groups_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_encode_seal_groups_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                                     ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_open_decode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                              ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_encode_seal_groups_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                          ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]),
    "qfec_open_decode_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_cauchy_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "qfec_synth_fill": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_ulonglong,
                                       ctypes.c_ulonglong, ctypes.c_void_p]),
    "qfec_synth_gather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]),
    "qfec_ctx_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    "qfec_ctx_get_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p,
                                           ctypes.POINTER(ctypes.c_int)]),
    "qfec_last_error": (ctypes.c_char_p, []),
    "qfec_last_kernels": (ctypes.c_char_p, []),
    "qfec_last_grids": (ctypes.c_char_p, []),
    "qfec_set_timing_events": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "qfec_version": (ctypes.c_int, []),
}

_lib = None


def load():
    """Load libquic_fec.so (cached).  Raises if it is absent or lacks a symbol."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make lib` (HIP extension required; "
                          "there is no CPU fallback)")
    # One HIP runtime per process.  torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, the one libquic_fec.so asks for): loading torch first makes the
    # dynamic linker bind our library to that copy.  Loaded the other way round, torch
    # would bring up a second runtime and see no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)   # AttributeError if the export is missing
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class FecError(RuntimeError):
    def __init__(self, rc, what):
        msg = load().qfec_last_error()
        super().__init__(f"{what} failed: rc={rc} ({msg.decode() if msg else ''})")
        self.rc = rc
