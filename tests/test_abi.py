"""CPU: the C-ABI library loads and exports every symbol include/quic_fec.h declares;
host-side tables match the oracle.  No compute calls (no GPU here)."""
import os
import re
import subprocess

import numpy as np
import pytest

from quic_amd import _lib, fec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    """Every function declared (QFEC_API) by the public headers include/*.h."""
    syms = set()
    for name in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if name.endswith(".h"):
            with open(os.path.join(ROOT, "include", name)) as f:
                text = f.read()
            syms |= set(re.findall(r"^QFEC_API\s+[\w\s\*]*?\b(\w+)\s*\(", text, re.M))
    return syms


def test_library_exports_every_header_symbol():
    syms = header_symbols()
    assert {"_cauchy_256_init", "cauchy_256_encode", "cauchy_256_decode",
            "qfec_encode_batch", "qfec_decode_batch"} <= syms
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert syms <= exported, syms - exported
    # nothing else leaks out of the C ABI (internal kernels/launchers are hidden)
    extra = {s for s in exported if not s.startswith(("_Z", "__")) and s not in syms}
    assert not extra, extra


def test_no_undefined_kernel_handles():
    """Every kernel the launchers name has its host-side handle in the library (a kernel
    body the host pass cannot compile drops the handle silently, and the library then fails
    to load on the GPU box)."""
    out = subprocess.run(["nm", "-u", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    missing = [line.split()[-1] for line in out.splitlines() if "4qfec" in line]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    from quic_amd import fec_group
    assert header_symbols() <= set(_lib.SIGNATURES) | set(fec_group._SIG)
    L = _lib.load()
    for name in header_symbols():
        assert getattr(L, name) is not None


def test_block_struct_layout():
    import ctypes
    # cauchy_256.h:52-55: { unsigned char *data; unsigned char row; }
    assert ctypes.sizeof(_lib.Block) == 16
    assert _lib.Block.row.offset == 8


def test_no_cpu_fallback_in_product():
    # the product library must not link or embed the oracle
    out = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in out
    ldd = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "ref_cauchy" not in ldd
    src = open(os.path.join(ROOT, "quic_amd", "fec.py")).read()
    assert "oracle" not in src.replace("oracle/_ref", "")


@pytest.mark.parametrize("k,m", [(32, 4), (10, 2), (10, 6), (128, 16), (10, 20), (250, 5),
                                 (200, 56), (1, 255), (249, 7)])
def test_cauchy_matrix_matches_oracle(oracle, k, m):
    np.testing.assert_array_equal(fec.cauchy_matrix(k, m), oracle.cauchy_matrix(k, m))


def test_cauchy_matrix_rejects_bad_params():
    with pytest.raises(ValueError):
        fec.cauchy_matrix(250, 7)
    with pytest.raises(ValueError):
        fec.cauchy_matrix(10, 1)


def test_init_version_mismatch_is_minus_one():
    # version check happens before any device access (cauchy_256.cpp:389-398)
    assert fec._cauchy_256_init(1) == -1


def test_no_environment_knobs_in_product():
    """Launch shapes are per-context options (qfec_ctx_set_option); the only environment
    variable the library reads is QFEC_DEVICE (device of the drop-ins' default context)."""
    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    names = set(re.findall(r"\bQFEC_[A-Z0-9_]+", out))
    assert names <= {"QFEC_DEVICE"}, names


def test_timing_events_hook_arguments():
    # qfec_set_timing_events: both events or neither (no GPU call is made)
    import ctypes
    L = _lib.load()
    assert L.qfec_set_timing_events(None, None) == 0
    assert L.qfec_set_timing_events(ctypes.c_void_p(1), None) == -2
    assert L.qfec_set_timing_events(None, ctypes.c_void_p(1)) == -2
    assert L.qfec_set_timing_events(None, None) == 0


def test_every_host_kernel_stub_has_device_code():
    """Each kernel a host object registers has a device entry (its .kd descriptor) in the
    same object's gfx950 code object (tools/check_stubs.py, which `make lib` also runs).  A
    host pass and a device pass of one source that see different file contents (an edit
    during a build) leave a stub the runtime cannot resolve: `Cannot find Symbol` and an
    abort at the first launch."""
    import glob
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_stubs
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "*.o")))
    if not objs or not os.path.exists(os.path.join(check_stubs.LLVM, "llvm-readelf")):
        pytest.skip("no build objects or no ROCm llvm tools")
    bad, n = check_stubs.check(objs)
    assert not bad, bad
    assert n >= 100


_STUB_SRC = r"""
#include <hip/hip_runtime.h>
#if defined(__HIP_DEVICE_COMPILE__) && defined(MISMATCH)
__global__ void probe_dev_kernel(int* p) { *p = 2; }     // the device pass sees another file
#else
__global__ void probe_kernel(int* p) { *p = 1; }
#endif
#if !defined(__HIP_DEVICE_COMPILE__)
extern "C" void probe_launch(int* p) { hipLaunchKernelGGL(probe_kernel, 1, 1, 0, 0, p); }
#endif
"""


@pytest.mark.parametrize("mismatch", [False, True])
def test_make_lib_refuses_a_stub_without_device_code(tmp_path, mismatch):
    """The Makefile's link rule runs the stub check: an object whose host pass registers a
    kernel its device pass does not contain fails `make` and leaves no library behind; a
    consistent object links."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    src = tmp_path / "probe.hip"
    src.write_text(_STUB_SRC)
    obj = tmp_path / "probe.o"
    flags = ["-Xarch_device", "-DMISMATCH"] if mismatch else []
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-fPIC", *flags, "-c", str(src),
                    "-o", str(obj)], check=True, capture_output=True)
    lib = tmp_path / "libprobe.so"
    lib.write_bytes(b"stale")      # a library from an earlier build must not survive a failure
    os.utime(lib, (0, 0))          # older than the object: make relinks it
    r = subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "Makefile"), f"LIB={lib}",
                        f"OBJS={obj}", str(lib)], capture_output=True, text=True)
    if mismatch:
        assert r.returncode != 0
        assert "without device code" in r.stderr and "probe_kernel" in r.stderr
        assert not lib.exists()
    else:
        assert r.returncode == 0, r.stderr
        assert lib.exists() and lib.read_bytes()[:4] == b"\x7fELF"


def test_grouped_packet_entry_points_reject_bad_arguments():
    """qfec_seal_groups_batch / qfec_encode_seal_groups_batch / qfec_open_decode_batch
    validate their arguments before any device access: a null context returns -2 (no GPU
    call is made; the k + m limits need a context and are covered by the GPU tests)."""
    L = _lib.load()
    args_seal = (1, 1, 1352, 0, None, None, None, 0, None, 0, None, 1352, None, 1400, None,
                 None)
    assert L.qfec_seal_groups_batch(None, *args_seal) == -2
    assert L.qfec_encode_seal_groups_batch(None, *args_seal) == -2
    assert L.qfec_open_decode_batch(None, 10, 1, 1352, 0, None, 1400, None, None, 16, None,
                                    None, None, None, None, None, None) == -2


def test_host_buffer_arguments_checked_before_the_call():
    """The host-to-host wrappers check every buffer's dtype and row count before the library
    call: the library copies whole rows into and out of them, so a short packet
    or length buffer would be overrun and an int64 length array misread.  The engine is never
    touched (None), so this runs without a GPU."""
    import torch
    k, m, bb, G = 10, 1, 1352, 3
    n = G * (k + m)
    u8, i32 = torch.uint8, torch.int32
    data = torch.zeros((G, k, bb), dtype=u8)
    hdr = torch.zeros((n, 20), dtype=u8)
    pkt = torch.zeros((n, 1400), dtype=u8)
    plen = torch.zeros(n, dtype=i32)
    bad = [
        dict(pkt=torch.zeros((n - 1, 1400), dtype=u8)),             # one packet row short
        dict(plen=torch.zeros(n - 1, dtype=i32)),                    # one length short
        dict(plen=torch.zeros(n, dtype=torch.int64)),                # int64 lengths
        dict(hdr_len=torch.zeros(n, dtype=torch.int64)),
        dict(hdr=torch.zeros((n, 20), dtype=torch.int8)),
        dict(data=torch.zeros((G, k, bb - 8), dtype=u8)),            # wrong block size
    ]
    for b in bad:
        a = dict(data=data, hdr=hdr, hdr_len=16, pkt=pkt, plen=plen)
        a.update(b)
        with pytest.raises(ValueError):
            fec.encode_seal_groups_host_into(None, k, m, bb, a["data"], a["hdr"], a["hdr_len"],
                                             bb, a["pkt"], a["plen"])
    with pytest.raises(TypeError):
        fec.encode_seal_groups_host_into(None, k, m, bb, data, hdr, 16, bb, pkt[:, ::2], plen)
    rmax = min(k, m)
    rec, rr, st = (torch.zeros((G, rmax, bb), dtype=u8), torch.zeros((G, rmax), dtype=u8),
                   torch.zeros(G, dtype=i32))
    for b in [dict(plen=torch.zeros(n + 5, dtype=i32)), dict(st=torch.zeros(G, dtype=torch.int64)),
              dict(rr=torch.zeros((G, rmax + 1), dtype=u8)), dict(ol=torch.zeros(n - 1, dtype=i32))]:
        a = dict(pkt=pkt, plen=plen, rec=rec, rr=rr, st=st, ol=torch.zeros(n, dtype=i32))
        a.update(b)
        with pytest.raises(ValueError):
            fec.open_decode_host_into(None, k, m, bb, a["pkt"], a["plen"], 16, a["rec"], a["rr"],
                                      a["st"], a["ol"])
    blocks, rows = torch.zeros((G, k, bb), dtype=u8), torch.zeros((G, k), dtype=u8)
    with pytest.raises(ValueError):
        fec.decode_recovered_host_into(None, k, m, bb, blocks, torch.zeros((G, k - 1), dtype=u8), rec,
                                       rr, st)
    with pytest.raises(ValueError):
        fec.decode_host_into(None, k, m, bb, blocks, rows, torch.zeros(G + 1, dtype=i32))
    with pytest.raises(ValueError):
        fec.encode_host_into(None, k, m, bb, data, torch.zeros((G, m + 1, bb), dtype=u8))
