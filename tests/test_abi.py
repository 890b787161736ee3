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
    same object's gfx950 code object.  A host pass and a device pass of one source that see
    different file contents (an edit during a build) leave a stub the runtime cannot
    resolve: `Cannot find Symbol` and an abort at the first launch."""
    import glob
    import shutil
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "*.o")))
    if not objs or not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        pytest.skip("no build objects or no ROCm llvm tools")
    tmp = tempfile.mkdtemp()
    try:
        checked = nhandles = 0
        for o in objs:
            fat = os.path.join(tmp, "fat.bin")
            r = subprocess.run([os.path.join(llvm, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}",
                                o, os.path.join(tmp, "scratch.o")], capture_output=True)
            if r.returncode != 0 or not os.path.exists(fat):
                continue                                  # host-only object
            co = os.path.join(tmp, "dev.co")
            subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--output={co}"], check=True, capture_output=True)
            dev = subprocess.run([os.path.join(llvm, "llvm-readelf"), "-s", co], check=True,
                                 capture_output=True, text=True).stdout
            kd = {ln.split()[-1][:-3] for ln in dev.splitlines() if ln.strip().endswith(".kd")}
            host = subprocess.run([os.path.join(llvm, "llvm-readelf"), "-s", "-W", o], check=True,
                                  capture_output=True, text=True).stdout
            # a kernel's host handle is an 8-byte OBJECT named exactly like the device entry
            stubs = {ln.split()[-1] for ln in host.splitlines()
                     if " OBJECT " in ln and " UND " not in ln and "_kernel" in ln.split()[-1]}
            missing = sorted(stubs - kd)
            assert not missing, f"{os.path.basename(o)}: host stubs without device code: {missing}"
            os.remove(fat)
            checked += 1
            nhandles += len(stubs)
        assert checked >= 5 and nhandles >= 100
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


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
