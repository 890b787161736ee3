"""Loopback file transfer with packet-group FEC (tools/loopback/fec_loopback.cpp).

Models the reference's end-to-end check (Script/tests.py:104-108 — send a file through the
lossy loopback, compare digests) on UDP 127.0.0.1 with a seeded dropper.  CPU: the tool run
with the oracle codec (and with the reference codec built in oracle/_ref when present) —
exercising the group framing, the wire format and reassembly.  GPU: --gpu-fec, per-group
and batched, must reproduce the CPU run exactly (same drops -> same revived set and digest)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "quic_amd", "bin", "fec_loopback")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle_fec.so")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_cauchy.so")


@pytest.fixture(scope="module")
def tool():
    if not os.path.exists(TOOL):
        subprocess.run(["make", "-C", ROOT, "tools"], check=True, capture_output=True)
    return TOOL


def run(tool, *args, codec=None, timeout=120):
    cmd = [tool, "--fec"] + list(args)
    cmd += ["--gpu-fec"] if codec is None else [f"--cpu-codec={codec}",
                                                f"--tables={ROOT}/quic_amd/data/cauchy_256_tables.bin"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.stdout.strip(), p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1]), p.returncode


CASES = [
    ("--m=10", "--k=1", "--bytes=13500", "--drop=4"),                   # BASELINE configs[0]
    ("--m=10", "--k=1", "--bytes=1000000", "--loss=0.005", "--seed=3"),
    ("--m=32", "--k=4", "--bytes=4000000", "--loss=0.02", "--seed=7"),
    ("--m=32", "--k=4", "--bytes=777777", "--drop=1,2,3,4,40,77,78"),  # ragged tail, parity losses
    ("--m=128", "--k=16", "--bytes=8000000", "--loss=0.05", "--seed=1"),
    ("--m=5", "--k=5", "--bytes=100000", "--loss=0.2", "--seed=11"),
]


@pytest.mark.parametrize("args", CASES)
def test_loopback_oracle_codec(tool, args):
    r, rc = run(tool, *args, codec=ORACLE_LIB)
    assert r["bytes_out"] == r["bytes"]
    if r["unrecovered"] == 0:
        assert rc == 0 and r["match"] and r["sha256_in"] == r["sha256_out"]
    else:
        assert rc == 1 and not r["match"]
    assert r["received_data"] + r["revived"] + r["unrecovered"] == r["packets_sent"] - r["fec_sent"]
    if "--drop=4" in args:
        assert (r["dropped"], r["revived"], r["unrecovered"]) == (1, 1, 0)


def test_loopback_reference_codec_agrees(tool):
    if not os.path.exists(REF_LIB):
        pytest.skip("reference codec not built (oracle/_ref)")
    for args in CASES:
        a, _ = run(tool, *args, codec=ORACLE_LIB)
        b, _ = run(tool, *args, codec=REF_LIB)
        for key in ("dropped", "revived", "unrecovered", "sha256_out"):
            assert a[key] == b[key], (args, key)


def test_loopback_zero_loss(tool):
    r, rc = run(tool, "--m=32", "--k=4", "--bytes=2000000", codec=ORACLE_LIB)
    assert rc == 0 and r["dropped"] == 0 and r["revived"] == 0 and r["match"]


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 64])
@pytest.mark.parametrize("args", CASES)
def test_loopback_gpu_matches_cpu(tool, args, batch):
    ref, _ = run(tool, *args, codec=ORACLE_LIB)
    extra = [f"--batch={batch}"] if batch else []
    got, rc = run(tool, *args, *extra)
    assert got["codec"] == "gpu"
    for key in ("dropped", "revived", "unrecovered", "sha256_in", "sha256_out", "match"):
        assert got[key] == ref[key], key
    assert rc == (0 if ref["match"] else 1)
