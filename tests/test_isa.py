"""ISA guard for the counted-vmcnt kernels (CPU only: hipcc cross-compiles gfx950).

gf_stream_kernel / gf_ring_kernel (quic_amd/csrc/gf_stream.hip), gf_bsyn_kernel (gf_bsyn.hip)
gf_psyn_kernel (gf_psyn.hip) and gf_dcol_kernel (gf_dcol.hip) keep their own count of the VMEM instructions they issued and wait with `s_waitcnt vmcnt(N)` for
exactly the pieces a block needs.  That is only sound if the compiler emits no VMEM
instruction outside the count (a global_load of a uniform byte, a register spill, say) and
inserts no vmcnt wait of its own (which would drain the pipeline).  This test compiles the
files and checks both."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
COUNTED = {"global_load_lds_dwordx4", "buffer_load_dwordx4", "buffer_store_dword", "buffer_store_dwordx2",
           "buffer_store_short", "buffer_store_byte"}
DMA = ("global_load_lds_dwordx4", "buffer_load_dwordx4")   # the latter only as `... lds`


DCOL = ["gf_dcol_e63", "gf_dcol_e83", "gf_dcol_d62", "gf_dcol_d82"]
PSYN = ["gf_psyn_1010", "gf_psyn_1015", "gf_psyn_1020", "gf_psyn_1515", "gf_psyn_55"]


@pytest.fixture(scope="module", params=["gf_stream", "gf_bsyn"] + PSYN + DCOL)
def stream_isa(tmp_path_factory, request):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    name = request.param
    src = os.path.join(ROOT, "quic_amd", "csrc", f"{name}.hip")
    # the build keeps the assembly its object was made from (Makefile SAVE_ASM); use it when
    # it is newer than every input, else compile the file here
    built = os.path.join(ROOT, "build", f"{name}-hip-amdgcn-amd-amdhsa-gfx950.s")
    csrc = os.path.join(ROOT, "quic_amd", "csrc")
    inputs = [src] + [os.path.join(ROOT, "tools", f) for f in ("gen_cauchy_const.py", "gen_win_jump.py")]
    # the headers the object was built from: its -MMD dependency file
    dep = os.path.join(ROOT, "build", f"{name}.d")
    if os.path.exists(dep):
        text = open(dep).read().replace("\\\n", " ")
        first = text.split("\n", 1)[0]
        inputs += [f for f in first.split(":", 1)[1].split() if os.path.exists(f)]
    else:
        inputs += [os.path.join(csrc, h) for h in ("fec_kernels.h", "gf_bitslice.h", "gf256.h",
                                                   "gf_dcol.h", "gf_psyn.h", "gf_winjump.h")]
    if os.path.exists(built) and all(os.path.getmtime(built) >= os.path.getmtime(f)
                                     for f in inputs):
        out = built
    else:
        out = str(tmp_path_factory.mktemp("isa") / f"{name}.s")
        for gen in ("gen_cauchy_const.py", "gen_win_jump.py"):
            subprocess.run(["python3", os.path.join(ROOT, "tools", gen)], check=True,
                           capture_output=True)
        extra = ["-mllvm", "-simplifycfg-sink-common=false"] if name.startswith("gf_psyn") else []
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", *extra,
                        "-mllvm", "-structurizecfg-skip-uniform-regions=true", "-DQFEC_BUILD",
                        "-I", os.path.join(ROOT, "build", "gen"), "-I", csrc,
                        "--cuda-device-only", "-S", "-o", out, src],
                       check=True, capture_output=True)
    with open(out) as f:
        text = f.read()
    bodies = {}
    for m in re.finditer(r"^(_ZN4qfec(?:12_GLOBAL__N_1)?\d+gf_\w+?_kernel\w+):", text, re.M):   # every kernel
        end = text.index(".Lfunc_end", m.end())
        bodies[m.group(1)] = text[m.end():end]
    assert len(bodies) >= (1 if name in DCOL + PSYN else 2), "expected the kernel instantiations"
    assert not re.search(r"\.private_segment_fixed_size:\s+[1-9]", text), "register spills"
    return bodies


def test_only_counted_vmem(stream_isa):
    for name, body in stream_isa.items():
        ops = re.findall(r"^\s+((?:global|buffer|flat|scratch)_\w+)", body, re.M)
        extra = sorted(set(ops) - COUNTED)
        assert not extra, f"{name}: VMEM outside the vmcnt bookkeeping: {extra}"
        assert any(d in ops for d in DMA)
        for line in re.findall(r"^\s+buffer_load_dwordx4[^\n]*", body, re.M):
            assert line.rstrip().endswith("lds"), f"{name}: register load: {line.strip()}"


def test_no_compiler_vmcnt_waits(stream_isa):
    for name, body in stream_isa.items():
        lines = body.split("\n")
        for i, line in enumerate(lines):
            if "s_waitcnt" in line and "vmcnt" in line:
                assert lines[i - 1].strip() == ";;#ASMSTART", \
                    f"{name}: compiler-inserted wait: {line.strip()}"
