#!/usr/bin/env python3
"""Build guard: every kernel a host object registers has device code in that object.

A HIP object carries a host pass (kernel stubs, the handles the runtime launches by name) and
a gfx950 code object (the kernels' .kd descriptors).  If the two passes of one source see
different file contents (an edit landing during a build), the host pass registers a stub the
device code lacks, and the runtime aborts at that kernel's first launch ("Cannot find Symbol",
round 3).  The Makefile runs this after every HIP compile and again on all objects before the
library is linked, and deletes what it was checking on a mismatch, so such a build can never
reach the GPU box.

  tools/check_stubs.py OBJ [OBJ ...]      exit 0: consistent, 1: mismatch, 2: tool failure
"""
import os
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def device_kernels(obj, tmp):
    """The .kd names of obj's gfx950 code object, or None for a host-only object."""
    fat = os.path.join(tmp, "fat.bin")
    if os.path.exists(fat):
        os.remove(fat)
    r = subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}",
                        obj, os.path.join(tmp, "scratch.o")], capture_output=True)
    if r.returncode != 0 or not os.path.exists(fat):
        return None
    co = os.path.join(tmp, "dev.co")
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True, capture_output=True)
    dev = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", co], check=True,
                         capture_output=True, text=True).stdout
    return {ln.split()[-1][:-3] for ln in dev.splitlines() if ln.strip().endswith(".kd")}


def host_stubs(obj):
    """Kernel handles the host pass defines: 8-byte OBJECT symbols named like the kernel."""
    host = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", "-W", obj], check=True,
                          capture_output=True, text=True).stdout
    out = set()
    for ln in host.splitlines():
        f = ln.split()
        if len(f) >= 8 and f[3] == "OBJECT" and f[6] != "UND" and f[2] == "8" and \
                f[-1].startswith("_Z") and "_kernel" in f[-1]:
            out.add(f[-1])
    return out


def check(objs):
    """[(obj, missing stubs)] for the objects that fail, and the number of stubs checked."""
    bad, n = [], 0
    tmp = tempfile.mkdtemp()
    try:
        for o in objs:
            kd = device_kernels(o, tmp)
            if kd is None:
                continue
            stubs = host_stubs(o)
            n += len(stubs)
            missing = sorted(stubs - kd)
            if missing:
                bad.append((o, missing))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return bad, n


def main(argv):
    if len(argv) < 2:
        print(__doc__.strip().splitlines()[-1], file=sys.stderr)
        return 2
    if not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        print("check_stubs: no ROCm llvm tools", file=sys.stderr)
        return 2
    try:
        bad, _ = check(argv[1:])
    except (subprocess.CalledProcessError, OSError) as e:
        print(f"check_stubs: {e}", file=sys.stderr)
        return 2
    for o, missing in bad:
        print(f"check_stubs: {o}: host kernel stubs without device code: {missing}",
              file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
