#!/usr/bin/env python3
"""Extract the Longhair Cauchy coefficient tables into a binary data fixture.

The reference codec selects its Cauchy matrices from precomputed tables
(`net/quic/core/libcat/cauchy_tables_256.inc:63-564`): full coefficient rows
for m = 2..6 (`CAUCHY_MATRIX_2..6`, row stride 256-m) and the X[]/Y[] vectors
used to build the matrix for m >= 7 (`CAUCHY_MATRIX_Y[256]`,
`CAUCHY_MATRIX_X[30876]`; consumed by `cauchy_256.cpp:422-480`).  These numbers
are the output of a search program (`tabgen.cpp`) that is not in the reference,
so they cannot be regenerated from first principles: parity bytes depend on
them, so they are carried as DATA.

Output: quic_amd/data/cauchy_256_tables.bin, the plain concatenation

    M2[1*254] | M3[2*253] | M4[3*252] | M5[4*251] | M6[5*250] | Y[256] | X[30876]

(34,902 bytes).  The HIP library embeds this file at build time; the oracle
reads it at init.  Run here only (the GPU box has no /root/reference); the
resulting .bin is committed.
"""
import hashlib
import os
import re
import sys

REF = "/root/reference/net/quic/core/libcat/cauchy_tables_256.inc"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "quic_amd", "data",
                   "cauchy_256_tables.bin")

# (name, expected element count) in blob order
LAYOUT = [("CAUCHY_MATRIX_2", 1 * 254), ("CAUCHY_MATRIX_3", 2 * 253),
          ("CAUCHY_MATRIX_4", 3 * 252), ("CAUCHY_MATRIX_5", 4 * 251),
          ("CAUCHY_MATRIX_6", 5 * 250), ("CAUCHY_MATRIX_Y", 256),
          ("CAUCHY_MATRIX_X", 30876)]


def parse(text):
    # strip comments, then pull `NAME[...] = { numbers };`
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    arrays = {}
    for m in re.finditer(r"(CAUCHY_MATRIX_\w+)\s*\[[^\]]*\]\s*=\s*\{([^}]*)\}", text):
        arrays[m.group(1)] = [int(v, 0) for v in m.group(2).replace("\n", " ").split(",")
                              if v.strip()]
    return arrays


def main():
    with open(REF) as f:
        arrays = parse(f.read())
    blob = bytearray()
    for name, n in LAYOUT:
        vals = arrays[name]
        if len(vals) > n:
            sys.exit(f"{name}: expected {n} values, found {len(vals)}")
        if len(vals) < n:
            # C semantics: a short initializer list zero-fills the rest of the
            # declared array (CAUCHY_MATRIX_Y lists 254 of its 256 entries).
            print(f"note: {name} has {len(vals)} initializers, zero-filled to {n}")
            vals = vals + [0] * (n - len(vals))
        if any(v < 0 or v > 255 for v in vals):
            sys.exit(f"{name}: value out of byte range")
        blob += bytes(vals)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "wb") as f:
        f.write(blob)
    print(f"wrote {len(blob)} bytes to {os.path.normpath(OUT)} "
          f"sha256={hashlib.sha256(blob).hexdigest()}")


if __name__ == "__main__":
    main()
