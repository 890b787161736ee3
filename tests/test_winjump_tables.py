"""CPU: the generated jump tables of gf_winjump.h (tools/gen_win_jump.py -> build/gen/win_jump.h)
compute the reference's bit-sliced product (cauchy_256.cpp:90-125: output sub-row r = XOR of the
input sub-rows t with bit t of c * alpha^r set, poly 0x187).

The leaves are parsed from the generated header and executed on random column words:
- the nibble tables (wz_mul_acc_rt): leaf (c & 15) of QF_NIB_LEAVES_LO, then leaf (c >> 4) of
  QF_NIB_LEAVES_HI, on the W/Z expansion of expand_wz (gf_bitslice.h), for all 256 c;
- the 256-leaf windowed table (win_mul_rt) on the lo/hi window of win_build, for all 256 c;
and every leaf has the fixed byte size the dispatch multiplies by (eight-byte VALU, four-byte
scalar instructions), so leaf c starts at table + size * c.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from tests.test_psyn_prep import _gf, bitsliced_apply

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "build", "gen", "win_jump.h")


@pytest.fixture(scope="module")
def tables():
    subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_win_jump.py")], check=True)
    text = open(HDR).read()

    def macro(name):
        m = re.search(r"#define %s \\\n((?:    \".*\\n\\t\" \\\n)+)" % name, text)
        assert m, name
        return re.findall(r"\"(.*?)\\n\\t\"", m.group(1))

    return {
        "lo": macro("QF_NIB_LEAVES_LO"),
        "hi": macro("QF_NIB_LEAVES_HI"),
        "win": macro("QF_WIN_JUMP_LEAVES"),
        "nib_bytes": int(re.search(r'#define QF_NIB_LEAF_BYTES_S "(\d+)"', text).group(1)),
        "win_bytes": int(re.search(r"#define QF_WIN_LEAF_BYTES (\d+)", text).group(1)),
    }


def split_leaves(ins, leaf_bytes):
    """Cut the instruction stream at multiples of the leaf size (the dispatch jumps to
    table + leaf_bytes * c); every leaf must hold exactly one s_branch, which ends it or (a
    leaf with nothing to add) starts it, padded with s_nop."""
    leaves, cur, nb = [], [], 0
    for i in ins:
        cur.append(i)
        nb += size(i)
        assert nb <= leaf_bytes, cur
        if nb == leaf_bytes:
            branches = [x for x in cur if x.startswith("s_branch")]
            assert len(branches) == 1 and (cur[-1].startswith("s_branch") or
                                           (cur[0].startswith("s_branch") and
                                            all(x == "s_nop 0" for x in cur[1:]))), cur
            leaves.append(cur)
            cur, nb = [], 0
    assert not cur
    return leaves


def size(i):
    if i.startswith("s_"):
        return 4
    if i.split(" ", 1)[0].endswith("_e32"):
        return 4
    return 8


def run_leaf(leaf, regs):
    for i in leaf:
        if i.startswith("s_"):
            continue
        op, args = i.split(" ", 1)
        args = [a.strip() for a in args.split("bitop3")[0].split(",")]
        vals = [regs[a[2:-1]] if a.startswith("%[") else int(a) for a in args[1:]]
        dst = args[0][2:-1]
        if op.startswith("v_mov"):
            regs[dst] = vals[0]
        elif op.startswith("v_xor_b32"):
            regs[dst] = vals[0] ^ vals[1]
        elif op.startswith("v_bitop3_b32"):
            assert "0x96" in i
            regs[dst] = vals[0] ^ vals[1] ^ vals[2]
        else:
            raise AssertionError(i)


def expand_wz(w8):
    W = list(w8) + [0] * 7
    Z = [0] * 14
    for i in range(7):
        Z[i] = W[i] ^ W[i + 1]
    for n in range(8, 15):
        W[n] = W[n - 1] ^ W[n - 6] ^ Z[n - 8]
    for i in range(7, 14):
        Z[i] = W[i] ^ W[i + 1]
    return W, Z


def window(w8):
    lo, hi = [0] * 16, [0] * 16
    for i in range(16):
        for t in range(4):
            if (i >> t) & 1:
                lo[i] ^= w8[t]
                hi[i] ^= w8[4 + t]
    return lo, hi


def test_leaf_sizes(tables):
    for name, nbytes, count in (("lo", "nib_bytes", 16), ("hi", "nib_bytes", 16),
                                ("win", "win_bytes", 256)):
        assert len(split_leaves(tables[name], tables[nbytes])) == count


def test_products_match_bitsliced_apply(tables, oracle):
    mul, _ = _gf(oracle)
    rng = np.random.default_rng(7)
    lo_l = split_leaves(tables["lo"], tables["nib_bytes"])
    hi_l = split_leaves(tables["hi"], tables["nib_bytes"])
    win_l = split_leaves(tables["win"], tables["win_bytes"])
    for trial in range(4):
        # 8 sub-rows of one 4-byte column word each, as uint32 words
        block = rng.integers(0, 256, 32, dtype=np.uint8)
        w8 = [int.from_bytes(bytes(block[4 * t:4 * t + 4]), "little") for t in range(8)]
        W, Z = expand_wz(w8)
        lo, hi = window(w8)
        for c in range(256):
            exp = bitsliced_apply(mul, c, block)
            exp_w = [int.from_bytes(bytes(exp[4 * t:4 * t + 4]), "little") for t in range(8)]
            # nibble jumps into an accumulator (starting from a random value)
            acc0 = [int(x) for x in rng.integers(0, 2**32, 8, dtype=np.uint64)]
            regs = {f"a{r}": acc0[r] for r in range(8)}
            regs.update({f"w{n}": W[n] for n in range(15)})
            regs.update({f"z{n}": Z[n] for n in range(14)})
            run_leaf(lo_l[c & 15], regs)
            run_leaf(hi_l[c >> 4], regs)
            assert [regs[f"a{r}"] ^ acc0[r] for r in range(8)] == exp_w, c
            # 256-leaf windowed product into a temporary
            regs = {f"l{i}": lo[i] for i in range(1, 16)}
            regs.update({f"h{i}": hi[i] for i in range(1, 16)})
            run_leaf(win_l[c], regs)
            assert [regs[f"t{r}"] for r in range(8)] == exp_w, c
