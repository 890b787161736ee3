"""CPU: the algebra gf_psyn (quic_amd/csrc/gf_psyn.hip) relies on, checked against the oracle.

1. For the QuicR preset codes with m >= 7 the reference's matrix (cauchy_256.cpp:422-480) is
   a column-scaled Cauchy matrix C[y][x] = b_x / (b_x + g_y) with distinct nodes (g_0 = 0
   gives the all-ones row 0, b_0 = 1), so every square submatrix is nonsingular and the
   kernel's Gauss-Jordan needs no pivoting in any row order.
2. A numpy model of the kernel's decode (bit-sliced apply of cauchy_256.cpp:90-125;
   syndromes of every parity row; received rows compacted ascending; the prep's Gauss-Jordan
   coefficients g[p][i], g[p][p] = 1 ^ 1/pivot, replayed on the data in place) recovers the
   same bytes as the oracle on random receive sets, repeated data rows included.
"""
import numpy as np
import pytest

from quic_amd import synth

PSYN = [(10, 10), (10, 15), (10, 20), (15, 15), (5, 5)]
CAUCHY_PSYN = [(10, 10), (10, 15), (10, 20), (15, 15)]   # m >= 7: column-scaled Cauchy


def _gf(oracle):
    mul = np.zeros((256, 256), np.uint8)
    for a in range(256):
        for b in range(256):
            mul[a, b] = oracle.gf_mul(a, b)
    inv = np.zeros(256, np.uint8)
    for a in range(1, 256):
        inv[a] = oracle.gf_div(1, a)
    return mul, inv


@pytest.fixture(scope="module")
def gf(oracle):
    return _gf(oracle)


def full_matrix(oracle, k, m):
    """[m][k] with row 0 = ones (cauchy_matrix gives rows 1 .. m - 1)."""
    return np.concatenate([np.ones((1, k), np.uint8), oracle.cauchy_matrix(k, m)], axis=0)


@pytest.mark.parametrize("k,m", CAUCHY_PSYN)
def test_preset_matrix_is_scaled_cauchy(oracle, gf, k, m):
    mul, inv = gf
    C = full_matrix(oracle, k, m)
    b = C[1] * 0
    # b_x / (b_x + g_y): with g_0 = 0, row 0 gives no information; recover g_y from column 0
    # (b_0 = 1: C[y][0] = 1 / (1 + g_y)) and b_x from row 1 (C[1][x] = b_x / (b_x + g_1))
    g = np.array([0] + [inv[C[y][0]] ^ 1 for y in range(1, m)], np.uint8)
    for x in range(k):
        cand = [bx for bx in range(1, 256) if bx != g[1] and
                mul[bx, inv[bx ^ g[1]]] == C[1][x]]
        assert len(cand) == 1
        b[x] = cand[0]
    assert b[0] == 1
    for y in range(m):
        for x in range(k):
            assert C[y][x] == mul[b[x], inv[b[x] ^ g[y]]]
    assert len(set(b.tolist())) == k and len(set(g.tolist())) == m
    assert not set(b.tolist()) & set(g.tolist())


def _nonsingular(mul, inv, S):
    """Gaussian elimination with pivoting over GF(256): is the square matrix S invertible?"""
    S = S.copy()
    r = S.shape[0]
    for p in range(r):
        nz = [i for i in range(p, r) if S[i][p]]
        if not nz:
            return False
        S[[p, nz[0]]] = S[[nz[0], p]]
        iv = int(inv[S[p][p]])
        for i in range(p + 1, r):
            if S[i][p]:
                S[i] ^= mul[int(mul[S[i][p], iv]), S[p]]
    return True


def test_fec_5_5_matrix_every_square_submatrix_nonsingular(oracle, gf):
    """FEC_5_5's matrix (the ones row and CAUCHY_MATRIX_5's rows, cauchy_256.cpp:428-442) is
    not built from Cauchy nodes in the code, so gf_psyn's no-pivoting Gauss-Jordan is justified
    exhaustively instead: every r x r submatrix (any r received parity rows, any r erased data
    rows) is nonsingular, hence every leading minor of the prep's S is nonzero."""
    import itertools
    mul, inv = gf
    k = m = 5
    C = full_matrix(oracle, k, m)
    for r in range(1, 6):
        for ys in itertools.combinations(range(m), r):
            for xs in itertools.combinations(range(k), r):
                assert _nonsingular(mul, inv, C[np.ix_(ys, xs)]), (ys, xs)


def bitsliced_apply(mul, c, block):
    """c (x) block in the reference's transposed 8 x 8 expansion (cauchy_256.cpp:90-125):
    output sub-row r = XOR of the input sub-rows t with bit t of c * alpha^r set."""
    s = block.size // 8
    sub = block.reshape(8, s)
    out = np.zeros_like(sub)
    a = int(c)
    for r in range(8):
        for t in range(8):
            if (a >> t) & 1:
                out[r] ^= sub[t]
        a = int(mul[a, 2])
    return out.reshape(-1)


def model_decode(mul, inv, C, k, m, blocks, rows):
    """The gf_psyn decode of one group; returns {data row: recovered block}."""
    first, extras = {}, []
    for i, r in enumerate(rows):
        if r < k and r not in first:
            first[r] = i
        else:
            extras.append(i)
    recs = [i for i, r in enumerate(rows) if r >= k]
    n = len(recs)
    era = [x for x in range(k) if x not in first][:n]
    bb = blocks.shape[1]
    T = [np.zeros(bb, np.uint8) for _ in range(m)]
    for x, i in sorted(first.items()):
        for y in range(m):
            T[y] ^= bitsliced_apply(mul, C[y][x], blocks[i])
    for i in extras:
        r = rows[i]
        if r >= k:
            T[r - k] ^= blocks[i]
        else:
            for y in range(m):
                T[y] ^= bitsliced_apply(mul, C[y][r], blocks[i])
    ys = sorted(rows[i] - k for i in recs)
    T = [T[y].copy() for y in ys]
    S = np.array([[C[y][e] for e in era] for y in ys], np.uint8)
    for p in range(n):                    # the prep's elimination, replayed on the data
        piv = int(S[p][p])
        assert piv != 0
        iv = int(inv[piv])
        coef = [(1 ^ iv) if i == p else int(mul[S[i][p], iv]) for i in range(n)]
        f = S[:, p].copy()
        for i in range(n):
            if i != p and f[i]:
                S[i] ^= mul[mul[f[i], iv], S[p]]
        S[p] = mul[S[p], iv]
        Tp = T[p].copy()
        for i in range(n):
            T[i] ^= bitsliced_apply(mul, coef[i], Tp)
    return {era[j]: T[j] for j in range(n)}


@pytest.mark.parametrize("k,m", PSYN)
def test_model_matches_oracle(oracle, gf, k, m):
    mul, inv = gf
    C = full_matrix(oracle, k, m)
    bb, G = 64, 12
    data = synth.group_data(70 + k + m, k, bb, G)
    p_or, _ = oracle.encode_batch(k, m, bb, data)
    rng = np.random.default_rng(k * 100 + m)
    for g in range(G):
        r = int(rng.integers(1, min(k, m) + 1))
        lost = sorted(rng.choice(k, r, replace=False))
        par = sorted(rng.choice(m, r, replace=False))
        rows = [x for x in range(k) if x not in lost] + [k + y for y in par]
        if g == 3:                                   # a repeated data row as an extra
            rows = list(range(k))
            a, b = (5, 7) if k >= 8 else (1, 3)
            rows[a], rows[b] = a + 1, k + 2
        rows = np.array(rows)[rng.permutation(k)]
        sent = np.concatenate([data[g], p_or[g]])
        blocks = sent[rows].copy()
        got = model_decode(mul, inv, C, k, m, blocks, [int(v) for v in rows])
        b_or, r_or, s_or = oracle.decode_batch(k, m, bb, blocks[None], rows[None].astype(np.uint8))
        assert s_or[0] == 0
        for slot in range(k):
            if rows[slot] >= k:                      # a recovery slot the decode rewrote
                x = int(r_or[0][slot])
                np.testing.assert_array_equal(got[x], b_or[0][slot])
