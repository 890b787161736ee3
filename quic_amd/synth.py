"""Synthetic FEC workloads: seeded packet-group data and loss patterns.

Shared by the tests, the golden-vector generator and bench.py so that every
party builds byte-identical inputs from a seed.

Data stream: byte b of a workload is byte (b % 8) (little-endian) of the 64-bit
word splitmix64_mix(seed + (b // 8 + 1) * 0x9E3779B97F4A7C15), i.e. the
sequential splitmix64 generator.  The HIP library's `qfec_synth_fill` kernel and
the C oracle's `oracle_fill_stream` produce the same stream, so huge inputs can
be generated on the device and small slices re-derived on the host.

Loss patterns follow the reference receiver (`quic_fec_group.cc:234-297`): of a
group's k data + m parity packets, r data rows and some parity rows are lost; the
decoder is handed the first k packets that arrived, each tagged with
row = packet_number - group_min (data 0..k-1, parity k..k+m-1).
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def stream_bytes(seed, offset, n):
    """n bytes of the seeded stream starting at byte `offset` (uint8 array)."""
    if n == 0:
        return np.zeros(0, np.uint8)
    w0 = offset // 8
    w1 = (offset + n + 7) // 8
    idx = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        words = _mix(np.uint64(seed) + (idx + np.uint64(1)) * GOLDEN)
    b = words.astype("<u8").view(np.uint8)
    s = offset - w0 * 8
    return b[s:s + n].copy()


def group_data(seed, k, bb, groups, first_group=0):
    """uint8 [groups][k][bb]: the stream laid out as consecutive groups."""
    off = first_group * k * bb
    return stream_bytes(seed, off, groups * k * bb).reshape(groups, k, bb)


def loss_patterns(k, m, r, groups, seed, mode="random", parity="random", shuffle=False):
    """Build per-group receive sets.

    Returns (rows [G][k] uint8, src [G][k] int16): slot i of group g holds the
    block with row rows[g][i]; src[g][i] indexes the group's sent blocks
    (0..k-1 data, k..k+m-1 parity), i.e. src == rows for these patterns.

    r      data blocks lost per group (0 <= r <= min(k, m)).
    mode   "random": a fresh set of lost data rows per group; "fixed": the same
           set for every group (rows 0..r-1).
    parity which parity rows stand in: "random" subset of size r, or "first"
           (rows k..k+r-1).
    shuffle  arrival order shuffled within the group (default: packet-number order).
    """
    if not 0 <= r <= min(k, m):
        raise ValueError("need 0 <= r <= min(k, m)")
    rng = np.random.default_rng(seed)
    # lost data rows: the r smallest of k random keys per group (uniform r-subset)
    if mode == "fixed":
        lost = np.broadcast_to(np.arange(r), (groups, r))
    else:
        lost = np.sort(np.argsort(rng.random((groups, k)), axis=1)[:, :r], axis=1)
    if parity == "first":
        par = np.broadcast_to(np.arange(r) + k, (groups, r))
    else:
        par = np.sort(np.argsort(rng.random((groups, m)), axis=1)[:, :r], axis=1) + k
    keep_mask = np.ones((groups, k), bool)
    np.put_along_axis(keep_mask, lost, False, axis=1)
    keep = np.nonzero(keep_mask)[1].reshape(groups, k - r)   # ascending per group
    rows = np.concatenate([keep, par], axis=1).astype(np.int64)
    if shuffle:
        perm = np.argsort(rng.random((groups, k)), axis=1)
        rows = np.take_along_axis(rows, perm, axis=1)
    return rows.astype(np.uint8), rows.astype(np.int16)


def assemble_received(data, parity, src):
    """blocks [G][k][bb] = the sent blocks named by src (host-side gather)."""
    G, k, bb = data.shape
    sent = np.concatenate([data, parity], axis=1)
    return np.take_along_axis(sent, src.astype(np.int64)[:, :, None].repeat(bb, axis=2), axis=1)
