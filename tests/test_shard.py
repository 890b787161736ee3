"""Multi-GPU sharding logic on CPU: world-size-2 gloo process groups.

Each rank builds its own weak-scaling shard exactly as bench.py does (byte offset into
the global splitmix64 stream, per-rank loss seed), encodes and decodes it with the CPU
oracle (the checker, not the product), and the ranks then check with gloo collectives
that the shards are disjoint and cover the global batch, that the union of the shards
is byte-identical to the single-process workload, and that the max-over-ranks time
reduction bench.py uses picks the slowest rank.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

from quic_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(a):
    return int.from_bytes(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], "little")


def _worker(rank, world, port, k, m, bb, G, seed, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        g0, n = shard.weak_range(G, rank)
        data = synth.group_data(seed, k, bb, n, first_group=g0)
        # same bytes as the device generator would write at this byte offset
        off = shard.data_byte_offset(g0, k, bb)
        assert np.array_equal(data.reshape(-1), synth.stream_bytes(seed, off, n * k * bb))
        parity, rc = O.encode_batch(k, m, bb, data)
        assert rc == 0
        rows, src = synth.loss_patterns(k, m, min(2, m), n, shard.loss_seed(seed, rank))
        recv = synth.assemble_received(data, parity, src)
        blocks, rows_out, status = O.decode_batch(k, m, bb, recv, rows)
        assert int(np.abs(status).max()) == 0
        # round trip: every slot now holds the data block its row names
        assert np.array_equal(blocks, np.take_along_axis(
            data, rows_out.astype(np.int64)[:, :, None].repeat(bb, axis=2), axis=1))

        ranges = [None] * world
        dist.all_gather_object(ranges, (g0, n))
        digests = [None] * world
        dist.all_gather_object(digests, (_digest(data), _digest(parity)))
        t = shard.max_over_ranks(0.5 + rank)          # rank 1 is the "slow" one
        q.put((rank, ranges, digests, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,m,bb", [(10, 1, 1352), (32, 4, 64)])
def test_weak_shards_gloo_world2(oracle, k, m, bb):
    import torch.multiprocessing as mp
    world, G, seed = 2, 6, 4242
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, m, bb, G, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    ranges = res[0][1]
    assert ranges == [(0, G), (G, G)]                  # disjoint, contiguous, covering
    assert all(r[3] == 1.5 for r in res)               # max over ranks
    # the union of the shards is the single-process workload of 2G groups
    full = synth.group_data(seed, k, bb, world * G)
    p_full, _ = oracle.encode_batch(k, m, bb, full)
    for rank, (dd, pd) in enumerate(res[0][2]):
        assert dd == _digest(full[rank * G:(rank + 1) * G])
        assert pd == _digest(p_full[rank * G:(rank + 1) * G])


def test_strong_range_partitions_evenly():
    for total in (0, 1, 7, 65536, 1048576):
        for world in (1, 2, 3, 4, 8):
            got = [shard.strong_range(total, world, r) for r in range(world)]
            assert sum(n for _, n in got) == total
            assert [lo for lo, _ in got] == sorted(lo for lo, _ in got)
            for (lo, n), (lo2, _) in zip(got, got[1:]):
                assert lo + n == lo2
            assert max(n for _, n in got) - min(n for _, n in got) <= 1
    with pytest.raises(ValueError):
        shard.strong_range(10, 2, 2)


def test_aggregate_goodput_is_whole_job():
    one = shard.aggregate_goodput_gib(65536, 1, 10, 1350, 1e-3)
    four = shard.aggregate_goodput_gib(65536, 4, 10, 1350, 1e-3)
    assert four == pytest.approx(4 * one)
