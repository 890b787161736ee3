"""Multi-process engine run on the GPU: two gloo ranks, each running the
ENGINE (libquic_fec.so, not the oracle) on its strong-split range of BASELINE config C
(1,048,576 groups of (32 + 4) x 1350 B), both on device 0 of the one-GPU box.

This is bench.py's N > 1 path minus RCCL (which refuses two ranks on one device): each
rank generates its range of the global splitmix64 stream by byte offset, encodes, loses
2 data blocks per group, decodes in the recovered-blocks layout and checks every
recovered block; sampled groups (including the first and last of each range) are checked
against the CPU oracle byte for byte, the ranges must tile the global batch, and the
max-over-ranks time reduction bench.py uses must return the slowest rank's time.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import time

    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from quic_amd import fec, shard, synth
        k, m, bb, r, seed = 32, 4, 1352, 2, 1357
        torch.cuda.set_device(0)
        g0, G = shard.strong_range(total, world, rank)
        eng = fec.FecEngine(0)
        data = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
        fec.synth_fill(data, seed=seed, byte_offset=shard.data_byte_offset(g0, k, bb))
        parity = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
        rows, src = synth.loss_patterns(k, m, r, G, shard.loss_seed(seed, rank))
        blocks = torch.empty((G, k, bb), dtype=torch.uint8, device="cuda")
        rec = torch.zeros((G, 4, bb), dtype=torch.uint8, device="cuda")
        rr = torch.zeros((G, 4), dtype=torch.uint8, device="cuda")
        st = torch.full((G,), 9, dtype=torch.int32, device="cuda")
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert eng.encode(k, m, bb, data, parity) == 0
        enc_kernels = fec.last_kernels()
        fec.synth_gather(data, parity, torch.from_numpy(src).cuda(), blocks, k, m, bb)
        eng.decode_recovered(k, m, bb, blocks, torch.from_numpy(rows).cuda(), rec, rr, status=st)
        dec_kernels = fec.last_kernels()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ok = int(st.abs().max()) == 0
        got = rr != 255
        ok = ok and bool((got.sum(dim=1) == r).all())
        g_idx = torch.arange(G, device="cuda")[:, None].expand(G, 4)[got]
        ok = ok and torch.equal(rec[got], data[g_idx, rr.long()[got]])
        # sampled groups vs the oracle: parity and recovered blocks
        sample = [0, 1, G // 2, G - 1]
        d_np = data[sample].cpu().numpy()
        p_or, _ = O.encode_batch(k, m, bb, d_np)
        par_ok = np.array_equal(parity[sample].cpu().numpy(), p_or)
        recv = synth.assemble_received(d_np, p_or, src[sample])
        b_or, r_or, s_or = O.decode_batch(k, m, bb, recv, rows[sample])
        rec_np, rr_np = rec[sample].cpu().numpy(), rr[sample].cpu().numpy()
        for i in range(len(sample)):
            era = sorted(set(range(k)) - set(int(x) for x in rows[sample[i]] if x < k))
            assert rr_np[i][:r].tolist() == era
            for j, e in enumerate(era):
                slot = [s for s in range(k) if r_or[i][s] == e][0]
                par_ok = par_ok and np.array_equal(rec_np[i][j], b_or[i][slot])
        # the first group of this range is the global stream at its offset
        stream_ok = np.array_equal(d_np[0].ravel(),
                                   synth.stream_bytes(seed, g0 * k * bb, k * bb))
        ranges = [None] * world
        dist.all_gather_object(ranges, (g0, G))
        tmax = shard.max_over_ranks(elapsed + 10.0 * rank)   # rank 1 made the slow one
        eng.close()
        q.put((rank, ranges, bool(ok), bool(par_ok), bool(stream_ok), tmax, elapsed,
               enc_kernels, dec_kernels))
    except Exception as e:   # report, do not hang the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_engine_strong_shards_gloo_world2():
    import torch.multiprocessing as mp
    world, total = 2, 1048576
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=110) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    res.sort(key=lambda x: x[0])
    for x in res:
        assert len(x) > 2, f"rank {x[0]} failed: {x[1]}"
    for p in procs:
        assert p.exitcode == 0
    assert res[0][1] == [(0, total // 2), (total // 2, total // 2)]   # tiles the batch
    for rank, ranges, ok, par_ok, stream_ok, tmax, elapsed, ek, dk in res:
        assert ok, f"rank {rank}: a recovered block differs from its original"
        assert par_ok, f"rank {rank}: sampled groups differ from the oracle"
        assert stream_ok, f"rank {rank}: shard bytes are not the global stream"
        assert "gf_ring" in ek and "bsyn" in dk, (ek, dk)
    slowest = max(res[1][6] + 10.0, res[0][6])
    assert all(abs(x[5] - slowest) < 1e-6 for x in res)
