#!/usr/bin/env python3
"""Device-resident FEC encode+decode benchmark (BASELINE.json `metric`).

One step = one encode of a batch of packet groups (data -> parity) plus one decode of a
receive set of the same batch (the first k packets that arrived, r data blocks lost per
group, recovered out of place), all inputs resident in HBM before timing starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload A|B|D] [--groups G]

Workloads (BASELINE.json configs):
  A  65,536 groups of (10 data + 1 XOR parity) x 1350 B payloads, 1-loss decode  [default]
  B  65,536 groups of (32 + 4) x 1350 B, GF(2^8) encode + 2-loss decode
  D  65,536 groups of (128 + 16) x 9000 B jumbo, GF(2^8) encode + 8-loss decode
Each 1350 B payload travels as a block_bytes = roundup8(1350 + 2) = 1352 B block
(2-byte length prefix, quic_fec_group.cc:109-121,344-352); jumbo 9000 B -> 9008 B.

Multi-GPU (torchrun, one rank per GPU): groups are independent, so every rank runs its
own contiguous shard of the same size (weak scaling) with no collective on the data
path; a barrier brackets the timed region and the max time over ranks is reported.

value  = goodput = total groups * k * payload_bytes / step time, GiB/s
roofline: the dominant kernel's algorithmic HBM bytes per launch / its mean launch time
(HIP events on the launch stream), against the 8.0 TB/s HBM3E peak.
cpu_baseline: the reference codec (oracle/_ref, compiled from the reference's own
sources) or the oracle port, timed on this host's cores over a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (k, m, payload, r, label)
    "A": (10, 1, 1350, 1, "65536 x (10+1) x 1350B XOR parity, 1-loss decode"),
    "B": (32, 4, 1350, 2, "65536 x (32+4) x 1350B GF(2^8), 2-loss decode"),
    "D": (128, 16, 9000, 8, "65536 x (128+16) x 9000B GF(2^8), 8-loss decode"),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def block_bytes(payload):
    bb = payload + 2
    return bb + (-bb) % 8


def cpu_baseline(k, m, bb, payload, r, data_h, blocks_h, rows_h, seconds):
    """Time the CPU codec on a bounded host sample (1 thread)."""
    from oracle import oracle as O
    use_ref = O.ref_available()
    kind = "reference" if use_ref else "port"
    G = data_h.shape[0]
    t_enc = t_dec = 0.0
    groups_done = 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds or groups_done == 0:
        t0 = time.perf_counter()
        O.encode_batch(k, m, bb, data_h, threads=1, use_ref=use_ref)
        t1 = time.perf_counter()
        b = blocks_h.copy()
        t2 = time.perf_counter()
        O.decode_batch(k, m, bb, b, rows_h, threads=1, use_ref=use_ref)
        t3 = time.perf_counter()
        t_enc += t1 - t0
        t_dec += t3 - t2   # (decode_batch copies its inputs: included, a few % at most)
        groups_done += G
    gib = groups_done * k * payload / 2**30
    return {
        "value": round(gib / (t_enc + t_dec), 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": f"{G} groups x {groups_done // G} passes of the same workload "
                  f"(encode + {r}-loss decode), host memory, 1 thread, "
                  f"{'oracle/_ref (reference libcat codec)' if use_ref else 'oracle port'}",
        "encode_s": round(t_enc, 3),
        "decode_s": round(t_dec, 3),
    }


# Which template argument of each kernel says "decode" (bool): the PMC summaries are split
# into the encode and the decode phase by it.
_DECODE_ARG = {"xor_dma_kernel": 2, "gf_apply_kernel": 1, "gf_ring_kernel": 5,
               "gf_stage_kernel": 1, "gf_stream_kernel": 2}
_DECODE_ONLY = ("decode_prep_kernel", "decode_prep_lane_kernel", "m1_prep_kernel",
                "scatter_recovered_kernel", "rows_k1_kernel")



class DeviceEvents:
    """HIP timing events recorded with a device-scope release (hipEventReleaseToDevice).

    torch.cuda.Event records with the default system-scope release, whose cache writeback
    and invalidate land inside the bracketed interval: A's 0.15 ms kernels measured 6-7 %
    longer between torch events than in rocprofv3.  These events come from the HIP runtime
    torch already loaded (same process, same streams), through ctypes."""
    RELEASE_TO_DEVICE = 0x40000000

    def __init__(self, n):
        import ctypes
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
        if path is None:
            raise RuntimeError("libamdhip64 is not loaded")
        self._ct = ctypes
        self._hip = hip = ctypes.CDLL(path)
        hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                            ctypes.c_void_p]
        hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.ev = []
        for _ in range(n):
            e = ctypes.c_void_p()
            if hip.hipEventCreateWithFlags(ctypes.byref(e), self.RELEASE_TO_DEVICE) != 0:
                raise RuntimeError("hipEventCreateWithFlags failed")
            self.ev.append(e)

    def record(self, i, stream):
        if self._hip.hipEventRecord(self.ev[i], ctypes_stream(stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_ms(self, i, j):
        t = self._ct.c_float()
        if self._hip.hipEventElapsedTime(self._ct.byref(t), self.ev[i], self.ev[j]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(t.value)

    def close(self):
        for e in self.ev:
            self._hip.hipEventDestroy(e)
        self.ev = []


def ctypes_stream(stream):
    import ctypes
    return ctypes.c_void_p(stream.cuda_stream)

def kernel_names(k, m, bb):
    """(encode, decode) kernel names the library picks for this shape (fec_api.cpp
    encode_impl / decode_*_impl, gf_stream_supported, launch_decode_prep)."""
    if m == 1:
        return "xor_dma_kernel<encode>", "xor_dma_kernel<decode>"
    rc = lambda n: min(1 << max(n - 1, 0).bit_length(), 8)
    rmax = min(k, m)
    stream = (bb == 1352 and (k * bb) % 16 == 0 and os.environ.get("QFEC_STREAM", "1") != "0")
    enc = ("gf_stream_kernel<encode>" if stream and m <= rc(m) and
           os.environ.get("QFEC_STREAM_ENC", "1") != "0" else "gf_apply_kernel<encode>")
    lane = (rmax <= 4 and k <= 64 and k % 4 == 0 and m * k <= 4096 and
            os.environ.get("QFEC_PREP_LANE", "1") != "0")
    prep = "decode_prep_lane_kernel" if lane else "decode_prep_kernel"
    dec = "gf_stream_kernel<decode>" if stream and rmax <= rc(rmax) else "gf_apply_kernel<decode>"
    return enc, prep + " + " + dec


def _phase(name):
    base = name.split("(")[0].replace("void ", "").replace("qfec::", "").strip()
    kern = base.split("<")[0]
    if kern.startswith("synth_"):
        return None
    if kern in _DECODE_ONLY:
        return "decode"
    if kern in _DECODE_ARG and "<" in base:
        args = [a.strip() for a in base[base.index("<") + 1:base.rindex(">")].split(",")]
        return "decode" if args[_DECODE_ARG[kern]] == "true" else "encode"
    return "encode" if kern == "replicate_kernel" else None


def pmc_traffic(workload, phase, groups):
    """HBM bytes per launch of `phase` from the newest committed PMC summary
    (profiles/r*/pmc_<workload>.json, written by tools/pmc_summary.py), scaled to
    `groups`.  None when no summary covers this workload."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{workload}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    tot = 0
    for name, e in d["kernels"].items():
        if _phase(name) == phase and "traffic_bytes" in e:
            tot += e["traffic_bytes"]
    if not tot:
        return None, None
    return round(tot * groups / d["groups"]), os.path.relpath(files[-1], ROOT)


def host_inclusive(eng, k, m, bb, payload, data, blocks, rows, steps, recovered):
    """Host-resident rate: pinned host buffers in and out, H2D + kernels + D2H through the
    library's pipelined host-pointer entry points (qfec_*_batch_host).  Never `value`."""
    import torch
    from quic_amd import fec
    G = data.shape[0]
    data_h = torch.empty(data.shape, dtype=torch.uint8, pin_memory=True)
    data_h.copy_(data)
    parity_h = torch.empty((G, m, bb), dtype=torch.uint8, pin_memory=True)
    blocks0 = torch.empty(blocks.shape, dtype=torch.uint8, pin_memory=True)
    blocks0.copy_(blocks)
    rows0 = rows.cpu()
    blocks_h = torch.empty_like(blocks0).pin_memory()
    rows_h = torch.empty_like(rows0).pin_memory()
    status_h = torch.zeros((G,), dtype=torch.int32).pin_memory()
    rmax = min(k, m)
    rec_h = torch.empty((G, rmax, bb), dtype=torch.uint8, pin_memory=True)
    rec_rows_h = torch.empty((G, rmax), dtype=torch.uint8, pin_memory=True)
    t_enc = t_dec = 0.0
    for i in range(steps + 1):
        blocks_h.copy_(blocks0)
        rows_h.copy_(rows0)
        t0 = time.perf_counter()
        fec.encode_host_into(eng, k, m, bb, data_h, parity_h)
        t1 = time.perf_counter()
        if recovered:
            fec.decode_recovered_host_into(eng, k, m, bb, blocks_h, rows_h, rec_h, rec_rows_h,
                                           status_h)
        else:
            fec.decode_host_into(eng, k, m, bb, blocks_h, rows_h, status_h)
        t2 = time.perf_counter()
        if i:                      # first pass warms the staging buffers
            t_enc += t1 - t0
            t_dec += t2 - t1
    ok = int(status_h.abs().max()) == 0
    if recovered:
        pcie = G * (k * bb + m * bb) + G * (k * bb + k + rmax * bb + rmax + 4)
    else:
        pcie = G * (k * bb + m * bb) + G * (2 * k * bb + 2 * k + 4)
    return {
        "value": round(G * k * payload / 2**30 / ((t_enc + t_dec) / steps), 3),
        "unit": "GiB/s",
        "encode_ms": round(t_enc / steps * 1e3, 3),
        "decode_ms": round(t_dec / steps * 1e3, 3),
        "pcie_bytes_per_step": pcie,
        "pcie_GBps": round(pcie / ((t_enc + t_dec) / steps) / 1e9, 2),
        "status_ok": ok,
        "note": "pinned host buffers; qfec_encode_batch_host + "
                + ("qfec_decode_batch_recovered_host (recovered blocks only)" if recovered
                   else "qfec_decode_batch_host (in place, cauchy_256_decode semantics)")
                + ", 64 MiB chunks, H2D/kernel/D2H pipelined; not the bench value",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="A", choices=sorted(WORKLOADS))
    ap.add_argument("--groups", type=int, default=65536, help="groups per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-groups", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check recovered data after timing")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (PCIe) leg")
    ap.add_argument("--decode-layout", default="recovered", choices=["recovered", "slots"],
                    help="recovered: qfec_decode_batch_recovered writes the r recovered blocks "
                         "of each group densely (what the receiver consumes); slots: "
                         "qfec_decode_batch writes them into their slots of a [G][k][bb] "
                         "buffer (cauchy_256_decode layout, out of place)")
    ap.add_argument("--host-steps", type=int, default=3)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # QFEC_BENCH_BACKEND=gloo rehearses the N>1 control flow with several ranks sharing
    # one GPU (RCCL refuses two ranks on one device); the data path has no collective
    # either way, only the barrier and the max-over-ranks of the elapsed time use it.
    backend = os.environ.get("QFEC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "gloo" and ndev > 0:
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from quic_amd import fec, shard, synth
    k, m, payload, r, label = WORKLOADS[args.workload]
    bb = block_bytes(payload)
    G = args.groups
    seed = 20251015

    eng = fec.FecEngine(local)
    eng.reserve(k, m, bb, G)
    stream = torch.cuda.current_stream(dev)

    # ---- resident inputs: this rank's shard [rank*G, (rank+1)*G) of the global workload
    data = torch.empty((G, k, bb), dtype=torch.uint8, device=dev)
    g0, _ = shard.weak_range(G, rank)
    fec.synth_fill(data, seed=seed, byte_offset=shard.data_byte_offset(g0, k, bb))
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device=dev)
    rc = eng.encode(k, m, bb, data, parity)
    assert rc == 0, rc
    rows_np, src_np = synth.loss_patterns(k, m, r, G, shard.loss_seed(seed, rank), mode="random",
                                          parity="random", shuffle=False)
    rows = torch.from_numpy(rows_np).to(dev)
    src = torch.from_numpy(src_np).to(dev)
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device=dev)
    fec.synth_gather(data, parity, src, blocks, k, m, bb)
    rmax = min(k, m)
    recovered = args.decode_layout == "recovered"
    if recovered:
        out = torch.zeros((G, rmax, bb), dtype=torch.uint8, device=dev)
        rows_out = torch.zeros((G, rmax), dtype=torch.uint8, device=dev)
    else:
        out = torch.zeros_like(blocks)
        rows_out = torch.zeros_like(rows)
    status = torch.zeros((G,), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    def step(i=None):
        if i is not None:
            rec(3 * i)
        eng.encode(k, m, bb, data, parity)
        if i is not None:
            rec(3 * i + 1)
        if recovered:
            eng.decode_recovered(k, m, bb, blocks, rows, out, rows_out, status=status)
        else:
            eng.decode(k, m, bb, blocks, rows, out=out, rows_out=rows_out, status=status)
        if i is not None:
            rec(3 * i + 2)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # ---- timed region: barrier + sync on both sides, K steps
    # per-kernel HIP events on the launch stream: device-scope release when the runtime
    # offers it (DeviceEvents), torch's default events otherwise
    try:
        dev_ev = DeviceEvents(3 * args.steps)
        event_kind = "hipEventReleaseToDevice"
        rec = lambda j: dev_ev.record(j, stream)
        elapsed_ev = dev_ev.elapsed_ms
    except Exception:
        dev_ev = None
        event_kind = "torch.cuda.Event"
        tev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * args.steps)]
        rec = lambda j: tev[j].record(stream)
        elapsed_ev = lambda a, b: tev[a].elapsed_time(tev[b])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    enc_ms = float(np.mean([elapsed_ev(3 * i, 3 * i + 1) for i in range(args.steps)]))
    dec_ms = float(np.mean([elapsed_ev(3 * i + 1, 3 * i + 2) for i in range(args.steps)]))
    if dev_ev is not None:
        dev_ev.close()

    elapsed = shard.max_over_ranks(elapsed, dev if backend == "nccl" else None)

    ms_per_step = elapsed * 1e3 / args.steps
    total_groups = G * world
    goodput = shard.aggregate_goodput_gib(G, world, k, payload, elapsed / args.steps)

    # algorithmic HBM bytes per launch: encode reads k, writes m blocks;
    # decode reads the k received blocks and writes the r recovered ones
    enc_bytes = G * (k + m) * bb
    dec_bytes = G * (k + r) * bb
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
    step_gbs = (enc_bytes + dec_bytes) / (enc_ms + dec_ms) / 1e6
    if enc_ms >= dec_ms:
        phase = "encode"
    else:
        phase = "decode"
    traffic, traffic_src = pmc_traffic(args.workload, phase, G)
    enc_kern, dec_kern = kernel_names(k, m, bb)
    if enc_ms >= dec_ms:
        dom = ("encode", enc_kern, enc_gbs, enc_bytes)
    else:
        dom = ("decode", dec_kern, dec_gbs, dec_bytes)

    verified = None
    if args.verify:
        if recovered:
            # every group recovered exactly r blocks, each equal to the data row it names
            got = rows_out != 255
            g_idx = torch.arange(G, device=dev)[:, None].expand(G, rmax)[got]
            verified = bool((got.sum(dim=1) == r).all()) and bool(
                torch.equal(out[got], data[g_idx, rows_out.long()[got]]))
        else:
            slot = rows.long() >= k
            g_idx = torch.arange(G, device=dev)[:, None].expand(G, k)[slot]
            verified = bool(torch.equal(out[slot], data[g_idx, rows_out.long()[slot]]))
        verified = verified and int(status.abs().max()) == 0

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n = min(args.cpu_groups, G)
        cpu = cpu_baseline(k, m, bb, payload, r, data[:n].cpu().numpy(),
                           blocks[:n].cpu().numpy(), rows_np[:n], args.cpu_seconds)

    host = None
    if rank == 0 and world == 1 and not args.no_host:
        host = host_inclusive(eng, k, m, bb, payload, data, blocks, rows, args.host_steps,
                              recovered)

    if rank == 0:
        line = {
            "metric": "device-resident FEC encode+decode GiB/s over 1350B-payload packet groups",
            "value": round(goodput, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 payload bytes, random per-group loss "
                    "patterns); device-resident",
            "config": {
                "workload": label,
                "groups_per_gpu": G,
                "groups_total": total_groups,
                "k": k, "m": m, "payload_bytes": payload, "block_bytes": bb,
                "losses_per_group": r,
                "parallelism": f"{world} independent group shards (no collective)",
                "decode_layout": args.decode_layout,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom[1],
                "achieved": round(dom[2], 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(dom[2] / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": dom[3],
                "timing": event_kind + " pairs around each launch, launch stream, timed steps",
            },
            "kernels": {
                "encode_ms": round(enc_ms, 5), "encode_GBps": round(enc_gbs, 1),
                "decode_ms": round(dec_ms, 5), "decode_GBps": round(dec_gbs, 1),
                "step_GBps": round(step_gbs, 1),
                "step_hbm_frac": round(step_gbs / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "host_inclusive": host,
        }
        if verified is not None:
            line["verified"] = verified
        print(json.dumps(line), flush=True)

    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
