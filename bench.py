#!/usr/bin/env python3
"""Device-resident FEC encode+decode benchmark (BASELINE.json `metric`).

One step = one encode of a batch of packet groups (data -> parity) plus one decode of a
receive set of the same batch (the first k packets that arrived, r data blocks lost per
group, recovered out of place), all inputs resident in HBM before timing starts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload A|B|C|D] [--groups G]
  torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1: one rank per GPU)

Workloads (BASELINE.json configs):
  A  65,536 groups of (10 data + 1 XOR parity) x 1350 B, 1-loss decode   [default, N = 1]
  B  65,536 groups of (32 + 4) x 1350 B, GF(2^8) encode + 2-loss decode
  C  1,048,576 groups of (32 + 4) x 1350 B split over the N GPUs (strong scaling),
     per-GPU and aggregate rates                                           [default, N > 1]
  D  65,536 groups of (128 + 16) x 9000 B jumbo, GF(2^8) encode + 8-loss decode
Each 1350 B payload travels as a block_bytes = roundup8(1350 + 2) = 1352 B block
(2-byte length prefix, quic_fec_group.cc:109-121,344-352); jumbo 9000 B -> 9008 B.

Multi-GPU: groups are independent, so every rank runs its own contiguous range of the
global workload (A/B/D: G per rank, weak scaling; C: a 1/N share of 1,048,576 groups,
strong scaling) with no collective on the data path; a barrier brackets the timed
region and the max time over ranks is reported.

value  = goodput = total groups * k * payload_bytes / step time, GiB/s
roofline: the dominant kernel's algorithmic HBM bytes per launch / its mean launch time
(HIP events on the launch stream), against the 8.0 TB/s HBM3E peak.
cpu_baseline: the reference codec (oracle/_ref, compiled from the reference's own
sources) or the oracle port, timed on this host's cores over a bounded sample, 1 thread
and one thread per core of this process's CPU share.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# name: (k, m, payload, losses r, groups, strong)  groups = per GPU (weak) or total (strong)
WORKLOADS = {
    "A": (10, 1, 1350, 1, 65536, False),
    "B": (32, 4, 1350, 2, 65536, False),
    "C": (32, 4, 1350, 2, 1048576, True),
    "D": (128, 16, 9000, 8, 65536, False),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "device-resident FEC encode+decode GiB/s over 1350B-payload packet groups"


def block_bytes(payload):
    bb = payload + 2
    return bb + (-bb) % 8


def workload_label(name, k, m, payload, r, groups_total, world):
    kind = "XOR parity" if m == 1 else "GF(2^8)"
    lab = f"{groups_total} x ({k}+{m}) x {payload}B {kind}, {r}-loss decode"
    if name == "P":
        lab = f"QuicR preset FEC_{k}_{m}: " + lab
    if world > 1:
        lab += f", {world} GPUs"
    return f"{name}: {lab}"


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Cores this process may use (the GPU box gives one GPU's job a share of the host;
    nproc shows the whole machine), capped at 16 as the box's CPU share."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def cpu_codec_rate(k, m, bb, payload, data_h, blocks_h, rows_h, seconds, threads, use_ref):
    """Time only the codec calls: encode into a preallocated parity buffer, decode in place
    on a fresh copy of the receive set made before its timer starts."""
    from oracle import oracle as O
    G = data_h.shape[0]
    parity = np.zeros((G, m, bb), np.uint8)
    work = np.empty_like(blocks_h)
    wrows = np.empty_like(rows_h)
    status = np.zeros(G, np.int32)
    t_enc = t_dec = 0.0
    passes = 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds or passes == 0:
        t0 = time.perf_counter()
        O.encode_into(k, m, bb, data_h, parity, threads=threads, use_ref=use_ref)
        t1 = time.perf_counter()
        np.copyto(work, blocks_h)
        np.copyto(wrows, rows_h)
        # a large np.copyto may stream past the caches (non-temporal stores), which left the
        # decode reading DRAM while the encode read cache-resident data (r02: A decode 8.4 vs
        # encode 32.6 GiB/s on one thread); one load per cache line brings the receive set
        # back, so both legs time the codec on cache-resident data
        np.bitwise_or.reduce(work.reshape(-1).view(np.uint64)[::8]) if work.size % 8 == 0 else None
        t2 = time.perf_counter()
        O.decode_inplace(k, m, bb, work, wrows, status, threads=threads, use_ref=use_ref)
        t3 = time.perf_counter()
        t_enc += t1 - t0
        t_dec += t3 - t2
        passes += 1
    gib = passes * G * k * payload / 2**30
    assert int(np.abs(status).max()) == 0
    return {"value": round(gib / (t_enc + t_dec), 4), "threads": threads, "passes": passes,
            "encode_GiBps": round(gib / t_enc, 3), "decode_GiBps": round(gib / t_dec, 3),
            "encode_s": round(t_enc, 3), "decode_s": round(t_dec, 3)}


def cpu_baseline(k, m, bb, payload, r, data_h, blocks_h, rows_h, seconds):
    """The CPU FEC path on this host: one thread, and one thread per core of the share."""
    from oracle import oracle as O
    use_ref = O.ref_available()
    kind = "reference" if use_ref else "port"
    n = cpu_share()
    G = data_h.shape[0] // n          # per-thread sample; the n-thread leg runs n of them
    one = cpu_codec_rate(k, m, bb, payload, data_h[:G], blocks_h[:G], rows_h[:G],
                         seconds * 0.6, 1, use_ref)
    many = cpu_codec_rate(k, m, bb, payload, data_h, blocks_h, rows_h, seconds * 0.4, n,
                          use_ref) if n > 1 else one
    return {
        "value": many["value"],
        "unit": "GiB/s",
        "cores": n,
        "kind": kind,
        "cpu_model": cpu_model(),
        "sample": f"{G} groups per thread ({n * G} for {n} threads) of the same workload "
                  f"(about 8 MB of data blocks per thread: cache-resident, as the packets a "
                  f"QUIC thread just handled), encode + {r}-loss decode in place, host memory, "
                  f"codec calls only "
                  f"(receive-set copies outside the timer), "
                  f"{'oracle/_ref (reference libcat codec)' if use_ref else 'oracle port'}",
        "threads_n": many,
        "threads_1": one,
    }


def loopback_config0():
    """BASELINE.json configs[0]: one FEC group of 10 x 1350 B payloads, XOR parity encode +
    1-loss recover through the loopback tool with the GPU off (the reference codec as
    the --cpu-codec library).  Returns the tool's JSON line with codec times in us."""
    tool = os.path.join(ROOT, "quic_amd", "bin", "fec_loopback")
    from oracle import oracle as O
    if not (os.path.exists(tool) and O.ref_available()):
        return None
    cmd = [tool, f"--cpu-codec={O.REF_SO}", "--fec", "--m=10", "--k=1", "--bytes=13500",
           "--drop=4", "--port=0"]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
        d = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:   # the bench line still prints; the failure is reported
        return {"error": repr(e)}
    return {"config": "BASELINE configs[0]: 1 group of 10 x 1350 B, XOR parity, packet 4 "
                      "dropped, loopback UDP, reference codec on the CPU",
            "match": d.get("match"), "revived": d.get("revived"),
            "encode_us": round(d["encode_s"] * 1e6, 2), "decode_us": round(d["decode_s"] * 1e6, 2),
            "wall_s": d.get("wall_s")}


# Which template argument of each kernel says "decode" (bool): the PMC summaries are split
# into the encode and the decode phase by it.
_DECODE_ARG = {"xor_dma_kernel": 2, "gf_apply_kernel": 1, "gf_ring_kernel": 3,
               "gf_stream_kernel": 2, "gf_dcol_kernel": 2}
_DECODE_ONLY = ("decode_prep_kernel", "decode_prep_lane_kernel", "m1_prep_kernel",
                "scatter_recovered_kernel", "rows_k1_kernel",
                "gf_bsyn_kernel", "decode_prep_bsyn_kernel", "gf_psyn_kernel",
                "decode_prep_psyn_kernel", "decode_prep_wide_kernel")
_ENCODE_ONLY = ("replicate_kernel",)


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
        if self._hip.hipEventRecord(self.ev[i], self._ct.c_void_p(stream.cuda_stream)) != 0:
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


def _phase(name):
    base = (name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            .replace("qfec::", "").strip())
    kern = base.split("<")[0]
    if kern.startswith("synth_"):
        return None
    if kern in _DECODE_ONLY:
        return "decode"
    if kern in _DECODE_ARG and "<" in base:
        args = [a.strip() for a in base[base.index("<") + 1:base.rindex(">")].split(",")]
        i = _DECODE_ARG[kern]
        if i >= len(args) or args[i] not in ("true", "false"):
            raise ValueError(f"bench._phase: no decode flag at template argument {i} of {base}")
        return "decode" if args[i] == "true" else "encode"
    return "encode" if kern in _ENCODE_ONLY else None


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


def packet_protection(eng, k, m, bb, data, parity, steps, stream):
    """The step next to the codec, each call timed from its kernels
    with the library's timing events (qfec_set_timing_events):
      encode_seal  SerializeFec: encode + seal of the G*m FEC packets (qfec_encode_seal_batch)
      seal         the same G*m seals alone (qfec_null_seal_batch)
      open         the receiver's NullDecrypter open of those packets (qfec_null_open_batch)
      seal_groups  every packet of every group, data and FEC, G*(k+m) seals in one launch
                   (qfec_seal_groups_batch; the reference seals data packets too)
      open_decode  the receiver batch over those G*(k+m) packets with one data packet per
                   group lost: open, place, fill the hole, decode (qfec_open_decode_batch)
    Reported beside the bench line, never `value`."""
    import torch
    from quic_amd import _lib
    lib = _lib.load()
    G = data.shape[0]
    n, hl = G * m, 16
    per = k + m
    na = G * per
    stride = (hl + 12 + bb + 3) // 4 * 4
    dev = data.device
    hdr = torch.arange(na * hl, dtype=torch.int32, device=dev).to(torch.uint8).view(na, hl)
    pkt = torch.empty((n, stride), dtype=torch.uint8, device=dev)
    pkt2 = torch.empty_like(pkt)
    pkt_len = torch.empty(n, dtype=torch.int32, device=dev)
    pkt_len2 = torch.empty_like(pkt_len)
    # the reference's decrypter copies the whole ciphertext to its output first
    plain = torch.empty((n, (bb + 12 + 3) // 4 * 4), dtype=torch.uint8, device=dev)
    plen = torch.empty(n, dtype=torch.int32, device=dev)
    apkt = torch.empty((na, stride), dtype=torch.uint8, device=dev)
    apkt_len = torch.empty(na, dtype=torch.int32, device=dev)
    g_lost = torch.arange(G, device=dev) * per + (torch.arange(G, device=dev) % k)
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device=dev)
    rows = torch.empty((G, k), dtype=torch.uint8, device=dev)
    olen = torch.empty(na, dtype=torch.int32, device=dev)
    rmax = min(k, m)
    rec = torch.empty((G, rmax, bb), dtype=torch.uint8, device=dev)
    rec_rows = torch.empty((G, rmax), dtype=torch.uint8, device=dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    names = ["encode_seal", "seal", "open", "seal_groups", "open_decode"]
    ev = DeviceEvents(2 * len(names))
    t = {x: 0.0 for x in names}
    try:
        for i in range(steps + 1):
            lib.qfec_set_timing_events(ev.ev[0], ev.ev[1])
            eng.encode_seal(k, m, bb, data, parity, hdr[:n], hl, pkt, pkt_len)
            lib.qfec_set_timing_events(ev.ev[2], ev.ev[3])
            eng.null_seal(hdr[:n], hl, parity.view(n, bb), bb, pkt2, pkt_len2)
            lib.qfec_set_timing_events(ev.ev[4], ev.ev[5])
            eng.null_open(pkt, pkt_len, hl, plain, plen)
            lib.qfec_set_timing_events(ev.ev[6], ev.ev[7])
            eng.seal_groups(k, m, bb, data, parity, hdr, hl, bb, apkt, apkt_len)
            lib.qfec_set_timing_events(None, None)
            apkt_len[g_lost] = -1
            lib.qfec_set_timing_events(ev.ev[8], ev.ev[9])
            eng.open_decode(k, m, bb, apkt, apkt_len, hl, blocks, rows, olen, rec, rec_rows,
                            status)
            lib.qfec_set_timing_events(None, None)
            torch.cuda.synchronize(dev)
            if i:   # the first pass is warmup
                for q, x in enumerate(names):
                    t[x] += ev.elapsed_ms(2 * q, 2 * q + 1) / steps
    finally:
        lib.qfec_set_timing_events(None, None)
        ev.close()
    # the same two group calls from host memory to host memory (pinned): the sender's and
    # the receiver's whole per-packet paths including H2D / D2H (never `value`)
    from quic_amd import fec
    data_h = torch.empty(data.shape, dtype=torch.uint8, pin_memory=True)
    data_h.copy_(data)
    hdr_h = hdr.cpu().pin_memory()
    hpkt = torch.empty((na, stride), dtype=torch.uint8, pin_memory=True)
    hpkt_len = torch.empty(na, dtype=torch.int32, pin_memory=True)
    hrcv_len = torch.empty(na, dtype=torch.int32, pin_memory=True)
    hrec = torch.empty((G, rmax, bb), dtype=torch.uint8, pin_memory=True)
    hrr = torch.empty((G, rmax), dtype=torch.uint8, pin_memory=True)
    hst = torch.empty(G, dtype=torch.int32, pin_memory=True)
    t_hs = t_ho = 0.0
    g_lost_h = g_lost.cpu()
    for i in range(steps + 1):
        t0 = time.perf_counter()
        fec.encode_seal_groups_host_into(eng, k, m, bb, data_h, hdr_h, hl, bb, hpkt, hpkt_len)
        t1 = time.perf_counter()
        hrcv_len.copy_(hpkt_len)
        hrcv_len[g_lost_h] = -1
        t2 = time.perf_counter()
        fec.open_decode_host_into(eng, k, m, bb, hpkt, hrcv_len, hl, hrec, hrr, hst)
        t3 = time.perf_counter()
        if i:
            t_hs += (t1 - t0) / steps
            t_ho += (t3 - t2) / steps
    lost_i = torch.arange(G, device=dev) % k
    host_ok = (bool((hpkt_len == hl + 12 + bb).all())
               and bool((hst == 0).all())
               and torch.equal(hrec[:, 0], data_h[torch.arange(G), lost_i.cpu()]))
    ok = (bool((plen == bb).all()) and torch.equal(plain[:, :bb], parity.view(n, bb))
          and torch.equal(pkt, pkt2) and bool((status == 0).all())
          and bool((rec_rows[:, 0] == lost_i.to(torch.uint8)).all())
          and torch.equal(rec[:, 0], data[torch.arange(G, device=dev), lost_i]))
    pkt_bytes = n * (hl + 12 + bb)
    all_bytes = na * (hl + 12 + bb)
    return {"packets": n, "header_bytes": hl, "encrypter": "NullEncrypter (FNV-1a-128 tag)",
            "encode_seal_ms": round(t["encode_seal"], 5), "seal_ms": round(t["seal"], 5),
            "open_ms": round(t["open"], 5),
            "seal_Mpkt_s": round(n / t["seal"] / 1e3, 2),
            "open_Mpkt_s": round(n / t["open"] / 1e3, 2),
            "seal_GBps": round(pkt_bytes / t["seal"] / 1e6, 1),
            "open_GBps": round(pkt_bytes / t["open"] / 1e6, 1),
            "group_packets": na,
            "seal_groups_ms": round(t["seal_groups"], 5),
            "seal_groups_GBps": round(all_bytes / t["seal_groups"] / 1e6, 1),
            "open_decode_ms": round(t["open_decode"], 5),
            "open_decode_GBps": round(all_bytes / t["open_decode"] / 1e6, 1),
            "round_trip_ok": ok,
            "host": {
                "encode_seal_groups_ms": round(t_hs * 1e3, 3),
                "open_decode_ms": round(t_ho * 1e3, 3),
                "GiBps": round(G * k * (bb - 2) / 2**30 / (t_hs + t_ho), 3),
                "pcie_GBps": round((G * k * bb + na * (hl + stride + 4)
                                    + na * (stride + 4) + G * rmax * (bb + 1) + 4 * G)
                                   / (t_hs + t_ho) / 1e9, 2),
                "ok": host_ok,
                "note": "qfec_encode_seal_groups_batch_host then qfec_open_decode_batch_host "
                        "on pinned host buffers (headers and data in, sealed packets out; "
                        "packets in, recovered blocks out), wall clock per call, "
                        "H2D/kernels/D2H pipelined in chunks"},
            "note": "kernel-bracketing events per call; one lane per packet (serial FNV "
                    "chain mod 2^96 in three 32-bit words), packets streamed through "
                    "LDS wave tiles, DESIGN.md 6.2; open_decode loses data packet "
                    "g % k of group g"}


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
        "groups": G,
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
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= WORLD_SIZE; N > 1 runs under torchrun, one rank per GPU)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: A on one GPU, C (strong scaling over 1,048,576 groups) "
                         "on several")
    ap.add_argument("--groups", type=int, default=None,
                    help="groups per GPU (A/B/D) or in total (C); default: the BASELINE size")
    ap.add_argument("--losses", type=int, default=None,
                    help="data blocks lost per group (default: the workload's)")
    ap.add_argument("--preset", default=None, metavar="K,M",
                    help="a QuicR FEC preset instead of the BASELINE codes (quic_fec_group.cc:"
                         "22-82: 5,5 10,10 10,15 10,20 15,15 250,5): 65,536 groups of (K + M) x "
                         "1350 B, min(K, M) // 2 losses unless --losses")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-groups", type=int, default=None,
                    help="groups per thread in the CPU sample (default: about 8 MB of data "
                         "blocks, so the reference's working set stays cache-resident as on "
                         "the QUIC thread)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true",
                    help="accepted for compatibility: every line verifies the timed steps")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (PCIe) leg")
    ap.add_argument("--loss-mode", choices=("random", "fixed"), default="random",
                    help="lost data rows: a fresh random set per group, or rows 0..r-1 in every "
                         "group")
    ap.add_argument("--parity", choices=("random", "first"), default="random",
                    help="parity rows received: a random r-subset per group, or the first r")
    ap.add_argument("--pp", action="store_true",
                    help="also time the packet-protection step (encode + NullEncrypter seal of "
                         "the FEC packets, open)")
    ap.add_argument("--host-groups", type=int, default=None,
                    help="groups in the host-inclusive leg (default: all, at most 4 GB)")
    ap.add_argument("--decode-layout", default="recovered", choices=["recovered", "slots"],
                    help="recovered: qfec_decode_batch_recovered writes the r recovered blocks "
                         "of each group densely (what the receiver consumes); slots: "
                         "qfec_decode_batch writes them into their slots of a [G][k][bb] "
                         "buffer (cauchy_256_decode layout, out of place)")
    ap.add_argument("--host-steps", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true",
                    help="launch each step's kernels one by one instead of replaying the step "
                         "captured once in a HIP graph")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="engine launch option (qfec_ctx_set_option), for A/B experiments")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpus = world if args.gpus is None else args.gpus
    if gpus != world:
        sys.exit(f"--gpus {gpus} but WORLD_SIZE={world}: launch N > 1 GPUs with "
                 f"`torchrun --nproc-per-node {gpus} bench.py --gpus {gpus}`")

    import torch
    import torch.distributed as dist

    # QFEC_BENCH_BACKEND=gloo rehearses the N>1 control flow with several ranks sharing
    # one GPU (RCCL refuses two ranks on one device); the data path has no collective
    # either way, only the barrier, the max-over-ranks time and the per-rank report use it.
    backend = os.environ.get("QFEC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "gloo" and ndev > 0:
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # QFEC_BENCH_PG=1 (under torchrun) keeps the process group at WORLD_SIZE = 1 too, so the
    # N > 1 control flow (RCCL init, barriers, gathers, the max-over-ranks all_reduce) runs on
    # one GPU: a rehearsal of the NCCL branch where no second GPU is available
    pg = world > 1 or os.environ.get("QFEC_BENCH_PG") == "1"
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from quic_amd import fec, shard, synth
    wname = args.workload or ("A" if world == 1 else "C")
    k, m, payload, r, groups_dflt, strong = WORKLOADS[wname]
    if args.preset:
        k, m = (int(x) for x in args.preset.split(","))
        wname, payload, r, groups_dflt, strong = "P", 1350, max(1, min(k, m) // 2), 65536, False
    if args.losses is not None:
        r = args.losses
    groups_arg = args.groups if args.groups is not None else groups_dflt
    bb = block_bytes(payload)
    if strong:
        g0, G = shard.strong_range(groups_arg, world, rank)
        total_groups = groups_arg
    else:
        g0, G = shard.weak_range(groups_arg, rank)
        total_groups = groups_arg * world
    seed = 20251015

    eng = fec.FecEngine(local)
    for o in args.opt:
        name, val = o.split("=", 1)
        eng.set_option(name, int(val))
    eng.reserve(k, m, bb, G)
    stream = torch.cuda.current_stream(dev)

    # ---- resident inputs: this rank's range [g0, g0 + G) of the global workload
    data = torch.empty((G, k, bb), dtype=torch.uint8, device=dev)
    fec.synth_fill(data, seed=seed, byte_offset=shard.data_byte_offset(g0, k, bb))
    parity = torch.zeros((G, m, bb), dtype=torch.uint8, device=dev)
    rc = eng.encode(k, m, bb, data, parity)
    assert rc == 0, rc
    rows_np, src_np = synth.loss_patterns(k, m, r, G, shard.loss_seed(seed, rank),
                                          mode=args.loss_mode, parity=args.parity, shuffle=False)
    rows = torch.from_numpy(rows_np).to(dev)
    src = torch.from_numpy(src_np).to(dev)
    blocks = torch.empty((G, k, bb), dtype=torch.uint8, device=dev)
    fec.synth_gather(data, parity, src, blocks, k, m, bb)
    del src
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

    kernels = {}

    def step(i=None):
        if i is not None:
            rec(4 * i, 4 * i + 1)
        eng.encode(k, m, bb, data, parity)
        kernels["encode"] = fec.last_kernels()
        if i is not None:
            rec(4 * i + 2, 4 * i + 3)
        if recovered:
            eng.decode_recovered(k, m, bb, blocks, rows, out, rows_out, status=status)
        else:
            eng.decode(k, m, bb, blocks, rows, out=out, rows_out=rows_out, status=status)
        kernels["decode"] = fec.last_kernels()
        if i is not None:
            rec(None, None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # The step (its encode and decode launches, every argument fixed) captured once in a HIP
    # graph and replayed: the same kernels with the same work, without the per-call host path.
    # Falls back to eager launches if capture is refused.
    graph, launch_mode = None, "eager launches"
    if not args.no_graph:
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    step()
            torch.cuda.current_stream(dev).wait_stream(side)
            g.replay()
            torch.cuda.synchronize(dev)
            graph, launch_mode = g, "HIP graph replay of the captured step"
        except Exception as e:   # the bench still runs, eagerly; the reason is reported
            launch_mode = f"eager launches (graph capture failed: {e!r:.120})"
            torch.cuda.synchronize(dev)

    def timed_step():
        if graph is not None:
            graph.replay()
        else:
            step()

    for _ in range(2):
        timed_step()
    torch.cuda.synchronize(dev)

    # The timed launches must prove they did the work: keep the parity the untimed encode
    # wrote, then poison every output the step writes (parity, recovered blocks, their rows,
    # status) so that what is checked after the timed region can only come from the timed
    # replays themselves.
    parity_ref = parity.clone()
    parity.zero_()
    out.zero_()
    rows_out.zero_()
    status.fill_(-99)

    # ---- timed region: barrier + sync on both sides, K steps, nothing else on the stream
    # (no timing events: they cost A about 3 % of its step time)
    if pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timed_step()
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # ---- what the timed steps wrote, checked before anything else touches the outputs:
    # the parity equals the untimed encode's, every group recovered exactly its r lost blocks
    # and each equals the data row it names, every status is 0
    verified = torch.equal(parity, parity_ref) and int(status.abs().max()) == 0
    del parity_ref
    if recovered:
        got = rows_out != 255
        g_idx = torch.arange(G, device=dev)[:, None].expand(G, rmax)[got]
        verified = verified and bool((got.sum(dim=1) == r).all()) and bool(
            torch.equal(out[got], data[g_idx, rows_out.long()[got]]))
    else:
        slot = rows.long() >= k
        g_idx = torch.arange(G, device=dev)[:, None].expand(G, k)[slot]
        verified = verified and bool(torch.equal(out[slot], data[g_idx, rows_out.long()[slot]]))
    del g_idx
    if pg:
        flags = [None] * world
        dist.all_gather_object(flags, verified)
        verified = all(flags)

    # ---- roofline pass (after the timed region, same K steps): per-phase kernel timing
    # with HIP events on the launch stream.  The library records a start event at its first
    # kernel's start and a stop event at its last kernel's end (qfec_set_timing_events ->
    # hipExtLaunchKernel), so a phase is timed from its kernels alone, as rocprofv3 times
    # them.  Fallback: event pairs recorded between the calls (these also count the
    # dispatch gaps, ~5-10 us per launch).
    from quic_amd import _lib
    lib = _lib.load()
    try:
        dev_ev = DeviceEvents(4 * args.steps)
        event_kind = "hipExtLaunchKernel start/stop events"

        def rec(a, b):
            ea = dev_ev.ev[a] if a is not None else None
            eb = dev_ev.ev[b] if b is not None else None
            if lib.qfec_set_timing_events(ea, eb) != 0:
                raise RuntimeError("qfec_set_timing_events failed")
        elapsed_ev = dev_ev.elapsed_ms
        # probe once outside the timed region: both events must have been recorded
        rec(0, 1)
        eng.encode(k, m, bb, data, parity)
        rec(None, None)
        torch.cuda.synchronize(dev)
        if not elapsed_ev(0, 1) > 0:
            raise RuntimeError("kernel events not recorded")
    except Exception:
        if lib.qfec_set_timing_events(None, None) != 0:
            raise
        dev_ev = None
        event_kind = "torch.cuda.Event pairs between calls"
        tev = [torch.cuda.Event(enable_timing=True) for _ in range(4 * args.steps)]
        pending = [None]   # stop event of the phase in progress

        def rec(a, b):
            if pending[0] is not None:
                tev[pending[0]].record(stream)
            if a is not None:
                tev[a].record(stream)
            pending[0] = b
        elapsed_ev = lambda a, b: tev[a].elapsed_time(tev[b])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    elapsed_events = time.perf_counter() - t0
    enc_ms = float(np.mean([elapsed_ev(4 * i, 4 * i + 1) for i in range(args.steps)]))
    dec_ms = float(np.mean([elapsed_ev(4 * i + 2, 4 * i + 3) for i in range(args.steps)]))
    if dev_ev is not None:
        dev_ev.close()

    # algorithmic HBM bytes per launch: encode reads k, writes m blocks;
    # decode reads the k received blocks and writes the r recovered ones
    enc_bytes = G * (k + m) * bb
    dec_bytes = G * (k + r) * bb
    enc_gbs = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_bytes / (dec_ms * 1e-3) / 1e9
    step_gbs = (enc_bytes + dec_bytes) / (enc_ms + dec_ms) / 1e6
    mine = {"rank": rank, "device": local, "groups": G, "first_group": g0,
            "wall_ms_per_step": round(elapsed * 1e3 / args.steps, 5),
            "wall_ms_per_step_with_events": round(elapsed_events * 1e3 / args.steps, 5),
            "GiBps": round(G * k * payload / 2**30 / (elapsed / args.steps), 3),
            "encode_ms": round(enc_ms, 5), "decode_ms": round(dec_ms, 5),
            "step_hbm_frac": round(step_gbs / HBM_PEAK_GBS, 4)}
    if pg:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]

    elapsed = shard.max_over_ranks(elapsed, dev if backend == "nccl" else None)
    ms_per_step = elapsed * 1e3 / args.steps
    goodput = total_groups * k * payload / 2**30 / (elapsed / args.steps)

    phase = "encode" if enc_ms >= dec_ms else "decode"
    # PMC summaries: profiles/r*/pmc_<A|B|D>.json, pmc_P<k>_<m>.json for the presets (C: B's)
    traffic, traffic_src = pmc_traffic(f"P{k}_{m}" if wname == "P" else "B" if wname == "C" else wname,
                                       phase, G)
    if phase == "encode":
        dom = (kernels["encode"], enc_gbs, enc_bytes, enc_ms)
    else:
        dom = (kernels["decode"], dec_gbs, dec_bytes, dec_ms)

    cpu = None
    cfg0 = None
    # the CPU baseline runs on rank 0 only, after the timed region (the other ranks wait at
    # the final barrier)
    if rank == 0 and not args.no_cpu_baseline:
        n = min((args.cpu_groups or max(16, (8 << 20) // (k * bb))) * cpu_share(), G)
        cpu = cpu_baseline(k, m, bb, payload, r, data[:n].cpu().numpy(),
                           blocks[:n].cpu().numpy(), rows_np[:n], args.cpu_seconds)
        cfg0 = loopback_config0()

    host = None
    if rank == 0 and world == 1 and not args.no_host:
        hg = args.host_groups or max(1, min(G, (4 << 30) // (2 * k * bb)))
        host = host_inclusive(eng, k, m, bb, payload, data[:hg], blocks[:hg], rows[:hg],
                              args.host_steps, recovered)

    pp = None
    if rank == 0 and world == 1 and args.pp:
        pp = packet_protection(eng, k, m, bb, data, parity, args.steps, stream)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(goodput, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 payload bytes, random per-group loss "
                    "patterns); device-resident",
            "config": {
                "workload": workload_label(wname, k, m, payload, r, total_groups, world),
                "groups_per_gpu": G,
                "groups_total": total_groups,
                "k": k, "m": m, "payload_bytes": payload, "block_bytes": bb,
                "losses_per_group": r,
                "parallelism": f"{world} independent group shards (no collective)",
                "process_group": f"{backend}, world {world}" if pg else "none",
                "decode_layout": args.decode_layout, "loss_mode": args.loss_mode,
                "parity_rows": args.parity,
                "options": args.opt,
                "launch": launch_mode,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom[0],
                "phase": phase,
                "achieved": round(dom[1], 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(dom[1] / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": dom[2],
                "launch_ms": round(dom[3], 5),
                "timing": event_kind + " on the launch stream, per phase, over a second pass "
                          "of the same K steps after the timed region",
            },
            "kernels": {
                "encode": kernels["encode"], "decode": kernels["decode"],
                "encode_ms": round(enc_ms, 5), "encode_GBps": round(enc_gbs, 1),
                "decode_ms": round(dec_ms, 5), "decode_GBps": round(dec_gbs, 1),
                "step_GBps": round(step_gbs, 1),
                "step_hbm_frac": round(step_gbs / HBM_PEAK_GBS, 4),
            },
            "per_gpu": per_rank,
            "cpu_baseline": cpu,
            "cpu_reference_config0": cfg0,
            "host_inclusive": host,
        }
        line["verified"] = verified
        line["verify"] = ("checked after the timed region, before any other launch: outputs "
                          "poisoned before the timed replays; parity equal to the untimed "
                          "encode's, every lost block recovered and equal to its data row, "
                          "status 0 (all groups, on the device)")
        if pp is not None:
            line["packet_protection"] = pp
        print(json.dumps(line), flush=True)

    eng.close()
    if pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
