"""Probe: gf_apply encode time vs sub-row alignment on the D shape (128 + 16, 16,384 groups).
bb = 9008 (s = 1126, odd sub-rows 2 bytes off a dword) against bb = 9024 (s = 1128, every
sub-row dword-aligned); both have 282 column words per sub-row.  Timing only."""
import sys
import torch
sys.path.insert(0, ".")
from quic_amd import fec

eng = fec.FecEngine(0)
k, m, G = 128, 16, 16384
for bb in (9008, 9024, 9008, 9024):
    eng.reserve(k, m, bb, G)
    data = torch.randint(0, 256, (G, k, bb), dtype=torch.uint8, device="cuda")
    par = torch.empty((G, m, bb), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        assert eng.encode(k, m, bb, data, par) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        eng.encode(k, m, bb, data, par)
    e1.record()
    torch.cuda.synchronize()
    print(f"bb={bb} s={bb // 8} encode_ms={e0.elapsed_time(e1) / 5:.3f}", flush=True)
    del data, par
    torch.cuda.empty_cache()
