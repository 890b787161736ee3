"""Diagnostic (not a test): where the wide-store encode differs from the oracle."""
import numpy as np
import torch
from quic_amd.fec import FecEngine
from quic_amd import synth
from oracle import oracle

k, m, bb, G = 5, 5, 1352, 11
data = synth.group_data(9010, k, bb, G)
p_or, _ = oracle.encode_batch(k, m, bb, data)
for wide in (0, 1):
    eng = FecEngine(0)
    eng.set_option("wide_st", wide)
    d = torch.from_numpy(data).cuda()
    p = torch.zeros((G, m, bb), dtype=torch.uint8, device="cuda")
    eng.encode(k, m, bb, d, p)
    pg = p.cpu().numpy()
    bad = pg != p_or
    print("wide", wide, "mismatch", bad.sum(), "per block j:", bad.sum(axis=(0, 2)).tolist())
    if bad.any():
        b = bad[0, 0]
        runs = []
        i = 0
        while i < bb:
            if b[i]:
                j = i
                while j < bb and b[j]:
                    j += 1
                runs.append((i, j))
                i = j
            else:
                i += 1
        print(" group0 block0 bad runs:", runs[:40])
        print(" per sub-row bad counts:", [int(bad[:, :, t * 169:(t + 1) * 169].sum()) for t in range(8)])
        g0 = pg[0, 0]; o0 = p_or[0, 0]
        print(" got[0:16]", g0[:16].tolist()); print(" exp[0:16]", o0[:16].tolist())
        print(" got[168:176]", g0[168:176].tolist()); print(" exp[168:176]", o0[168:176].tolist())
