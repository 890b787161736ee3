#!/usr/bin/env python3
"""One line per bench JSON log: encode / decode kernel ms and GB/s, step GiB/s, options.
   python tools/benchtab.py gpurun_out/*.log"""
import json
import sys

for p in sys.argv[1:]:
    line = None
    for ln in open(p, errors="replace"):
        if ln.startswith('{"metric"'):
            line = ln
    if not line:
        continue
    d = json.loads(line)
    k = d.get("kernels", {})
    print(f"{p.split('/')[-1][:48]:48s} {d['value']:8.1f} GiB/s  enc {k.get('encode_ms', 0):7.3f} ms "
          f"{k.get('encode_GBps', 0):6.0f}  dec {k.get('decode_ms', 0):7.3f} ms {k.get('decode_GBps', 0):6.0f} GB/s"
          f"  frac {d['roofline']['frac']:.3f} {d.get('verified')}")
