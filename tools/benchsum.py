#!/usr/bin/env python3
"""One summary line per bench log: the last JSON line of each file named on the command line
(gpurun_out/<step>.log as written by tools/gpu_session.sh)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = [x for x in open(path) if x.startswith("{")]
        d = json.loads(lines[-1])
    except (OSError, IndexError, ValueError) as e:
        print(f"{path}: no bench line ({e.__class__.__name__})")
        continue
    k = d["kernels"]
    print(f"{path}: {d['value']} GiB/s  ms/step {d['ms_per_step']}  enc {k['encode_ms']} ms "
          f"({k['encode_GBps']} GB/s)  dec {k['decode_ms']} ms ({k['decode_GBps']} GB/s)  "
          f"frac {d['roofline']['frac']}  verified {d.get('verified')}  "
          f"[{k['encode']} | {k['decode']}]")
