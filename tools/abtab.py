#!/usr/bin/env python3
"""Table of the bench lines of a gpu_steps.sh session, in step order.

  python tools/abtab.py <step> [<step> ...]      (the same step list given to gpu_steps.sh)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dry = subprocess.run(["bash", os.path.join(ROOT, "tools", "gpu_steps.sh")] + sys.argv[1:],
                     env=dict(os.environ, GPU_STEPS_DRY="1"), capture_output=True, text=True,
                     cwd=ROOT).stdout
for spec in dry.splitlines():
    name = spec.split("::")[0]
    path = os.path.join(ROOT, "gpurun_out", name + ".log")
    if not os.path.exists(path):
        print(f"{name:44s} (no log)")
        continue
    lines = [l for l in open(path) if l.startswith("{")]
    if not lines:
        tail = [l.strip() for l in open(path) if "passed" in l or "failed" in l]
        print(f"{name:44s} {tail[-1] if tail else '(no bench line)'}")
        continue
    d = json.loads(lines[-1])
    k = d["kernels"]
    print(f"{name:44s} {d['value']:8.1f} GiB/s  enc {k['encode_ms']:7.3f}  dec {k['decode_ms']:7.3f} ms"
          f"  frac {d['roofline']['frac']:.3f}")
