#!/usr/bin/env python3
"""Print the qfec kernels of a rocprofv3 kernel_stats.csv: calls, mean / min / max (us).

  python tools/kstats.py gpurun_out/prof_<tag>/run_kernel_stats.csv [...]
"""
import csv
import re
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "qfec::" not in n:
            continue
        n = n.replace("(anonymous namespace)::", ""); short = re.sub(r"\(.*$", "", n).replace("void ", "")
        short = short.replace("qfec::(anonymous namespace)::", "").replace("qfec::", "")
        print(f"  {short:60s} calls {int(r['Calls']):4d}  mean {float(r['AverageNs'])/1e3:10.1f}"
              f"  min {float(r['MinNs'])/1e3:10.1f}  max {float(r['MaxNs'])/1e3:10.1f} us")
