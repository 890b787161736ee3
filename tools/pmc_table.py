#!/usr/bin/env python3
"""Per-kernel mean of every counter in a tools/pmc_issue.sh output directory.

  python tools/pmc_table.py gpurun_out/pmci_<tag> [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "qfec::"
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in vals.items():
        print(name[:110])
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
