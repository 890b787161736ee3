#!/usr/bin/env python3
"""Per-kernel mean of every counter in a tools/pmc.sh output directory (all passes), with the
kernel-trace duration of the same dispatches.

  python tools/pmc_disp.py gpurun_out/pmc_D_<tag> [--match dcol]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for d in sorted(glob.glob(os.path.join(a.pmc_dir, "*"))):
        kt = {}
        for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
            for r in csv.DictReader(open(f)):
                kt[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        seen = set()
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "qfec" not in name or a.match not in name:
                    continue
                short = (name.replace("void ", "").replace("(anonymous namespace)::", "")
                         .split("(")[0])
                vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (short, r["Dispatch_Id"])
                if key not in seen and r["Dispatch_Id"] in kt:
                    seen.add(key)
                    durs[short].append(kt[r["Dispatch_Id"]])
    for k, d in vals.items():
        print(f"== {k}  (mean duration {sum(durs[k]) / max(1, len(durs[k])):.3f} ms over {len(durs[k])})")
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main()
