#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into a per-kernel HBM traffic table.

  python tools/pmc_summary.py gpurun_out/pmc_A_r01 profiles/r01/pmc_A.json --groups 65536

Correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE
(KiB) reports half the bytes of a wide coalesced streaming read (16 B per lane,
global_load and LDS-DMA alike), so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE reads
16-byte-per-lane streaming stores exactly.  The XOR kernel's 8-byte stores are checked
against their known byte count in DESIGN.md (WRITE_SIZE within 5 % of the algorithmic
write bytes).  Values are per launch (mean over the profiled dispatches of that kernel).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out_json")
    ap.add_argument("--groups", type=int, required=True, help="groups per launch profiled")
    ap.add_argument("--workload", default="")
    args = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(args.pmc_dir, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not name.startswith("void qfec::") and not name.startswith("qfec::"):
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"workload": args.workload, "groups": args.groups, "kernels": {}}
    for name, d in vals.items():
        mean = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"dispatches": max(len(v) for v in d.values())}
        e.update({c: round(v, 1) for c, v in mean.items()})
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            rd = 2.0 * mean["FETCH_SIZE"] * 1024
            wr = mean["WRITE_SIZE"] * 1024
            e["read_bytes"] = round(rd)
            e["write_bytes"] = round(wr)
            e["traffic_bytes"] = round(rd + wr)
        out["kernels"][name] = e
    os.makedirs(os.path.dirname(os.path.abspath(args.out_json)), exist_ok=True)
    with open(args.out_json, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for name, e in out["kernels"].items():
        print(f"{name[:70]:70s} traffic/launch = {e.get('traffic_bytes')}")


if __name__ == "__main__":
    main()
