#!/usr/bin/env python3
"""Per-dispatch PMC values of the qfec kernels matching a pattern, for several pmc.sh runs.

  python tools/pmc_disp_cmp.py <kernel substring> gpurun_out/pmc_D_pmcold_D gpurun_out/pmc_D_pmc_D ...

FETCH_SIZE is printed as read GB (2 x KiB, MI355X_MICROARCH.md correction), WRITE_SIZE as
GB, GRBM_GUI_ACTIVE as M cycles, instruction counts as G.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

pat = sys.argv[1]
for d in sys.argv[2:]:
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for c, v in sorted(vals.items()):
        if c == "FETCH_SIZE":
            s = [2 * x * 1024 / 1e9 for x in v]
            unit = "GB rd"
        elif c == "WRITE_SIZE":
            s = [x * 1024 / 1e9 for x in v]
            unit = "GB wr"
        elif c == "GRBM_GUI_ACTIVE":
            s = [x / 1e6 for x in v]
            unit = "Mcyc"
        else:
            s = [x / 1e9 for x in v]
            unit = "G"
        mean = sum(s) / len(s)
        out.append(f"{c} {unit} mean {mean:.3f} [{min(s):.3f}..{max(s):.3f}] n={len(s)}")
    print(os.path.basename(d))
    for o in out:
        print("   ", o)
