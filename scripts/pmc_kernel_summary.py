#!/usr/bin/env python3
"""Average per-dispatch PMC values of dispatches whose kernel name contains
PATTERN (exact substring, 'true'/'false' allowed) across rocprofv3 pass dirs:
pmc_kernel_summary.py TAG 'env_kernel<16, false, true, false, 0>' [root]"""
import collections
import csv
import glob
import sys

tag, pat = sys.argv[1], sys.argv[2]
root = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/{tag}_p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:40s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
