#!/usr/bin/env python3
"""Average per-dispatch PMC values of one kernel across rocprofv3 pass dirs."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
tag = sys.argv[2] if len(sys.argv) > 2 else "pmc"
pat = sys.argv[3] if len(sys.argv) > 3 else "env_kernel"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/{tag}_p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"] and "true" not in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:40s} n={len(v):3d} avg={sum(v)/len(v):16.1f}")
