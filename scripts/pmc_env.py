#!/usr/bin/env python3
"""Per-env-step PMC values of the rollout-buffer env kernel (F steps per
launch, N agents) from rocprofv3 --pmc pass dirs: pmc_env.py 'glob' [F]."""
import collections
import csv
import glob
import sys

pat = sys.argv[1]
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
vals = collections.defaultdict(list)
for f in sorted(glob.glob(pat)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "env_kernel<8, false, true, false" in k:
            n = int(r["Grid_Size"]) // 4
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]) / (n * F))
for k, v in sorted(vals.items()):
    print(f"  {k:28s} n={len(v):3d} per env-step {sum(v) / len(v):10.3f}")
