#!/usr/bin/env python3
"""Per-launch averages of every PMC counter of one kernel over rocprofv3
counter_collection CSVs:  pmc_table.py <kernel substring> <csv> [<csv> ...]
(also per wave-step when --wave-steps is given)."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("kernel")
ap.add_argument("csvs", nargs="+")
ap.add_argument("--wave-steps", type=float, default=0.0, help="wave-steps per launch (waves x steps)")
a = ap.parse_args()
vals = collections.defaultdict(list)
for f in a.csvs:
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    avg = sum(v) / len(v)
    extra = f"  per wave-step {avg / a.wave_steps:10.2f}" if a.wave_steps else ""
    print(f"{k:28s} n={len(v):4d} avg/launch {avg:16.1f}{extra}")
