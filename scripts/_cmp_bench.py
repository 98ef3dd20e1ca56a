#!/usr/bin/env python3
"""Print the headline and collector / learner legs of bench JSON lines, and
the top kernels of rocprofv3 kernel_stats CSVs (diagnostics helper)."""
import csv
import json
import sys

for f in sys.argv[1:]:
    if f.endswith(".csv"):
        for r in list(csv.DictReader(open(f)))[:8]:
            print(f"  {r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):6.2f} %")
        continue
    s = open(f).read()
    i = s.find('{"metric"')
    d = json.loads(s[i:].splitlines()[0])
    print(f, d["value"], d["roofline"]["frac"])
    for k in ("collector_lstm", "collector_mlp"):
        c = d.get(k)
        if c:
            print(f"  {k}: {c['value'] / 1e6:.1f} M/s  {c['ms_per_step']} ms/step  policy frac {c['policy_frac_of_mfma_peak']}"
                  f"  learner {c['learner']['value'] / 1e6:.2f} M/s ({c['learner']['frac_of_f32_mfma_peak']})")
