#!/usr/bin/env python3
"""HBM bytes per launch of the bench's dominant kernel from the rocprofv3
FETCH_SIZE / WRITE_SIZE passes (scripts/profile.sh), written into
profiles/pmc_traffic.json under the key bench.py looks up
(``{W}x{D}x{H}_L{L}_N{N}_F{F}_W{warmup}_K{steps}``).

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM section: gfx950 tallies the
128-B requests of wide coalesced reads at 64 B); WRITE_SIZE is taken as is.
Both are KB.  Only full F-step launches of the kernel are averaged (the
window's shorter warmup / remainder launches are dropped by size).

usage: traffic_record.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                          --kernel 'env_kernel<8, false, true, false, 2>' --key 32x32x8_L10_N65536_F16_W32_K5408
                          --source '...'  [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import json
from pathlib import Path


def per_dispatch(path, counter, kernel):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel!r} in {path}")
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--env-steps-per-launch", type=int, default=65536 * 16)
    ap.add_argument("--source", default="")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"))
    a = ap.parse_args()
    # the window's short launches (the warmup and the remainder, fewer than F
    # steps) are left out: only dispatches within 25 % of the largest count
    full = lambda v: [x for x in v if x >= 0.75 * max(v)]  # noqa: E731
    f = full(per_dispatch(a.fetch, "FETCH_SIZE", a.kernel))
    w = full(per_dispatch(a.write, "WRITE_SIZE", a.kernel))
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    hbm = int(round((2 * fk + wk) * 1024))
    rec = {"hbm_bytes_per_launch": hbm, "fetch_size_kb_raw": round(fk, 1), "write_size_kb": round(wk, 1),
           "read_bytes_per_env_step": round(2 * fk * 1024 / a.env_steps_per_launch, 1),
           "write_bytes_per_env_step": round(wk * 1024 / a.env_steps_per_launch, 1),
           "env_steps_per_launch": a.env_steps_per_launch, "launches": [len(f), len(w)],
           "source": a.source or f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes: {a.fetch}, {a.write}"}
    out = Path(a.out)
    db = json.loads(out.read_text()) if out.exists() else {}
    db[a.key] = rec
    out.write_text(json.dumps(db, indent=1) + "\n")
    print(a.key, json.dumps(rec))


if __name__ == "__main__":
    main()
