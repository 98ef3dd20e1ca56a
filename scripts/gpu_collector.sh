#!/bin/bash
# Collector legs of bench.py (f32 / bf16 PPO-LSTM on P3_training, PPO-MLP on
# P2_training) and a rocprofv3 kernel-trace summary of the f32 PPO-LSTM leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-coll}
COMMON="--learner-batch 0 --simple 0 --episode-window 0 --fuse-check 0 --single-step-check 0 --cpu-seconds 0 --steps 16 --warmup 4"
timeout -k 10 300 python bench.py --collector lstm,mlp --collector-bf16 1 $COMMON > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python - "$TAG" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}_bench.json").read().strip().splitlines()[-1])
for k in ("collector_lstm", "collector_lstm_bf16", "collector_mlp"):
    print(k, d[k]["value"], d[k]["ms_per_step"], d[k]["policy_frac_of_mfma_peak"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o c --output-format csv -- python3 bench.py --collector lstm --collector-bf16 0 $COMMON > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/{sys.argv[1]}_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Percentage"])
PY
