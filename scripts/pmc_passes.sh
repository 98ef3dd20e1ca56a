#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per pass) on a short bench run.
# Soft-fails a pass that exits with an ordinary error (e.g. counters that do
# not fit one pass); stops on a fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
BARGS=${BENCH_ARGS:-}
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters -d gpurun_out/${TAG}_p$i -o p$i --output-format csv -- python3 bench.py --steps 16 --warmup 4 --cpu-seconds 0 $BARGS > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "[pass $i: $counters] rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done < "${PASSES:-scripts/pmc_passes.txt}"
exit 0
