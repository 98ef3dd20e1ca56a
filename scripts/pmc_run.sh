#!/bin/bash
# PMC passes (one rocprofv3 run per line of $PASSES) over one python script:
#   TAG=x PASSES=scripts/pmc_passes_mfma.txt bash scripts/pmc_run.sh scripts/gemm_bench.py 5
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters -d gpurun_out/${TAG}_p$i -o p$i --output-format csv -- python3 "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "[pass $i: $counters] rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done < "${PASSES:-scripts/pmc_passes_mfma.txt}"
exit 0
