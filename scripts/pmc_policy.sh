#!/bin/bash
# rocprofv3 kernel trace + PMC passes (one run per pass) of the f32 policy
# kernels alone (scripts/policy_f32_prof.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pf32}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o t --output-format csv -- python3 scripts/policy_f32_prof.py 10 $@ > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; echo "[trace] rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters -d gpurun_out/${TAG}_p$i -o p$i --output-format csv -- python3 scripts/policy_f32_prof.py 5 $@ > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "[pass $i: $counters] rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done < "${PASSES:-scripts/pmc_passes_mfma.txt}"
exit 0
