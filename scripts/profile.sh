#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then PMC
# counters in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one
# TCC pass on gfx950).  Outputs under gpurun_out/prof_*; a fault or timeout
# ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BARGS=${BENCH_ARGS:-}
TAG=${TAG:-r01}
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step prof_list 120 rocprofv3 -L
step prof_trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace_$TAG -o trace --output-format csv -- python3 bench.py --steps 400 --warmup 40 --cpu-seconds 0 $BARGS
step prof_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch_$TAG -o fetch --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 $BARGS
step prof_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write_$TAG -o write --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 $BARGS
step prof_l2 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_l2_$TAG -o l2 --output-format csv -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 $BARGS
exit 0
