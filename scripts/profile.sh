#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats (headline
# F and the F=1 drop-in call, separately, since both dispatch the same kernel
# symbol), then PMC counters in their own passes (FETCH_SIZE and WRITE_SIZE do
# not fit one TCC pass on gfx950).  Outputs under gpurun_out/<TAG>_*; a fault
# or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BARGS="${BENCH_ARGS:-} --single-step-check 0 --collector none --simple 0 --fuse-check 0 --room-sets none"
# the driver's own window (--steps 20 --warmup 5): the headline launches only
DARGS="--steps 20 --warmup 5 --cpu-seconds 0 --episode-window 0 $BARGS"
TAG=${TAG:-r02}
PASSES=${PASSES:-dtrace,dfetch,dwrite,trace,simple,simple_fetch,simple_write,trace_f1,fetch,write,l2,sq,sqw,tcp}
# the env-only room-set legs (P2 / P3, 1,024 steps after 32 warmup, F=128), one set per run
SARGS="--steps 20 --warmup 5 --cpu-seconds 0 --episode-window 0 --single-step-check 0 --collector none --simple 0 --fuse-check 0 --room-set-steps 1024"
step() {
  local name=$1 t=$2; shift 2
  [[ ",$PASSES," == *",$name,"* ]] || return 0
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -h '"metric"' "gpurun_out/${TAG}_$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step dtrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_dtrace -o trace --output-format csv -- python3 bench.py $DARGS
step dfetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_dfetch -o fetch --output-format csv -- python3 bench.py $DARGS
step dwrite 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_dwrite -o write --output-format csv -- python3 bench.py $DARGS
step trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o trace --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step simple 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_simple -o trace --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 --single-step-check 0 --collector none  --simple 1 --fuse-check 0 --episode-window 0 --room-sets none
step simple_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_simple_fetch -o fetch --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 --single-step-check 0 --collector none  --simple 1 --fuse-check 0 --episode-window 0 --room-sets none
step simple_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_simple_write -o write --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 --single-step-check 0 --collector none  --simple 1 --fuse-check 0 --episode-window 0 --room-sets none
step trace_f1 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace_f1 -o trace --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 $BARGS --fuse 1
step fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o fetch --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o write --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step l2 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_l2 -o l2 --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM -d gpurun_out/${TAG}_sq -o sq --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step sqw 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/${TAG}_sqw -o sqw --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
step tcp 400 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/${TAG}_tcp -o tcp --output-format csv -- python3 bench.py --steps 5408 --warmup 32 --cpu-seconds 0 $BARGS
for SET in P2_training P3_training; do
  step ${SET}_trace 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${SET}_trace -o trace --output-format csv -- python3 bench.py $SARGS --room-sets $SET
  step ${SET}_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_${SET}_fetch -o fetch --output-format csv -- python3 bench.py $SARGS --room-sets $SET
  step ${SET}_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_${SET}_write -o write --output-format csv -- python3 bench.py $SARGS --room-sets $SET
done
exit 0
