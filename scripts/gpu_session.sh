#!/bin/bash
# One GPU session of named steps (STEPS=a,b,...), each under its own time
# limit; a fault / abort / timeout ends the session (a test failure, exit 1,
# does not).  Logs under gpurun_out/<TAG>_<step>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s}
run() {
  local name=$1 t=$2; shift 2
  [[ ",$STEPS," == *",$name,"* ]] || return 0
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc ($(( $(date +%s) - t0 )) s)"
  tail -n 12 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
EPROF="python3 scripts/env_prof.py --lib 3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_eprof.so"
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run ltests 600 python3 -u -m pytest tests/test_learn_ops.py tests/test_ppo.py -m gpu -x -q --timeout 300 --timeout-method thread
run tests 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
run counters 120 rocprofv3 -L
run placement 900 python3 scripts/placement_probe.py ${PLACE_ARGS:-}
run bench_drv 300 python3 bench.py --steps 20 --warmup 5 --json-out gpurun_out/${TAG}_bench_drv.json
run eprof_p3 300 $EPROF --room P3_training --F 128 --steps 1024 --reps 1
run eprof_p3f1 300 $EPROF --room P3_training --F 1 --steps 200 --reps 1
run eprof_p2 300 $EPROF --room P2_training --F 128 --steps 1024 --reps 1
run eprof_box 300 $EPROF --room 32x32x8 --F 20 --warmup 5 --reps 5
run eprof_boxf1 300 $EPROF --room 32x32x8 --F 1 --steps 200 --reps 1
run learn_lstm 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_learn_lstm -o trace --output-format csv -- python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm
run learn_mlp 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_learn_mlp -o trace --output-format csv -- python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy mlp
# paired / same-allocation A/B: AB_ARGS / AB_SAME_ARGS hold the variants and configs
run ab 900 python3 scripts/ab.py ${AB_ARGS:-}
run ab_same 900 python3 scripts/ab_same.py ${AB_SAME_ARGS:-}
# the end-of-round profile passes (kernel traces, FETCH / WRITE of the driver window and the P-set legs)
run final_prof 1500 env TAG=${TAG}_fp PASSES=${FPASSES:-dtrace,dfetch,dwrite,trace_f1,P2_training_trace,P2_training_fetch,P2_training_write,P3_training_trace,P3_training_fetch,P3_training_write} bash scripts/profile.sh
run collect_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_collect -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0
run sq_p3 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/${TAG}_sq_p3 -o sq --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --single-step-check 0 --collector none --simple 0 --fuse-check 0 --episode-window 0 --room-sets P3_training --room-set-steps 256
run learn_lstm_gk16 300 env VOXNAV_LIB=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_gk16.so python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm
run learn_mlp_gk16 300 env VOXNAV_LIB=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_gk16.so python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy mlp
run gemm 200 python3 scripts/gemm_bench.py 20
run gemm_k32 200 env VN_GEMM_GKD=32 python3 scripts/gemm_bench.py 20
run learn_mlp_k32 300 env VN_GEMM_GKD=32 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy mlp
run learn_mlp_plain 300 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy mlp
run gemm_gk16 200 env VOXNAV_LIB=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_gk16.so python3 scripts/gemm_bench.py 20
run gemm_pmc 300 env TAG=${TAG}_gpmc bash scripts/pmc_run.sh scripts/gemm_bench.py 3
run learn_pmc 400 env TAG=${TAG}_lpmc bash scripts/pmc_run.sh scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 4 --policy lstm
run prof 1000 env TAG=${TAG}_p PASSES=${PPASSES:-dtrace,dfetch,dwrite,trace_f1} bash scripts/profile.sh
run ddp2 600 env VOXNAV_BENCH_SHARED_DEVICE=1 python3 bench.py --gpus 2 --steps 256 --warmup 32 --agents 16384 --cpu-seconds 0 --simple 0 --room-sets none
run bench 600 python3 bench.py ${BENCH_ARGS:-}
exit 0
