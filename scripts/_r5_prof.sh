set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05h PASSES=dtrace,dfetch,dwrite,trace_f1,P2_training_trace,P2_training_fetch,P2_training_write,P3_training_trace,P3_training_fetch,P3_training_write bash scripts/profile.sh; rc=$?; echo "profile rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_collect -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 > gpurun_out/r05h_collect.log 2>&1; echo "collect rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_learn_lstm -o trace --output-format csv -- python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r05h_learn_lstm.log 2>&1; echo "learn rc=$?"
