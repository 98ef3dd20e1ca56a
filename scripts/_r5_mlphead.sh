set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_collector_gpu.py > gpurun_out/r5b_coltests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5b_coltests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="python3 bench.py --steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 --learner-minibatches 2"
timeout -k 10 300 $B > gpurun_out/r5b_bench_fused.json 2> gpurun_out/r5b_bench_fused.err; echo "bench rc=$?"
VOXNAV_MLP_HEAD=0 timeout -k 10 300 $B > gpurun_out/r5b_bench_unfused.json 2> gpurun_out/r5b_bench_unfused.err; echo "bench0 rc=$?"
