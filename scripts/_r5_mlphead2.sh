set -u
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_collector_gpu.py -k "mlp_head" > gpurun_out/r5d_mhtests.log 2>&1
rc=$?; echo "mh tests rc=$rc"; tail -8 gpurun_out/r5d_mhtests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_collector_gpu.py tests/test_eval_checkpoint.py tests/test_ppo.py -k "collector_matches or kernels_match or evaluate or learn_loop" > gpurun_out/r5d_coltests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r5d_coltests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 --learner-minibatches 2"
timeout -k 10 300 $B > gpurun_out/r5d_bench_fused.json 2> gpurun_out/r5d_bench_fused.err; echo "bench rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5d_prof -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 --learner-minibatches 2 --collector mlp > gpurun_out/r5d_prof.log 2>&1; echo "prof rc=$?"
