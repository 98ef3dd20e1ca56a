# round 5: row kernels -- parity of both layouts + the default pick, microbench, learner A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_learn_ops.py -k "rows" > gpurun_out/r5s_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/r5s_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rows_bench.py 256,512 > gpurun_out/r5s_rb.log 2>&1 || exit 5
cat gpurun_out/r5s_rb.log
for i in 1 2; do
  VOXNAV_ROWS_V1=1 timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5s_v1_$i.log 2>&1 || exit 3
  timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5s_auto_$i.log 2>&1 || exit 4
  grep -h "ms/minibatch" gpurun_out/r5s_v1_$i.log gpurun_out/r5s_auto_$i.log
done
