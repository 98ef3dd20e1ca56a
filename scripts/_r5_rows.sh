# round 5: the two-blocks-per-CU row kernels -- parity, then a same-box A/B of the learner
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_learn_ops.py -k "rows" > gpurun_out/r5r_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 15 gpurun_out/r5r_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  VOXNAV_ROWS_V1=1 timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5r_v1_$i.log 2>&1 || exit 3
  timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5r_v2_$i.log 2>&1 || exit 4
  grep -h "ms/minibatch" gpurun_out/r5r_v1_$i.log gpurun_out/r5r_v2_$i.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5r_learn -o trace --output-format csv -- python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5r_learn.log 2>&1; echo "prof rc=$?"
