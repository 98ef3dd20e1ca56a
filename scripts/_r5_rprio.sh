set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_learn_ops.py tests/test_ppo.py > gpurun_out/r5rp_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/r5rp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rows_bench.py 512 > gpurun_out/r5rp_rb.log 2>&1 || exit 5
grep -v amdgpu.ids gpurun_out/r5rp_rb.log
for i in 1 2; do
  VOXNAV_ROWS_PRIO=0 timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5rp_off_$i.log 2>&1 || exit 3
  timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5rp_on_$i.log 2>&1 || exit 4
  grep -h "ms/minibatch" gpurun_out/r5rp_off_$i.log gpurun_out/r5rp_on_$i.log
done
