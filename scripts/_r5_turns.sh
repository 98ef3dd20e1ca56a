set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_learn_ops.py -k "rows" > gpurun_out/r5t_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r5t_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rows_bench.py 512 > gpurun_out/r5t_rb.log 2>&1 || exit 5
cat gpurun_out/r5t_rb.log | grep -v amdgpu.ids
timeout -k 10 300 python3 scripts/rows_diag.py > gpurun_out/r5t_diag.log 2>&1 || exit 6
grep -v "first CUs\|amdgpu.ids\|pair rel" gpurun_out/r5t_diag.log
