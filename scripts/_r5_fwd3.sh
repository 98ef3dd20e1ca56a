set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_learn_ops.py -k "rows" > gpurun_out/r5f_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/r5f_tests.log | tail -n 25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rows_bench.py 256,512 > gpurun_out/r5f_rb.log 2>&1 || exit 5
grep -v amdgpu.ids gpurun_out/r5f_rb.log
