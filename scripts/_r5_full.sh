set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r5z_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5z_gputests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/r5z_gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r5z_bench_default.json 2> gpurun_out/r5z_bench_default.err; echo "bench default rc=$?"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5z_bench_drv.json 2> gpurun_out/r5z_bench_drv.err; echo "bench drv rc=$?"
