# round 5 final tree: smoke, full GPU suite, default + driver-window bench, then the profile passes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f4_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r5f4_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5f4_gputests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r5f4_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r5f4_bench_default.json 2> gpurun_out/r5f4_bench_default.err; echo "bench default rc=$?"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5f4_bench_drv.json 2> gpurun_out/r5f4_bench_drv.err; echo "bench drv rc=$?"
bash scripts/_r5_prof.sh
