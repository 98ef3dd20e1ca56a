set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_episode_gpu.py tests/test_vec_env.py tests/test_monitor_gpu.py tests/test_collector_gpu.py tests/test_eval_checkpoint.py > gpurun_out/r5q_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/r5q_tests.log
[ $rc -eq 0 ] || exit $rc
L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
timeout -k 10 800 python3 scripts/ab.py --variants "prio:$L,noprio:$V/libvoxnav_noprio.so" --configs 65536:32x32x8:10:20,65536:32x32x8:10:128,65536:32x32x8:10:1,65536:P3_training:10:128,65536:P2_training:10:128,65536:P3_training:10:1 --steps 1024 --rounds 9 > gpurun_out/r5q_ab.log 2>&1; echo "ab rc=$?"
grep Gsteps gpurun_out/r5q_ab.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5q_drv_$i.json 2> gpurun_out/r5q_drv_$i.err; echo "drv $i rc=$?"; python3 scripts/_cmp_bench.py gpurun_out/r5q_drv_$i.json; done
