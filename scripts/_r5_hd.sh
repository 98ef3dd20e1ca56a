# round 5: the per-agent room descriptor read beside the state -- env parity, then same-process A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_episode_gpu.py tests/test_vec_env.py tests/test_monitor_gpu.py tests/test_eval_checkpoint.py tests/test_sharding_gloo.py > gpurun_out/r5h2_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r5h2_tests.log
[ $rc -eq 0 ] || exit $rc
L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
timeout -k 10 600 python3 scripts/ab.py --variants "hd:$L,nohd:$V/libvoxnav_nohd.so" --configs 65536:32x32x8:10:20,65536:32x32x8:10:1,65536:P3_training:10:1,65536:P3_training:10:128,65536:32x32x8:10:128 --steps 640 --rounds 3 > gpurun_out/r5h2_ab.log 2>&1; echo "ab rc=$?"
tail -n 12 gpurun_out/r5h2_ab.log
