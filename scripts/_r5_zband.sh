set -u
mkdir -p gpurun_out
VOXNAV_ZBAND=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_episode_gpu.py tests/test_vec_env.py tests/test_monitor_gpu.py > gpurun_out/r5c_envtests.log 2>&1
rc=$?; echo "envtests rc=$rc"; tail -15 gpurun_out/r5c_envtests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
timeout -k 10 300 python3 scripts/ab.py --variants "zb:$L:VOXNAV_ZBAND=1,dm:$L" --configs 65536:P3_training:10:128,65536:P2_training:10:128,65536:P3_training:10:1 --steps 1024 --rounds 3 > gpurun_out/r5c_ab_zband.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/r5c_ab_zband.log
