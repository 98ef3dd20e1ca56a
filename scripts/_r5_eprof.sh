set -u
mkdir -p gpurun_out
E="python3 scripts/env_prof.py --lib 3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_eprof.so"
timeout -k 10 200 $E --room P3_training --F 128 --steps 1024 --reps 1 > gpurun_out/r5e_eprof_p3_dm.log 2>&1; echo "dm rc=$?"
VOXNAV_ZBAND=1 timeout -k 10 200 $E --room P3_training --F 128 --steps 1024 --reps 1 > gpurun_out/r5e_eprof_p3_zb.log 2>&1; echo "zb rc=$?"
timeout -k 10 200 $E --room 32x32x8 --F 128 --steps 1024 --reps 1 > gpurun_out/r5e_eprof_box.log 2>&1; echo "box rc=$?"
cat gpurun_out/r5e_eprof_p3_dm.log gpurun_out/r5e_eprof_p3_zb.log gpurun_out/r5e_eprof_box.log | grep -v amdgpu.ids
