set -u
mkdir -p gpurun_out
E="python3 scripts/env_prof.py --lib 3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_eprof.so"
timeout -k 10 200 $E --room 32x32x8 --F 20 --warmup 5 --reps 3 > gpurun_out/r5wt_drv.log 2>&1; echo "drv rc=$?"
timeout -k 10 200 $E --room 32x32x8 --F 128 --steps 1024 > gpurun_out/r5wt_f128.log 2>&1; echo "f128 rc=$?"
timeout -k 10 200 $E --room 32x32x8 --F 1 --steps 64 > gpurun_out/r5wt_f1.log 2>&1; echo "f1 rc=$?"
cat gpurun_out/r5wt_drv.log gpurun_out/r5wt_f128.log gpurun_out/r5wt_f1.log | grep -v amdgpu.ids
