set -u
mkdir -p gpurun_out
L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
timeout -k 10 600 python3 scripts/ab.py --variants "base:$L,slprio1:$V/libvoxnav_slprio1.so,slprio3:$V/libvoxnav_slprio3.so" --configs 65536:32x32x8:4:128:simple,65536:32x32x8:4:20:simple,65536:32x32x8:4:1:simple --steps 1024 --rounds 9 > gpurun_out/r5sl_ab.log 2>&1; echo "ab rc=$?"
grep Gsteps gpurun_out/r5sl_ab.log
