set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
timeout -k 10 800 python3 scripts/ab.py --variants "base:$L,prio2:$V/libvoxnav_prio2.so,prio3f:$V/libvoxnav_prio3f.so,prio2f:$V/libvoxnav_prio2f.so" --configs 65536:32x32x8:10:20,65536:32x32x8:10:128,65536:P3_training:10:128,65536:P2_training:10:128 --steps 1024 --rounds 11 > gpurun_out/r5p3_ab.log 2>&1; echo "ab rc=$?"
grep Gsteps gpurun_out/r5p3_ab.log
