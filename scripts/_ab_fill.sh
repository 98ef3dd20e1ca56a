L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
python3 scripts/ab.py --variants "new:$L,prev:$V/libvoxnav_prev.so" --configs 65536:32x32x8:10:1,65536:P3_training:10:1,65536:32x32x8:10:128,65536:P3_training:10:128,65536:32x32x8:10:20 --steps 1024 --rounds 3
