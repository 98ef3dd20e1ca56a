L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
python3 scripts/ab.py --variants "defer:$L,nodefer:$L:VOXNAV_DEFER=0" --configs 65536:P3_training:10:128,65536:P2_training:10:128,65536:P3_training:10:1,65536:100x40x8:10:128 --steps 1024 --rounds 3
