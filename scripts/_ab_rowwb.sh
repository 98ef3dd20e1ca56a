L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
python3 scripts/ab.py --variants "base:$L,rowwb:$V/libvoxnav_rowwb.so" --configs 65536:P3_training:10:128,65536:P2_training:10:128,65536:P3_training:10:1 --steps 1024 --rounds 3
