L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
python3 scripts/ab.py --variants "base:$L,nobyte:$V/libvoxnav_nobyte.so,norowst:$V/libvoxnav_norowst.so,nomark:$V/libvoxnav_nomark.so" --configs 65536:P3_training:10:128,65536:P2_training:10:128 --steps 1024 --rounds 3
