L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
python3 scripts/ab.py --variants "nt:$L,plain:$V/libvoxnav_obs0.so,sc1:$V/libvoxnav_obs2.so" --configs 65536:32x32x8:10:1,65536:P3_training:10:1 --steps 512 --rounds 3
