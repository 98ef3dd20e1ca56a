L=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
python3 scripts/ab.py --variants "base:$L,nopend:$V/libvoxnav_nopend.so,noobs:$V/libvoxnav_noobs.so,nopend_noobs:$V/libvoxnav_nopend_noobs.so,nopstore:$V/libvoxnav_nopstore.so,nomark:$V/libvoxnav_nomark.so,obs0:$V/libvoxnav_obs0.so,obs3:$V/libvoxnav_obs3.so" --configs 65536:P3_training:10:128,65536:P2_training:10:128 --steps 1024 --rounds 3
