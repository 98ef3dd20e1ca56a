set -u
mkdir -p gpurun_out
for r in 1 2; do for p in 0 1 2; do echo "prio=$p"; VOXNAV_MH_PRIO=$p timeout -k 10 120 python3 scripts/mlp_head_bench.py --M 65536 --K0 80 --reps 100 2>&1 | grep M=; VOXNAV_MH_PRIO=$p timeout -k 10 120 python3 scripts/mlp_head_bench.py --M 65536 --K0 256 --reps 100 2>&1 | grep M=; done; done
