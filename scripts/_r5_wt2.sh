set -u
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/env_wt.py --F 20 --warmup 5 > gpurun_out/r5wt2.log 2>&1; echo rc=$?
timeout -k 10 200 python3 scripts/env_wt.py --F 128 --warmup 32 >> gpurun_out/r5wt2.log 2>&1; echo rc=$?
timeout -k 10 200 python3 scripts/env_wt.py --F 1 --warmup 5 >> gpurun_out/r5wt2.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/r5wt2.log
