set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5va_auto_$i.log 2>&1 || exit 3
  VOXNAV_ROWS_V2=1 timeout -k 10 200 python3 scripts/ppo_bench.py --agents 65536 --batch 65536 --minibatches 8 --policy lstm > gpurun_out/r5va_v2_$i.log 2>&1 || exit 4
  echo "auto: $(grep -h ms/minibatch gpurun_out/r5va_auto_$i.log)"; echo "v2:   $(grep -h ms/minibatch gpurun_out/r5va_v2_$i.log)"
done
