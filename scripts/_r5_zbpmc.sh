set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
S="--steps 20 --warmup 5 --cpu-seconds 0 --episode-window 0 --single-step-check 0 --collector none --simple 0 --fuse-check 0 --room-set-steps 512 --room-sets P3_training"
for mode in dm zb; do
  if [ $mode = zb ]; then export VOXNAV_ZBAND=1; else unset VOXNAV_ZBAND; fi
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5h_${mode}_fetch -o fetch --output-format csv -- python3 bench.py $S > gpurun_out/r5h_${mode}_fetch.log 2>&1; echo "$mode fetch rc=$?"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5h_${mode}_write -o write --output-format csv -- python3 bench.py $S > gpurun_out/r5h_${mode}_write.log 2>&1; echo "$mode write rc=$?"
done
