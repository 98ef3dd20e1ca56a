# round 5: the collector's vf branch on a second stream -- parity, then same-box A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_collector_gpu.py > gpurun_out/r5v_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/r5v_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 --fuse-check 0 --learner-minibatches 0"
for i in 1 2; do
  VOXNAV_VF_OVERLAP=0 timeout -k 10 300 python3 bench.py $B > gpurun_out/r5v_off_$i.json 2> gpurun_out/r5v_off_$i.err || exit 3
  timeout -k 10 300 python3 bench.py $B > gpurun_out/r5v_on_$i.json 2> gpurun_out/r5v_on_$i.err || exit 4
  python3 - <<PY
import json
for tag in ("off", "on"):
    d = json.loads(open(f"gpurun_out/r5v_{tag}_$i.json").read().strip().splitlines()[-1])
    print(tag, "C4", round(d["collector_lstm"]["value"] / 1e6, 2), "M", d["collector_lstm"]["ms_per_step"], "ms;  C3", round(d["collector_mlp"]["value"] / 1e6, 2), "M", d["collector_mlp"]["ms_per_step"], "ms frac", d["collector_mlp"]["policy_frac_of_mfma_peak"])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5v_prof -o trace --output-format csv -- python3 bench.py $B --collector mlp > gpurun_out/r5v_prof.log 2>&1; echo "prof rc=$?"
