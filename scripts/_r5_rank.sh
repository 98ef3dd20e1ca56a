set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/ab_same.py --var VOXNAV_ENV_PRIO --values 7,19,35,67,3 --configs 65536:32x32x8:10:20,65536:32x32x8:10:128,65536:P3_training:10:128 --rounds 9 > gpurun_out/r5rk2_ab.log 2>&1; echo ab rc=$?
grep config gpurun_out/r5rk2_ab.log
BEST=$(python3 - <<'PY'
import json
r = [json.loads(l) for l in open("gpurun_out/r5rk2_ab.log") if l.startswith("{")]
score = {}
for d in r:
    if d["config"] == "65536:32x32x8:10:20":
        score[d["VOXNAV_ENV_PRIO"]] = d["paired_ratio_vs_3_median"]
print(max(score, key=score.get))
PY
)
echo "best=$BEST"
: > gpurun_out/r5rk2_wt.log
for v in 3 $BEST; do echo "prio=$v" >> gpurun_out/r5rk2_wt.log; VOXNAV_ENV_PRIO=$v timeout -k 10 200 python3 scripts/env_wt.py --F 20 --warmup 5 >> gpurun_out/r5rk2_wt.log 2>&1 || exit 3; done
grep "prio=\|rank" gpurun_out/r5rk2_wt.log
VOXNAV_ENV_PRIO=$BEST timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5rk2_tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/r5rk2_tests.log
VOXNAV_ENV_PRIO=$BEST timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5rk2_drv.json 2> gpurun_out/r5rk2_drv.err; echo "drv rc=$?"
python3 scripts/_cmp_bench.py gpurun_out/r5rk2_drv.json
