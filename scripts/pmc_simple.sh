#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per pass) over the simpleEnv bench
# instantiation alone: 65,536 agents, 32x32x8, L=4, 128-step launches.
# LIB / CFG / STEPS select the library and the ab.py config.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-psimple}
LIB=${LIB:-3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so}
CFG=${CFG:-65536:32x32x8:4:128:simple}
STEPS=${STEPS:-1024}
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $counters -d gpurun_out/${TAG}_p$i -o p$i --output-format csv -- python3 scripts/ab.py --variants base:$LIB --configs $CFG --steps $STEPS --rounds 1 > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "[pass $i: $counters] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done < "${PASSES:-scripts/pmc_passes_sq.txt}"
exit 0
