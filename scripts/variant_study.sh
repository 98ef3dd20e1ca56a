#!/bin/bash
# Variant study (diagnostics builds under _lib/variants): interleaved A/B of
# whole builds (scripts/ab.py), a paired runtime-switch A/B on one allocation
# (scripts/ab_same.py) and per-variant FETCH / WRITE passes over one env
# window (scripts/env_window.py).  Every step has its own time limit; a
# fault / abort / timeout ends the script.  Parameters (environment):
#   TAG          output prefix under gpurun_out/
#   AB_VARIANTS  name:lib.so[:ENV=V],...      AB_CONFIGS  N:room:L:F,...
#   SAME_LIB     lib for ab_same               SAME_VAR / SAME_VALUES / SAME_CONFIGS
#   PMC_VARIANTS name:lib.so,...               PMC_WINDOW  env_window.py args
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-vs}
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -h '^{' "gpurun_out/${TAG}_$name.log" | cut -c1-220
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/${TAG}_$name.log"; exit $rc; fi
}
if [ -n "${AB_VARIANTS:-}" ]; then
  step ab 900 python3 scripts/ab.py --variants "$AB_VARIANTS" --configs "${AB_CONFIGS:-65536:32x32x8:10:20}" \
    --steps "${AB_STEPS:-256}" --rounds "${AB_ROUNDS:-5}"
fi
if [ -n "${SAME_VAR:-}" ]; then
  step same 900 env ${SAME_LIB:+VOXNAV_LIB=$SAME_LIB} python3 scripts/ab_same.py --var "$SAME_VAR" \
    --values "${SAME_VALUES:-1,0}" --configs "${SAME_CONFIGS:-65536:32x32x8:10:20}" --rounds "${SAME_ROUNDS:-9}"
fi
for item in $(echo "${PMC_VARIANTS:-}" | tr ',' ' '); do
  name=${item%%:*}; lib=${item#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    step "pmc_${name}_$c" 300 rocprofv3 --pmc $c -d "gpurun_out/${TAG}_pmc_${name}_$c" -o pmc --output-format csv \
      -- python3 scripts/env_window.py --lib "$lib" ${PMC_WINDOW:---room P3_training --F 128 --warmup 32 --steps 1024}
  done
done
exit 0
