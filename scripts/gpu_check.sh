#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench.  Each step has its own
# time limit; a fault / abort / timeout ends the session (test failures,
# exit 1, do not).  Logs go to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc ($(( $(date +%s) - t0 )) s)"
  tail -n 5 "gpurun_out/$name.log"
  return $rc
}
soft() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
STEPS=${STEPS:-smoke,tests,bench}
if [[ $STEPS == *smoke* ]]; then run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; soft $rc || exit $rc; fi
if [[ $STEPS == *tests* ]]; then run pytest_gpu 1100 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-}; rc=$?; soft $rc || exit $rc; fi
if [[ $STEPS == *bench* ]]; then run bench 600 python bench.py ${BENCH_ARGS:-}; rc=$?; soft $rc || exit $rc; fi
exit 0
