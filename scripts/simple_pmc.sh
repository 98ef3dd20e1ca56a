#!/bin/bash
# rocprofv3 passes over the simpleEnv step kernels (group = 4 lanes per agent,
# split = stepping + store wave): kernel trace/stats, SQ instruction mix and
# wave states, FETCH/WRITE.  Outputs under gpurun_out/${TAG}_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sp}
V=3d-navigation-reinforcement-learning_amd/voxnav/_lib/libvoxnav.so
for G in 1 0; do
  AB="scripts/ab.py --variants g$G:$V:VOXNAV_SIMPLE_GROUP=$G --configs 65536:32x32x8:4:16:simple --steps 1600 --rounds 1"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_g${G}_trace -o trace --output-format csv -- python3 $AB > gpurun_out/${TAG}_g${G}_trace.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/${TAG}_g${G}_sq -o sq --output-format csv -- python3 $AB > gpurun_out/${TAG}_g${G}_sq.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM -d gpurun_out/${TAG}_g${G}_sqw -o sqw --output-format csv -- python3 $AB > gpurun_out/${TAG}_g${G}_sqw.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_g${G}_fetch -o fetch --output-format csv -- python3 $AB > gpurun_out/${TAG}_g${G}_fetch.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_g${G}_write -o write --output-format csv -- python3 $AB > gpurun_out/${TAG}_g${G}_write.log 2>&1 || exit $?
  echo "G=$G done"; tail -1 gpurun_out/${TAG}_g${G}_trace.log
done
exit 0
