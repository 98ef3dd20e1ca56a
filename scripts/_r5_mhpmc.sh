set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 20 --warmup 5 --episode-window 0 --single-step-check 0 --simple 0 --room-sets none --cpu-seconds 0 --learner-minibatches 1 --collector mlp --collector-rollouts 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r5f_mh_p1 -o p1 --output-format csv -- python3 bench.py $B > gpurun_out/r5f_mh_p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/r5f_mh_p2 -o p2 --output-format csv -- python3 bench.py $B > gpurun_out/r5f_mh_p2.log 2>&1; echo "p2 rc=$?"
