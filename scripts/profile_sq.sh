#!/bin/bash
# SQ counter pass on the step kernel (one pass, 8 SQ slots) + clock counter pass.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_sq
mkdir -p $O
BENCH="$R/bench.py --cpu-seconds 0 --no-graph --steps 200 --warmup 20"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/sq -o run --output-format csv -- python3 $BENCH > $O/sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex k_step -d $O/sq2 -o run --output-format csv -- python3 $BENCH > $O/sq2.log 2>&1 || exit $?
