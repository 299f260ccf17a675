#!/bin/bash
# SQ counter passes on k_obs over scripts/exp/obs_parts.py (5 output subsets x 23
# launches each, in order); summarised per subset by scripts/obs_pmc_parts.py.
set -u
export TMPDIR=/tmp
R=$(pwd)
TAG=${TAG:-obs}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
C="$R/scripts/exp/obs_parts.py"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_obs -d $O/sq -o run --output-format csv -- python3 $C > $O/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex k_obs -d $O/sq2 -o run --output-format csv -- python3 $C > $O/sq2.log 2>&1 || exit $?
python3 scripts/obs_pmc_parts.py $O > $O/parts.json
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_obs -d $O/write -o run --output-format csv -- python3 $C > $O/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_obs -d $O/fetch -o run --output-format csv -- python3 $C > $O/fetch.log 2>&1 || exit $?
python3 scripts/obs_pmc_parts.py $O > $O/parts.json
