#!/bin/bash
# SQ counters for ablation builds 0 (full) and 1 (no shaping)
set -u
export TMPDIR=/tmp
R=$(pwd)
for A in ${VARIANTS:-0 1}; do
  O=$R/gpurun_out/prof_ab$A
  mkdir -p $O
  MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$A.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/sq -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --no-graph --steps 200 --warmup 20 > $O/sq.log 2>&1 || exit $?
done
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
