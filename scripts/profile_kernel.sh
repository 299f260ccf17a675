#!/bin/bash
# usage: profile_kernel.sh <kernel-regex> <tag> <python args...>
# kernel trace + stats, then SQ counter pass and FETCH/WRITE passes for one kernel.
set -u
export TMPDIR=/tmp
R=$(pwd)
K=$1; TAG=$2; shift 2
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 "$@" > $O/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d $O/sq -o run --output-format csv -- python3 "$@" > $O/sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/fetch -o run --output-format csv -- python3 "$@" > $O/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/write -o run --output-format csv -- python3 "$@" > $O/write.log 2>&1 || exit $?
