#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof
mkdir -p $O
BENCH="$R/bench.py --cpu-seconds 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $BENCH --steps ${STEPS:-2000} --warmup 100 > $O/trace_bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/pmc_fetch -o run --output-format csv -- python3 $BENCH --no-graph --steps 300 --warmup 20 > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/pmc_write -o run --output-format csv -- python3 $BENCH --no-graph --steps 300 --warmup 20 > $O/pmc_write.log 2>&1 || exit $?
find $O -name "*.csv" | head -50
