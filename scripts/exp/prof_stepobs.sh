#!/bin/bash
# rocprofv3 kernel stats of config 3 (bench_configs --config 3: step, builder, and the fused
# k_step_obs) and WRITE_SIZE of k_step_obs.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_stepobs
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3 > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step_obs -d $O/w -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3 > $O/w.log 2>&1 || exit $?
find $O -name "*.csv" | sort
