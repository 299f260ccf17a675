#!/bin/bash
# Kernel traces of the driver's bench command (20 steps) and of a long run, for the
# per-dispatch timeline of k_step (durations and gaps) and the round's --stats summary.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_${TAG:-short}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/short -o run --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --graph-only --fused-k 0 > $O/short.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/long -o run --output-format csv -- \
    python3 $R/bench.py --steps 2000 --warmup 20 --cpu-seconds 0 --graph-only --fused-k 0 > $O/long.log 2>&1 || exit $?
find $O -name "*.csv" | sort
