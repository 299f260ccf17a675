#!/bin/bash
# rocprofv3 kernel trace + stats of the config-4 and config-5 step slices
# (scripts/bench_configs.py --config 4 / 5); summaries under gpurun_out/prof_<tag>_c4 / _c5.
set -u
export TMPDIR=/tmp
R=$(pwd)
TAG=${TAG:-round}
for C in 4 5; do
  O=$R/gpurun_out/prof_${TAG}_c$C
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config $C > $O/trace.log 2>&1 || exit $?
  tail -1 $O/trace.log
done
