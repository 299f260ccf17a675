#!/bin/bash
# Full-size PMC passes for the config-4 (65,536 mixed-map envs) and config-5 (131,072 envs) bench launches,
# so bench.py's roofline.traffic has a record of the exact launch it times (profile_r05.sh measured a
# 16,384-env config-5 slice).  Outputs under gpurun_out/prof_r05/{c4,c5full}/{fetch,write};
# scripts/collect_profiles_r05.py picks them up.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_r05
mkdir -p $O
pmc() {   # dir log counter rx -- bench args
  local d=$1 lg=$2 c=$3 rx=$4; shift 4
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$rx" -d $O/$d -o run --output-format csv -- python3 $R/bench.py "$@" > $O/$lg.log 2>&1
  local rc=$?; echo "pmc $d rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/$lg.log; exit $rc; }; return 0
}
E="--cpu-seconds 0 --no-graph --graph-only --fused-k 0 --no-floor --steps 100 --warmup 10"
for k in fetch write; do
  case $k in fetch) C=FETCH_SIZE ;; write) C=WRITE_SIZE ;; esac
  pmc c4/$k c4_$k $C "k_step_rows" $E --config 4   # config 4 runs four envs per wavefront (k_step_rows)
  pmc c5full/$k c5full_$k $C "k_step[<(]" $E --config 5
done
