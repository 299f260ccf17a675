#!/bin/bash
# Same-box A/B of builder variants with scripts/exp/c3_time.py (medians of 15 graph replays of 20
# calls), VARIANTS interleaved REPS times.  main = the in-tree libmdl.so.
set -u
R=$(pwd)
O=$R/gpurun_out/abc3t
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python3 $R/scripts/exp/c3_time.py > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    echo "$V $rep $(cat $O/${V}_$rep.json)"
  done
done
