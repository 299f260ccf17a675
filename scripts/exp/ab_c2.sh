#!/bin/bash
# Same-box A/B of step builds on config 2 (2000 steps, graph replay) and config 5: main (in-tree) vs VARIANTS.
set -u
R=$(pwd); O=$R/gpurun_out/abc2; mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in main ${VARIANTS}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/bench.py --cpu-seconds 0 --fused-k 0 --no-floor --graph-only \
        --steps 2000 --warmup 200 > $O/${V}_c2_$rep.json 2> $O/${V}_c2_$rep.err || { tail -5 $O/${V}_c2_$rep.err; exit 1; }
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/bench.py --cpu-seconds 0 --fused-k 0 --no-floor --graph-only \
        --config 5 --steps 300 --warmup 30 > $O/${V}_c5_$rep.json 2> $O/${V}_c5_$rep.err || { tail -5 $O/${V}_c5_$rep.err; exit 1; }
    python3 -c "
import json
a = json.loads(open('$O/${V}_c2_$rep.json').read().strip().splitlines()[-1])
b = json.loads(open('$O/${V}_c5_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'c2 %.3f us' % (a['ms_per_step'] * 1e3), 'c5 %.2f us' % (b['ms_per_step'] * 1e3))"
  done
done
