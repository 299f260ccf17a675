#!/bin/bash
# Same-box A/B of library variants on the driver's command (bench.py --steps 20 --warmup 5, timed
# region only), a fresh process per run, the variants interleaved $REPS times.
set -u
R=$(pwd)
O=$R/gpurun_out/abdrv
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --fused-k 0 --graph-only \
        > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${V}_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'driver value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step'] * 1e3))"
  done
done
