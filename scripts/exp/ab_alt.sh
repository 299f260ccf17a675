#!/bin/bash
# Same-box A/B of library variants on the IDQ/qmix featurizers (bench_configs.py --config alt).
set -u
R=$(pwd)
O=$R/gpurun_out/abalt
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python3 $R/scripts/bench_configs.py --config alt > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${V}_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'alt us %.2f' % d['us_per_call'], 'TB/s %.2f' % (d['write_bytes'] / d['us_per_call'] / 1e6))"
  done
done
