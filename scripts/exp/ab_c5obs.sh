#!/bin/bash
# Same-box A/B of the general builder k_obs at config 5 (scripts/bench_configs.py --config 5: the
# 4096-env observation chunk), the variants interleaved $REPS times.
set -u
R=$(pwd)
O=$R/gpurun_out/abc5
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 300 python3 $R/scripts/bench_configs.py --config 5 > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${V}_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'c5 step us %.2f' % d['step_us'], 'obs chunk us %.1f' % d['obs_chunk_us'])"
  done
done
