#!/bin/bash
# Same-box A/B of observation-builder variants (scripts/ab_build.sh): scripts/bench_configs.py
# --config ${CONFIG:-3b}, the variants interleaved $REPS times; prints the builder's us per call.
set -u
R=$(pwd)
O=$R/gpurun_out/abobs
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/scripts/bench_configs.py --config ${CONFIG:-3b} --steps 100 --warmup 10 \
        > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${V}_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'obs us %.1f' % d['obs_us'], 'TB/s %.2f' % (d['obs_roofline']['achieved_GBs'] / 1e3), 'step_obs us %.1f' % d['step_obs_fused_us'])"
  done
done
