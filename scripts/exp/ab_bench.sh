#!/bin/bash
# Same-box A/B of step-kernel variants (scripts/ab_build.sh): bench.py config 2 (or $CONFIG),
# 2000 graph-replayed steps, the variants interleaved $REPS times; prints us per step.
# VARIANTS: names under marl-delivery_amd/build/ab/ ("main" = marl_gpu/libmdl.so).
set -u
R=$(pwd)
O=$R/gpurun_out/ab
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python3 $R/bench.py --config ${CONFIG:-2} ${BENCH_EXTRA:-} --cpu-seconds 0 --fused-k 0 --graph-only \
        --steps ${STEPS:-2000} --warmup 100 > $O/${V}_$rep.json 2> $O/${V}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${V}_$rep.json').read().strip().splitlines()[-1])
print('$V', $rep, 'us/step %.3f' % (d['ms_per_step'] * 1e3), 'event %.3f' % (d['gpu_event_ms_per_step'] * 1e3))"
  done
done
