#!/bin/bash
# Same-box A/B of step-kernel variants on BASELINE config 5 (131,072 envs, 64x64, 16 robots) and
# config 2 (the headline): bench.py per variant, interleaved REPS times (us per step, wall).
set -u
R=$(pwd)
O=$R/gpurun_out/abc5
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in ${VARIANTS:-main}; do
    if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
    for C in ${CONFIGS:-5}; do
      MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/bench.py --config $C ${BENCH_EXTRA:-} --steps ${STEPS:-300} --warmup 30 \
          --cpu-seconds 0 --fused-k 0 --no-floor --graph-only > $O/${V}_${C}_$rep.json 2> $O/${V}_${C}_$rep.err || exit $?
      python3 -c "
import json
d = json.loads(open('$O/${V}_${C}_$rep.json').read().strip().splitlines()[-1])
print('$V', 'c$C', $rep, 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'event %.2f' % (d['gpu_event_ms_per_step'] * 1e3))"
    done
  done
done
