#!/bin/bash
# Ablation timings at two env counts (profiling only): API path us/step.
set -u
R=$(pwd)
mkdir -p gpurun_out
for A in ${VARIANTS:-0 1 2 4 8 32 64 127}; do
  for E in 4096 16384; do
    MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$A.so timeout -k 10 120 python bench.py --cpu-seconds 0 --fused-k 0 --envs $E --steps 1000 --warmup 50 > gpurun_out/ablate_${A}_$E.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/ablate_${A}_$E.json').read().strip().splitlines()[-1]);print('ablate $A E $E', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
