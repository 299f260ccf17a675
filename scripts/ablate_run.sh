#!/bin/bash
# Time bench.py's workload against every ablation build (profiling only):
# API path (graph replay, us/step) and fused bench mode (us/step).
set -u
R=$(pwd)
mkdir -p gpurun_out
for A in ${VARIANTS:-0 1 2 3 4 8 15}; do
  MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$A.so timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 1000 --warmup 100 > gpurun_out/ablate_$A.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/ablate_$A.json').read().strip().splitlines()[-1]);print('ablate $A', round(d['ms_per_step']*1e3,2), 'us/step api', round(d['fused_bench_mode']['ms_per_step']*1e3,2), 'us/step fused')"
done
