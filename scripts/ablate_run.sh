#!/bin/bash
# Time bench.py's workload against every ablation build (profiling only).
set -u
R=$(pwd)
mkdir -p gpurun_out
for A in 0 1 2 3 4 8 15; do
  MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$A.so timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > gpurun_out/ablate_$A.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/ablate_$A.json').read().strip().splitlines()[-1]);print('ablate $A', round(d['ms_per_step']*1e3,2), 'us/step', round(d['eager']['ms_per_step']*1e3,2), 'eager', round(d['roofline']['kernel_us_isolated_event_pair'],2),'iso')"
done
