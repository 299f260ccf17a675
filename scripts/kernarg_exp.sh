#!/bin/bash
set -u
R=$(pwd)
for KA in 0 1; do
  for A in 0 15; do
    HIP_FORCE_DEV_KERNARG=$KA MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$A.so timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > gpurun_out/ka_${KA}_$A.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/ka_${KA}_$A.json').read().strip().splitlines()[-1]);print('kernarg=$KA ablate=$A', round(d['ms_per_step']*1e3,2), 'us/step graph', round(d['eager']['ms_per_step']*1e3,2), 'eager')"
  done
done
