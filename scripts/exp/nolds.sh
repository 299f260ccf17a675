#!/bin/bash
# Experiment (profiling only): does the step kernel's dynamic LDS request cost
# launch time?  T = 60000 so no env resets inside the run.
set -u
R=$(pwd)
for E in 1024 4096; do
for L in std nolds; do
  if [ $L = std ]; then LP=$R/marl-delivery_amd/marl_gpu/libmdl.so; else LP=$R/marl-delivery_amd/build/ablate/libmdl_nolds.so; fi
  MDL_PROFILING=1 MDL_LIB_PATH=$LP timeout -k 10 120 python bench.py --cpu-seconds 0 --fused-k 0 --T 60000 --envs $E --steps 2000 --warmup 50 > gpurun_out/nolds_${L}_$E.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/nolds_${L}_$E.json').read().strip().splitlines()[-1]);print('$L E=$E', round(d['ms_per_step']*1e3,3), 'us/step')"
done; done
