#!/bin/bash
# Early whole-slab zero fill A/B (MDL_OBS_EARLYFILL 0 / 1 / 3): GPU parity suite on
# the in-tree build, then configs 3 and 3b per variant, interleaved twice.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for V in 0 1 3; do
    for C in 3 3b; do
      MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_ef$V.so timeout -k 10 200 python3 scripts/bench_configs.py --config $C > gpurun_out/ef_${V}_${C}_$rep.json || exit 1
      echo "ef$V $C rep$rep: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ef_${V}_${C}_$rep.json').read().strip().splitlines()[-1]); print({k:v for k,v in d.items() if 'us' in k or 'obs' in k})")"
    done
  done
done
