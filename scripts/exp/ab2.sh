#!/bin/bash
# Same-box A/B of two builds of libmdl.so (build/ablate/libmdl_A.so, libmdl_B.so):
# bench.py (config 2: graph + fused legs) and bench_configs configs 4 and 5 (step only),
# interleaved three times.  Also runs the GPU parity tests against build B first.
set -u
mkdir -p gpurun_out/ab2
if [ "${TESTS:-1}" = "1" ]; then
  MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_B.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
      -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab2/pytest_B.log 2>&1
  rc=$?; tail -2 gpurun_out/ab2/pytest_B.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2 3; do
  for V in A B; do
    L=marl-delivery_amd/build/ablate/libmdl_$V.so
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --cpu-seconds 0 \
        > gpurun_out/ab2/c2_${V}_$rep.json 2>/dev/null || exit 1
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python scripts/bench_configs.py --config 4 > gpurun_out/ab2/c4_${V}_$rep.json 2>/dev/null || exit 1
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python scripts/bench_configs.py --config 5 > gpurun_out/ab2/c5_${V}_$rep.json 2>/dev/null || exit 1
    python3 - <<EOF
import json
l = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
d = l('gpurun_out/ab2/c2_${V}_$rep.json'); c4 = l('gpurun_out/ab2/c4_${V}_$rep.json'); c5 = l('gpurun_out/ab2/c5_${V}_$rep.json')
print('$V', $rep, 'c2 api %.3f fused %.3f | c4 step %.3f | c5 step %.3f' % (d['ms_per_step']*1e3,
      d['fused_bench_mode']['ms_per_step']*1e3, c4['step_us'], c5['step_us']))
EOF
  done
done
