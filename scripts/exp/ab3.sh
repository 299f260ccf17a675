#!/bin/bash
# Same-box A/B (builds A, B): config 2 at 1024 / 2048 / 4096 envs (graph + fused), configs 4 and 5,
# after the GPU parity tests against build B.
set -u
mkdir -p gpurun_out/ab3
if [ "${TESTS:-1}" = "1" ]; then
  MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_B.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ab3/pytest_B.log 2>&1
  rc=$?; tail -2 gpurun_out/ab3/pytest_B.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for V in A B; do
    L=marl-delivery_amd/build/ablate/libmdl_$V.so
    line="$V $rep"
    for E in 1024 2048 4096; do
      MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python bench.py --envs $E --steps 2000 --warmup 100 --cpu-seconds 0 \
          > gpurun_out/ab3/c2_${V}_${E}_$rep.json 2>/dev/null || exit 1
      line="$line | E$E $(python3 -c "import json; d=json.loads(open('gpurun_out/ab3/c2_${V}_${E}_$rep.json').read().strip().splitlines()[-1]); print('%.3f/%.3f' % (d['ms_per_step']*1e3, d['fused_bench_mode']['ms_per_step']*1e3))")"
    done
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python scripts/bench_configs.py --config 4,5 > gpurun_out/ab3/c45_${V}_$rep.json 2>/dev/null || exit 1
    line="$line | $(python3 -c "import json; ls=[json.loads(l) for l in open('gpurun_out/ab3/c45_${V}_$rep.json') if l.startswith('{')]; print(' '.join('c%s %.3f' % (d['config'], d['step_us']) for d in ls))")"
    echo "$line"
  done
done
