#!/bin/bash
# Quick GPU iteration: parity tests (all gpu-marked) then a short bench without the CPU leg.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_quick.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > gpurun_out/bench_quick.json 2>/dev/null || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_quick.json').read().strip().splitlines()[-1]);print('api', round(d['ms_per_step']*1e3,3), 'us/step; fused', round(d['fused_bench_mode']['ms_per_step']*1e3,3), 'us/step; value', '%.3e'%d['value'])"
for E in 16384; do
timeout -k 10 200 python bench.py --cpu-seconds 0 --fused-k 0 --envs $E --steps 1000 --warmup 50 > gpurun_out/bench_quick_$E.json 2>/dev/null || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_quick_$E.json').read().strip().splitlines()[-1]);print('E=$E api', round(d['ms_per_step']*1e3,3), 'us/step')"
done
