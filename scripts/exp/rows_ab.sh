#!/bin/bash
# Four-envs-per-wavefront step (k_step_rows) check + A/B against one env per wavefront (k_step):
# the rows-vs-wave parity tests, the whole GPU suite, then interleaved bench legs per layout.
# SKIP_SUITE=1 skips the suite.  Outputs under gpurun_out/rows/.
set -u
O=gpurun_out/rows; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_step_rows.py > $O/rows_tests.log 2>&1
rc=$?; echo "rows_tests rc=$rc"; tail -3 $O/rows_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/rows_tests.log | head -20; exit $rc; }
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  timeout -k 10 600 python3 -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -2 $O/suite.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/suite.log | head -20; exit $rc; }
fi
B="--cpu-seconds 0 --fused-k 0"
for rep in 1; do
  for L in wave rows; do
    timeout -k 10 120 python3 bench.py $B --step-layout $L --steps 2000 --warmup 200 > $O/c2_${L}_$rep.json 2> $O/c2_${L}_$rep.err
    rc=$?; echo "c2 $L $rep rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c2_${L}_$rep.err; exit $rc; }
    timeout -k 10 120 python3 bench.py $B --step-layout $L --config 4 --steps 300 --warmup 20 > $O/c4_${L}_$rep.json 2> $O/c4_${L}_$rep.err
    rc=$?; echo "c4 $L $rep rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c4_${L}_$rep.err; exit $rc; }
  done
done
for E in 1024 2048 8192 16384; do
  timeout -k 10 120 python3 bench.py $B --envs $E --steps 2000 --warmup 200 > $O/sweep_$E.json 2> $O/sweep_$E.err
  rc=$?; echo "sweep $E rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/sweep_$E.err; exit $rc; }
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err; echo "driver rc=$?"
for f in $O/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f'.split('/')[-1], f\"{d['value']:.4e}\", round(d['ms_per_step']*1e3,3), 'floor', d.get('launch_floor_ms_per_step') and round(d['launch_floor_ms_per_step']*1e3,3), 'over', d.get('over_floor_us') and round(d['over_floor_us'],3), d['config'].get('step_layout'))"; done
