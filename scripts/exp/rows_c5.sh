#!/bin/bash
# rows-layout parity tests, then config 5 (131,072 envs, A = 16, P = 100) and config 4 with each layout.
set -u
O=gpurun_out/rows_c5; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_step_rows.py "tests/test_gpu_parity.py::test_vs_oracle_rows_layout" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for L in wave rows; do
    for C in 5 4; do
      timeout -k 10 200 python3 bench.py --config $C --step-layout $L --cpu-seconds 0 --fused-k 0 --graph-only --steps 300 --warmup 30 > $O/c${C}_${L}_$rep.json 2> $O/c${C}_${L}_$rep.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 $O/c${C}_${L}_$rep.err; exit $rc; }
      python3 -c "
import json
d=json.loads(open('$O/c${C}_${L}_$rep.json').read().strip().splitlines()[-1])
print('c$C $L $rep', f\"{d['value']:.4e}\", round(d['ms_per_step']*1e3,3), d['config']['step_layout'])"
    done
  done
done
