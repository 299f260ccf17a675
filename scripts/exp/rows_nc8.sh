#!/bin/bash
# rows tests (8-chunk cases), then k_step_rows vs k_step at shapes other than the configs':
# P = 100 (eight chunks per lane) and A = 8, at 16,384 and 65,536 envs.
set -u
O=gpurun_out/rows_nc8; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step_rows.py "tests/test_gpu_parity.py::test_vs_oracle_rows_layout" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for S in "--packages 100 --envs 16384" "--packages 100 --envs 65536" "--agents 8 --packages 64 --envs 16384" "--agents 8 --packages 64 --envs 65536"; do
    for L in wave rows; do
      t=$(echo "$S $L $rep" | tr ' -' '__')
      timeout -k 10 200 python3 bench.py $S --step-layout $L --cpu-seconds 0 --fused-k 0 --graph-only --steps 300 --warmup 30 > $O/$t.json 2> $O/$t.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 $O/$t.err; exit $rc; }
      python3 -c "
import json
d=json.loads(open('$O/$t.json').read().strip().splitlines()[-1])
print('$S', '$L', $rep, round(d['ms_per_step']*1e3,3), d['config']['step_layout'])"
    done
  done
done
