#!/bin/bash
# GPU suite + config-2 / config-4 bench lines on the current build (rows layout adopted above 10,240 envs).
set -u
O=gpurun_out/rows_check; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python3 -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $O/suite.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/suite.log | head -20; exit $rc; }
timeout -k 10 200 python3 bench.py --config 4 --cpu-seconds 2 --fused-k 0 --steps 300 --warmup 30 > $O/c4.json 2> $O/c4.err; echo "c4 rc=$?"
timeout -k 10 200 python3 bench.py --cpu-seconds 2 --steps 2000 --warmup 200 > $O/c2.json 2> $O/c2.err; echo "c2 rc=$?"
for f in $O/c4.json $O/c2.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', f\"{d['value']:.4e}\", round(d['ms_per_step']*1e3,3), 'floor', d.get('launch_floor_ms_per_step'), d['config']['step_layout'], d['roofline']['kernel'], d['roofline']['frac'])"; done
