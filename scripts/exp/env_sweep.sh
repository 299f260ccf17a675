#!/bin/bash
# Config-2 step time vs envs per GPU (waves per SIMD): is the step's time the issue of all waves
# (scales with envs) or one wave's dependent chain (flat)?  Lines to gpurun_out/sweep/.
set -u
O=gpurun_out/sweep; mkdir -p $O
for E in 1024 2048 4096 6144 8192; do
  timeout -k 10 120 python3 bench.py --envs $E --cpu-seconds 0 --fused-k 0 --steps 2000 --warmup 200 > $O/e$E.json 2> $O/e$E.err
  rc=$?; echo "envs $E rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/e$E.err; exit $rc; }
done
for E in 1024 2048 4096 6144 8192; do python3 -c "
import json; d=json.loads(open('$O/e$E.json').read().strip().splitlines()[-1])
print($E, round(d['ms_per_step']*1e3,3), 'floor', round(d['launch_floor_ms_per_step']*1e3,3), 'over', round(d['over_floor_us'],3))"; done
