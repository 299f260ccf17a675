#!/bin/bash
# Round 4: the driver's bench command (--steps 20 --warmup 5) with bench.py's setup order as committed
# (B: git stash copy bench_head.py) and as in the tree (both graph captures before the upload replay
# and the warmup), interleaved; plus the 2000-step line of each.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/drvab
mkdir -p $O
run() { timeout -k 10 240 python3 "$@" --cpu-seconds 0 2>>$O/err.log | grep '^{' ; }
for i in 1 2 3 4; do
  run bench.py --steps 20 --warmup 5 > $O/new_$i.json || exit 1
  run scripts/exp/bench_head.py --steps 20 --warmup 5 > $O/head_$i.json || exit 1
done
run bench.py > $O/new_long.json || exit 1
run scripts/exp/bench_head.py > $O/head_long.json || exit 1
for f in $O/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), 'e9', round(d['ms_per_step']*1e3,3), 'us wall', round(d['gpu_event_ms_per_step']*1e3,3), 'us event')"; done
