#!/bin/bash
# Round 4: where the driver's short bench line (--steps 20 --warmup 5) loses against the long run:
# repeated driver-shaped runs, host-wait spin, longer K, and a kernel + HIP-runtime trace of the
# graph-only run (graph launch call vs the first timed kernel, per-dispatch durations and gaps).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/drv
mkdir -p $O
run() { timeout -k 10 240 python3 bench.py "$@" --cpu-seconds 0 --fused-k 0 2>>$O/err.log | grep '^{' ; }
for i in 1 2 3; do run --steps 20 --warmup 5 > $O/k20_$i.json || exit 1; done
for i in 1 2; do run --steps 20 --warmup 5 --host-wait spin > $O/k20spin_$i.json || exit 1; done
run --steps 100 --warmup 5 > $O/k100.json || exit 1
run --steps 400 --warmup 5 > $O/k400.json || exit 1
run --steps 20 --warmup 200 > $O/k20w200.json || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --fused-k 0 --graph-only > $O/trace_bench.log 2>&1 || exit 1
for f in $O/k*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e9,3), 'e9', round(d['ms_per_step']*1e3,3), 'us wall', round(d['gpu_event_ms_per_step']*1e3,3), 'us event')"; done
