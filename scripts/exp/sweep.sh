#!/bin/bash
# Launch-floor probes + step kernel time vs envs per GPU (profiling only).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/floor.py > gpurun_out/floor.json 2> gpurun_out/floor.err || exit $?
for E in 1024 2048 4096 8192 16384; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 500 --warmup 50 --envs $E > gpurun_out/sweep_$E.json 2>/dev/null || exit $?
done
cat gpurun_out/floor.json
for E in 1024 2048 4096 8192 16384; do python -c "import json;d=json.load(open('gpurun_out/sweep_$E.json'));print($E, d['roofline']['kernel_us'])"; done
