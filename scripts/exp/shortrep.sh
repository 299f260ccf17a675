#!/bin/bash
# The driver's bench command five times on one box (spread of the 20-step figure).
set -u
mkdir -p gpurun_out/shortrep
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/shortrep/$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/shortrep/$i.json').read().strip().splitlines()[-1]);print('$i value %.3e wall %.3f event %.3f' % (d['value'], d['ms_per_step']*1e3, d['gpu_event_ms_per_step']*1e3))"
done
