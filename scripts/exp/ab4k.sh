#!/bin/bash
# Same-box A/B at 4096 envs only (graph + fused), three reps.
set -u
mkdir -p gpurun_out/ab4k
for rep in 1 2 3; do
  for V in A B; do
    MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_$V.so timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --cpu-seconds 0 > gpurun_out/ab4k/${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab4k/${V}_$rep.json').read().strip().splitlines()[-1]); print('$V', $rep, round(d['ms_per_step']*1e3,3), round(d['fused_bench_mode']['ms_per_step']*1e3,3))"
  done
done
