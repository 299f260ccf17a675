#!/bin/bash
# Same-box A/B of the observation builder (configs 3 and 3b) between build A and build B.
set -u
mkdir -p gpurun_out/obsab
for rep in 1 2; do
  for V in A B; do
    for C in 3 3b; do
      MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_$V.so timeout -k 10 200 python scripts/bench_configs.py --config $C \
          > gpurun_out/obsab/${C}_${V}_$rep.json 2>gpurun_out/obsab/${C}_${V}_$rep.err
      python3 -c "import json;d=json.loads(open('gpurun_out/obsab/${C}_${V}_$rep.json').read().strip().splitlines()[-1]);print('$V', $rep, 'config $C obs %.2f step %.2f step+obs %.2f fused %s' % (d['obs_us'], d['step_us'], d['step_plus_obs_us'], d.get('step_obs_fused_us')))" || true
    done
  done
done
