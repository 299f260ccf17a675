#!/bin/bash
# Round 4: config-5 step A/B (bench.py --config 5, 131,072 envs on one GPU) of the product build against
# build/ab/libmdl_${B:?}.so, ${REPS:-3} interleaved repeats; then config 2 the same way.
set -u
O=gpurun_out/r04/c5ab_$B
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for V in prod $B; do
    for C in 5 2; do
      if [ $V = prod ]; then
        timeout -k 10 200 python3 bench.py --config $C --cpu-seconds 0 --fused-k 0 --steps 2000 --warmup 100 > $O/${V}_c${C}_$rep.json 2> $O/${V}_c${C}_$rep.err || exit $?
      else
        MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ab/libmdl_$B.so timeout -k 10 200 python3 bench.py --config $C --cpu-seconds 0 --fused-k 0 --steps 2000 --warmup 100 > $O/${V}_c${C}_$rep.json 2> $O/${V}_c${C}_$rep.err || exit $?
      fi
      python3 -c "import json,sys; d=json.loads(open('$O/${V}_c${C}_$rep.json').read().strip().splitlines()[-1]); print('$V config $C rep $rep: %.3f us/step %.3e agent-steps/s' % (d['ms_per_step']*1e3, d['value']))"
    done
  done
done
