#!/bin/bash
# The driver's command (bench.py --steps 20 --warmup 5) under launch / host-wait variants, a
# fresh process per run as the driver runs it, the variants interleaved $REPS times.
# Variants: name:extra-args (graph steps per replay, hipSetDeviceFlags schedule mode).
set -u
O=gpurun_out/region_ab
mkdir -p $O
VARS=${VARS:-"base: spin:--host-wait=spin g10:--graph-steps=10 g5:--graph-steps=5 g5spin:--graph-steps=5,--host-wait=spin"}
for rep in $(seq 1 ${REPS:-3}); do
  for V in $VARS; do
    N=${V%%:*}; X=${V#*:}; X=${X//,/ }
    timeout -k 10 120 python3 bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} --cpu-seconds 0 --fused-k 0 --graph-only $X \
        > $O/${N}_$rep.json 2> $O/${N}_$rep.err || exit $?
    python3 -c "
import json
d = json.loads(open('$O/${N}_$rep.json').read().strip().splitlines()[-1])
print('$N', $rep, 'value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step'] * 1e3),
      'event %.2f' % (d['gpu_event_ms_per_step'] * 1e3), d['host_wait'], d['graph_steps'])"
  done
done
