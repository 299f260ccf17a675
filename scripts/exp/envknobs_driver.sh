#!/bin/bash
# Experiment (profiling only): HIP runtime graph knobs vs the driver's short timed region
# (bench.py --steps 20 --warmup 5, fresh process per run; envknobs.sh measured long runs).
set -u
mkdir -p gpurun_out/knobs
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --fused-k 0 --graph-only \
      > gpurun_out/knobs/k.json 2>/dev/null || return $?
  python3 -c "import json;d=json.loads(open('gpurun_out/knobs/k.json').read().strip().splitlines()[-1]);print('$*', 'value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'event %.2f' % (d['gpu_event_ms_per_step']*1e3))"
}
for rep in 1 2 3; do
  run X=base || exit $?
  run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit $?
  run DEBUG_HIP_GRAPH_BATCH_SIZE=1 || exit $?
  run DEBUG_HIP_GRAPH_BATCH_SIZE=4 || exit $?
  run DEBUG_HIP_FORCE_GRAPH_QUEUES=1 || exit $?
  run DEBUG_HIP_FORCE_GRAPH_QUEUES=0 || exit $?
done
