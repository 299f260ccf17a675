#!/bin/bash
# Experiment (profiling only): HIP runtime knobs vs graph-replayed step time.
set -u
run() {
  env "$@" timeout -k 10 120 python bench.py --cpu-seconds 0 --fused-k 0 --steps 3000 --warmup 100 > gpurun_out/knob.json 2>/dev/null || return $?
  python3 -c "import json;d=json.loads(open('gpurun_out/knob.json').read().strip().splitlines()[-1]);print('$*', round(d['ms_per_step']*1e3,3), 'us/step, eager', round(d['eager']['ms_per_step']*1e3,3))"
}
run X=1 || exit $?
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit $?
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit $?
run HIP_FORCE_DEV_KERNARG=0 || exit $?
run HIP_FORCE_DEV_KERNARG=1 || exit $?
run AMD_DIRECT_DISPATCH=0 || exit $?
run DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 || exit $?
run X=2 || exit $?
