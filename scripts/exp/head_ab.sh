#!/bin/bash
# The driver's command (--steps 20 --warmup 5) with the timed region's first graphs split off
# (--graph-head), fresh process per run, interleaved reps.  Lines in gpurun_out/head/.
set -u
O=gpurun_out/head; mkdir -p $O
for rep in 1 2 3; do
  for H in none 1 1,3 2,6 1,2,4 4; do
    hh=$H; [ "$H" = none ] && hh=""
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --fused-k 0 --no-floor --graph-only --graph-head "$hh" > $O/h${H}_$rep.json 2> $O/h${H}_$rep.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/h${H}_$rep.err; exit $rc; }
    python3 -c "
import json
d=json.loads(open('$O/h${H}_$rep.json').read().strip().splitlines()[-1])
print('head', '$H', $rep, f\"{d['value']:.4e}\", 'wall %.3f' % (d['ms_per_step']*1e3), 'event %.3f' % (d['gpu_event_ms_per_step']*1e3), d['graph_chunks'])"
  done
done
timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 --cpu-seconds 0 --fused-k 0 --no-floor --graph-only --graph-head 1,3 > $O/long_13.json 2>&1; python3 -c "
import json
d=json.loads(open('$O/long_13.json').read().strip().splitlines()[-1])
print('long 1,3', f\"{d['value']:.4e}\", 'wall %.3f' % (d['ms_per_step']*1e3), d['graph_chunks'])"
