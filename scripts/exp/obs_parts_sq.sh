#!/bin/bash
# Per-output time and SQ counters per wave of k_obs_small, config 3 (OBS_MO_MP=4,5) and 3b (100,100):
# the builder skips the sections of outputs it is not asked for (profiling only).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/obs_parts
mkdir -p $O
for MM in 4,5 100,100; do
  OBS_MO_MP=$MM timeout -k 10 120 python3 scripts/exp/obs_parts.py > $O/time_$MM.json 2>/dev/null || exit $?
  echo "times $MM: $(cat $O/time_$MM.json)"
  for W in all actor_map actor_vec critic_map critic_vec; do
    OBS_MO_MP=$MM OBS_WHICH=$W timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_obs_small -d $O/sq_${MM}_$W -o run --output-format csv -- python3 scripts/exp/obs_parts.py > $O/sq_${MM}_$W.log 2>&1 || exit $?
    python3 - $O/sq_${MM}_$W "$MM $W" <<'PY'
import csv, glob, collections, json, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v) // 2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print(sys.argv[2], json.dumps({n.replace("SQ_", ""): round(v / w, 1) for n, v in sorted(m.items()) if n != "SQ_WAVES"}))
PY
  done
done
