#!/bin/bash
# SQ counters per wave of k_obs_small on config 3b (16384 envs, MO = MP = 100): the whole builder
# and the actor vectors alone (OBS_WHICH), one rocprofv3 PMC pass each.
set -u
export TMPDIR=/tmp
R=$(pwd)
for W in all actor_vec; do
  O=$R/gpurun_out/obs_sq3b/$W
  mkdir -p $O
  OBS_WHICH=$W OBS_MO_MP=100,100 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_obs_small" -d $O/sq -o run --output-format csv -- python3 $R/scripts/exp/obs_parts.py > $O/sq.log 2>&1 || exit $?
  python3 - <<PY
import csv, glob, collections, json
agg = collections.defaultdict(list)
for f in glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v)//2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print("$W", json.dumps({n: round(v / w, 1) for n, v in sorted(m.items())}))
PY
done
