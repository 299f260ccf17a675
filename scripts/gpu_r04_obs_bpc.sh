#!/bin/bash
# Round 4: the small observation builder with a capped grid (MDL_OBS_BPC workgroups per CU; waves loop
# over envs so one env's stores drain while the next is computed) vs one wave per env (0); configs 3 / 3b,
# interleaved repeats; then SQ counters per wave of k_obs_small on config 3 (one wave per env and BPC=${SQ_BPC:-4}).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/obs_bpc
mkdir -p $O
for rep in 1 2; do
  for B in 0 1 2 4 8; do
    MDL_OBS_BPC=$B timeout -k 10 300 python3 scripts/bench_configs.py --config 3,3b > $O/bpc${B}_$rep.jsonl 2> $O/bpc${B}_$rep.err || exit $?
    python3 - $O/bpc${B}_$rep.jsonl bpc$B <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], d["config"], "obs %.1f us %.2f TB/s" % (d["obs_us"], d["obs_roofline"]["achieved_GBs"] / 1e3),
              "step+obs fused %.1f us" % d["step_obs_fused_us"], "two launches %.1f" % d["step_plus_obs_us"])
PY
  done
done
for B in 0 ${SQ_BPC:-4}; do
  MDL_OBS_BPC=$B timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_obs_small -d $O/sq$B -o run --output-format csv -- python3 scripts/bench_configs.py --config 3 --steps 40 > $O/sq$B.log 2>&1 || exit $?
  python3 - $O/sq$B $B <<'PY'
import csv, glob, collections, json, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v) // 2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print("bpc", sys.argv[2], "k_obs_small per wave", json.dumps({n: round(v / w, 1) for n, v in sorted(m.items())}))
PY
done
