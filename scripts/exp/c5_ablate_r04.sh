#!/bin/bash
# Config-5 per-section costs on the round-4 build: for each ablation build (scripts/ablate.sh, MDL_ABLATE bits:
# 1 shaped reward, 2 tracker update, 4 movement, 8 package actions, 32 nearest-package scan, 64 carried gather)
# bench.py --config 5 (131,072 envs, 1000 graph-replayed steps) and SQ counters per wave (16,384-env slice, eager).
set -u
export TMPDIR=/tmp
R=$(pwd)
for V in ${VARIANTS:-0 1 2 4 8 32 64}; do
  O=$R/gpurun_out/r04/c5abl/$V
  mkdir -p $O
  L=$R/marl-delivery_amd/build/ablate/libmdl_$V.so
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 200 python3 $R/bench.py --config 5 --cpu-seconds 0 --fused-k 0 --steps 1000 --warmup 50 > $O/bench.json 2> $O/bench.err || exit $?
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_step" -d $O/sq -o run --output-format csv -- python3 $R/bench.py --config 5 --total-envs 16384 --cpu-seconds 0 --fused-k 0 --no-graph --graph-only --steps 200 --warmup 10 > $O/sq.log 2>&1 || exit $?
  python3 - $O $V <<'PY'
import csv, glob, collections, json, sys
O, V = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(O + "/sq/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v)//2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
b = json.loads(open(O + "/bench.json").read().strip().splitlines()[-1])
print(json.dumps({"ablate": int(V), "us_per_step_131072": round(b["ms_per_step"] * 1e3, 2),
                  "per_wave": {n.replace("SQ_", ""): round(v / w, 1) for n, v in sorted(m.items()) if n != "SQ_WAVES"}}))
PY
done
