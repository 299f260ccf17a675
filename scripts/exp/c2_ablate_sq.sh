#!/bin/bash
# Per-section cost of the headline step kernel k_step<true,1,false,5> (config 2: map1, A = 5,
# P = 50, 4096 envs): for each ablation build (scripts/ablate.sh; each MDL_ABLATE bit removes one
# section: 1 shaped reward, 2 tracker update, 4 movement, 8 package actions, 16 move-validity
# fetch, 32 nearest-package search, 64 carried-package gather) the SQ counters per wave (eager
# launches, 300 steps) and the graph-replayed time per step (bench.py, 2000 steps).
# BENCH_ARGS / OUT: another configuration, e.g. BENCH_ARGS="--config 5 --total-envs 16384" OUT=c5ab.
set -u
export TMPDIR=/tmp
R=$(pwd)
for V in ${VARIANTS:-0 1 2 4 8 16 32 64}; do
  O=$R/gpurun_out/${OUT:-c2ab}/$V
  mkdir -p $O
  L=$R/marl-delivery_amd/build/ablate/libmdl_$V.so
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_step" -d $O/sq -o run --output-format csv -- python3 $R/bench.py ${BENCH_ARGS:-} --no-graph --cpu-seconds 0 --fused-k 0 --graph-only --steps 300 --warmup 20 > $O/sq.log 2>&1 || exit $?
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python3 $R/bench.py ${BENCH_ARGS:-} --cpu-seconds 0 --fused-k 0 --graph-only --steps 2000 --warmup 100 > $O/bench.json 2> $O/bench.err || exit $?
  python3 - <<PY
import csv, glob, collections, json
agg = collections.defaultdict(list)
for f in glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v)//2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
b = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print(json.dumps({"ablate": $V, "us_per_step": round(b["ms_per_step"] * 1e3, 3),
                  "per_wave": {n: round(v / w, 1) for n, v in sorted(m.items())}}))
PY
done
