#!/bin/bash
# SQ counters of the config-5 step kernel (64x64, A = 16, P = 100, 16384 envs).
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_c5
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_step" -d $O/sq -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 5 > $O/sq.log 2>&1 || exit $?
python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("$O/sq/*/run_counter_collection.csv") + glob.glob("$O/sq/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sorted(v)[len(v)//2] for n, v in c.items()}
    w = m["SQ_WAVES"]
    print(k, {n: round(v / w, 1) for n, v in m.items()})
PY
