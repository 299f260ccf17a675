#!/bin/bash
# Per-section dynamic instruction counts of the config-5 step kernel: SQ counters per wave
# for the ablation builds (build/ablate/libmdl_<bits>.so, scripts/ablate.sh; each MDL_ABLATE
# bit removes one section of the step), config 5 slice, 100 steps.
set -u
export TMPDIR=/tmp
R=$(pwd)
for V in ${VARIANTS:-0 1 2 4 8 32 64}; do
  O=$R/gpurun_out/c5ab/$V
  mkdir -p $O
  MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ablate/libmdl_$V.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex "k_step" -d $O/sq -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 5 --steps 100 --warmup 5 > $O/sq.log 2>&1 || exit $?
  python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("$O/sq/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v)//2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print("ablate $V", {n: round(v / w, 1) for n, v in sorted(m.items())})
PY
done
