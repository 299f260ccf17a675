#!/bin/bash
# SQ instruction counts per wave of the config-5 step kernel (16,384-env slice, eager launches) per
# variant (main = in-tree libmdl.so, else build/ab/libmdl_<name>.so).
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/c5sq
mkdir -p $O
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
  for C in ${CONFIGS:-5}; do
    if [ $C = 5 ]; then X="--config 5 --total-envs 16384"; else X="--config $C"; fi
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step \
      -d $O/${V}_$C -o run --output-format csv -- python3 $R/bench.py $X --no-graph --graph-only --fused-k 0 --cpu-seconds 0 --no-floor --steps 200 --warmup 20 > $O/${V}_$C.log 2>&1 || exit $?
    python3 - $O/${V}_$C "$V c$C" <<'PY'
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
