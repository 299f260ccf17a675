#!/bin/bash
# SQ counters per wave of k_step_rows vs k_step, config 2 (4096 envs) and config 4 (65,536 mixed-map envs).
set -u
export TMPDIR=/tmp
O=$(pwd)/gpurun_out/rows_sq; mkdir -p $O
E="--cpu-seconds 0 --no-graph --graph-only --fused-k 0 --no-floor --steps 100 --warmup 10"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
for L in rows wave; do
  for C in 2 4; do
    timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "k_step" -d $O/${L}_c$C -o run --output-format csv -- python3 $(pwd)/bench.py $E --config $C --step-layout $L > $O/${L}_c$C.log 2>&1
    rc=$?; echo "$L c$C rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/${L}_c$C.log; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.path.join(os.getcwd(), "gpurun_out/rows_sq")
for d in sorted(glob.glob(O + "/*_c*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
    w = m.get("SQ_WAVES", 1)
    print(os.path.basename(d.rstrip("/")), "waves", w, {k: round(v / w, 1) for k, v in sorted(m.items()) if k != "SQ_WAVES"})
PY
