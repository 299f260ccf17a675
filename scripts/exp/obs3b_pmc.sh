#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the observation builder on config 3b (1007-dim actor vectors)
# and config 3: is the write traffic above the output bytes (partial-line rewrites)?
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_obs3b
mkdir -p $O
for C in 3b 3; do
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_obs_small -d $O/w$C -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config $C > $O/w$C.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_obs_small -d $O/f$C -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config $C > $O/f$C.log 2>&1 || exit $?
done
python3 - <<PY
import csv, glob
for C in ("3b", "3"):
    for k in ("w", "f"):
        v = sorted(float(r["Counter_Value"]) for f in glob.glob("$O/%s%s/*/run_counter_collection.csv" % (k, C)) for r in csv.DictReader(open(f)))
        if v: print(C, k, "median KB", v[len(v)//2], "n", len(v))
PY
