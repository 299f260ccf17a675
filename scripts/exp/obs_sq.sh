#!/bin/bash
# SQ counters of the observation builder (config 3) and of k_step_obs (config 3, step_obs).
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_obs_sq
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_obs_small|k_step_obs" -d $O/sq -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3 > $O/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR --kernel-include-regex "k_obs_small|k_step_obs" -d $O/sq2 -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3 > $O/sq2.log 2>&1 || exit $?
python3 - <<PY
import csv, glob, collections
for d in ("sq", "sq2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob("$O/%s/*/run_counter_collection.csv" % d) + glob.glob("$O/%s/run_counter_collection.csv" % d):
        for r in csv.DictReader(open(f)):
            k = "k_step_obs" if "k_step_obs" in r["Kernel_Name"] else "k_obs_small"
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        print(k, {n: sorted(v)[len(v)//2] for n, v in c.items()})
PY
