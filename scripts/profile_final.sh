#!/bin/bash
# Final profile pass of the committed build (round 3): rocprofv3 kernel trace + stats of the bench's
# 2000-step graph run (config 2), then separate PMC passes on eager launches of k_step (SQ set,
# FETCH_SIZE, WRITE_SIZE) for config 2 and the config-5 16384-env slice, and kernel trace + stats
# of bench_configs.py --config 3,3b,4,5.  Outputs under gpurun_out/prof_${TAG}.
set -u
export TMPDIR=/tmp
R=$(pwd)
TAG=${TAG:-r03}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
B="$R/bench.py --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B --graph-only --fused-k 0 --steps 2000 --warmup 20 > $O/trace_bench.log 2>&1 || exit $?
P="$B --no-graph --fused-k 0 --graph-only --steps 300 --warmup 20"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/c2/sq -o run --output-format csv -- python3 $P > $O/c2_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/c2/fetch -o run --output-format csv -- python3 $P > $O/c2_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/c2/write -o run --output-format csv -- python3 $P > $O/c2_write.log 2>&1 || exit $?
P5="$P --config 5 --total-envs 16384"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/c5/fetch -o run --output-format csv -- python3 $P5 > $O/c5_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/c5/write -o run --output-format csv -- python3 $P5 > $O/c5_write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/configs -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3,3b,4,5 > $O/configs.jsonl 2> $O/configs.err || exit $?
python3 $R/scripts/traffic_json.py $O/traffic.json $R/profiles/r03/fetch_calibration.json c2=$O/c2 "c5=$O/c5:16384,16,100,synthetic64.txt" > $O/traffic.log || exit $?
python3 - <<PY
import csv, glob, collections, json
for d in ("trace", "configs"):
    for f in glob.glob("$O/%s/**/run_kernel_stats.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            print(d, r["Name"][:60], r["Calls"], "avg %.2f us" % (float(r["AverageNs"]) / 1e3))
agg = collections.defaultdict(list)
for f in glob.glob("$O/c2/sq/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sorted(v)[len(v)//2] for n, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print("c2 per wave", json.dumps({n: round(v / w, 1) for n, v in sorted(m.items())}))
PY
cat $O/traffic.log
# the driver's exact bench command under the kernel trace (its 20 timed + 5 warmup graph steps and
# the eager / fused / isolated legs after the timed region)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || exit $?
for f in $(find $O/driver -name run_kernel_stats.csv); do cp $f $O/driver_kernel_stats.csv; done
tail -1 $O/driver_bench.json | cut -c1-300
