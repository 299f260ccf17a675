#!/bin/bash
# Round 4: observation builder A/B -- the product build (records + flat emission pass) against the
# round-3 wave-per-env builder (build/ab/libmdl_slab.so, -DMDL_OBS_RECORD=0), configs 3 and 3b,
# interleaved repeats; then rocprofv3 kernel stats of the product build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/obs_ab
mkdir -p $O
for rep in 1 2; do
  for V in rec slab; do
    if [ $V = rec ]; then
      timeout -k 10 300 python3 scripts/bench_configs.py --config 3,3b > $O/${V}_$rep.jsonl 2> $O/${V}_$rep.err || exit $?
    else
      MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ab/libmdl_slab.so timeout -k 10 300 python3 scripts/bench_configs.py --config 3,3b > $O/${V}_$rep.jsonl 2> $O/${V}_$rep.err || exit $?
    fi
    python3 - $O/${V}_$rep.jsonl $V <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], d["config"], "obs %.1f us %.2f TB/s" % (d["obs_us"], d["obs_roofline"]["achieved_GBs"] / 1e3),
              "step+obs fused %.1f us" % d["step_obs_fused_us"], "two launches %.1f" % d["step_plus_obs_us"], "step %.2f" % d["step_us"])
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_configs.py --config 3,3b > $O/prof.jsonl 2> $O/prof.err || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r04/obs_ab/prof/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:70], r["Calls"], "avg %.2f us" % (float(r["AverageNs"]) / 1e3))
PY
