#!/bin/bash
# Round-6 profile pass of the committed build (outputs under gpurun_out/prof_r06; scripts/collect_profiles_r06.py
# copies the summaries and the per-dispatch PMC rows into profiles/r06/final/ and regenerates profiles/traffic.json):
#   1. rocprofv3 kernel trace + stats of the driver's exact bench command (bench.py --steps 20 --warmup 5)
#   2. kernel trace + stats of the 2000-step graph-replayed config-2 bench (the timed region only)
#   3. kernel trace + stats of bench.py --config 3 / 4 / 5 (the kernels those lines time)
#   4. PMC passes on eager launches, one counter set per pass (FETCH_SIZE, WRITE_SIZE, the SQ set) of the
#      exact launches the bench lines time: config 2 (k_step, 4,096 envs), config 3 (k_step_obs, 16,384),
#      config 4 (k_step_rows, 65,536 mixed-map envs), config 5 (131,072 envs, the layout AUTO takes)
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_r06
mkdir -p $O
run() {   # name seconds cmd...: stdout to $O/name.json, stderr to $O/name.err
  local n=$1 s=$2; shift 2
  timeout -k 10 $s "$@" > $O/$n.json 2> $O/$n.err
  local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }; return 0
}
pmc() {   # dir log regex -- bench args   (counters in $PMC)
  local d=$1 lg=$2 rx=$3; shift 3
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "$rx" -d $O/$d -o run --output-format csv -- python3 $R/bench.py "$@" > $O/$lg.log 2>&1
  local rc=$?; echo "pmc $d rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/$lg.log; exit $rc; }; return 0
}
run driver_bench 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5
run trace_bench 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --graph-only --fused-k 0 --steps 2000 --warmup 20
run c3_bench 300 rocprofv3 --kernel-trace --stats -d $O/c3trace -o run --output-format csv -- python3 $R/bench.py --config 3 --cpu-seconds 0 --graph-only --steps 300 --warmup 20
run c4_bench 300 rocprofv3 --kernel-trace --stats -d $O/c4trace -o run --output-format csv -- python3 $R/bench.py --config 4 --cpu-seconds 0 --graph-only --fused-k 0 --steps 300 --warmup 20
run c5_bench 300 rocprofv3 --kernel-trace --stats -d $O/c5trace -o run --output-format csv -- python3 $R/bench.py --config 5 --cpu-seconds 0 --graph-only --fused-k 0 --steps 300 --warmup 20
E="--cpu-seconds 0 --no-graph --graph-only --fused-k 0 --no-floor --steps 100 --warmup 10"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for k in fetch write sq; do
  case $k in fetch) PMC=FETCH_SIZE ;; write) PMC=WRITE_SIZE ;; sq) PMC=$SQ ;; esac
  pmc c2/$k c2_$k "k_step[<(]" $E
  pmc c3/$k c3_$k "k_step_obs" $E --config 3
  pmc c4/$k c4_$k "k_step_rows" $E --config 4
  pmc c5full/$k c5full_$k "k_step" $E --config 5
done
tail -1 $O/driver_bench.json | cut -c1-300
exit 0
