#!/bin/bash
# Round-4 profile pass of the committed build (outputs under gpurun_out/prof_r04; scripts/collect_profiles_r04.py
# copies the summaries and the per-dispatch PMC rows into profiles/r04/ and regenerates profiles/traffic.json):
#   1. rocprofv3 kernel trace + stats of the driver's exact bench command (bench.py --gpus 1 --steps 20 --warmup 5)
#   2. kernel trace + stats of the 2000-step graph-replayed bench (the timed region only)
#   3. PMC passes on eager launches of k_step, one counter set per pass: SQ (per-wave instruction mix),
#      FETCH_SIZE, WRITE_SIZE -- config 2 (4096 envs) and the config-5 16,384-env slice
#   4. kernel trace + stats of bench_configs.py --config 3,3b,4,5
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_r04
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || exit $?
B="$R/bench.py --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B --graph-only --fused-k 0 --steps 2000 --warmup 20 > $O/trace_bench.json 2> $O/trace_bench.err || exit $?
P="$B --no-graph --fused-k 0 --graph-only --steps 300 --warmup 20"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/c2/sq -o run --output-format csv -- python3 $P > $O/c2_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/c2/fetch -o run --output-format csv -- python3 $P > $O/c2_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/c2/write -o run --output-format csv -- python3 $P > $O/c2_write.log 2>&1 || exit $?
P5="$P --config 5 --total-envs 16384"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/c5/sq -o run --output-format csv -- python3 $P5 > $O/c5_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/c5/fetch -o run --output-format csv -- python3 $P5 > $O/c5_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/c5/write -o run --output-format csv -- python3 $P5 > $O/c5_write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/configs -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3,3b,4,5 > $O/configs.jsonl 2> $O/configs.err || exit $?
tail -1 $O/driver_bench.json | cut -c1-200
