#!/bin/bash
# Round profile pass (rocprofv3): kernel trace + stats of the bench command,
# then separate PMC passes (SQ set, FETCH_SIZE, WRITE_SIZE) on eager launches
# of k_step, and trace + FETCH/WRITE of k_obs on config 3.  Summaries go to
# gpurun_out/prof_<tag>/summary_*.json (copied into profiles/ by hand).
set -u
export TMPDIR=/tmp
R=$(pwd)
TAG=${TAG:-round}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
B="$R/bench.py --cpu-seconds 0"
# --graph-only: the trace holds the warmup and the timed graph replay only, so the
# stats average is the timed region's (bench.py's kernel_us)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B --graph-only --fused-k 0 --steps 2000 --warmup 20 > $O/trace_bench.log 2>&1 || exit $?
P="$B --no-graph --fused-k 0 --steps 300 --warmup 20"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_step -d $O/sq -o run --output-format csv -- python3 $P > $O/sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_step -d $O/fetch -o run --output-format csv -- python3 $P > $O/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_step -d $O/write -o run --output-format csv -- python3 $P > $O/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $TAG k_step > $O/summary_step.json || exit $?
O3=$R/gpurun_out/prof_${TAG}_obs
mkdir -p $O3
C="$R/scripts/bench_configs.py --config 3"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O3/trace -o run --output-format csv -- python3 $C > $O3/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_obs -d $O3/fetch -o run --output-format csv -- python3 $C > $O3/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_obs -d $O3/write -o run --output-format csv -- python3 $C > $O3/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py ${TAG}_obs k_obs > $O3/summary_obs.json || exit $?
ls $O $O3
# config 3b (1007-dim actor vectors): kernel trace + stats only
O3B=$R/gpurun_out/prof_${TAG}_obs3b
mkdir -p $O3B
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O3B/trace -o run --output-format csv -- python3 $R/scripts/bench_configs.py --config 3b > $O3B/trace.log 2>&1 || exit $?
ls $O3B
