#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the step kernel's access shapes (scripts/exp/fetch_cal.hip):
# one rocprofv3 PMC pass per counter, then a summary (ratio of counted to algorithmic bytes per
# shape and placement) into gpurun_out/fetch_cal/summary.json.  Build first:
#   hipcc --offload-arch=gfx950 -O2 scripts/exp/fetch_cal.hip -o build/fetch_cal
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/fetch_cal
mkdir -p $O
timeout -k 10 60 $R/build/fetch_cal 64 > $O/plain.jsonl 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $R/build/fetch_cal 64 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $R/build/fetch_cal 64 > $O/write.log 2>&1 || exit $?
python3 $R/scripts/fetch_cal_summary.py $O > $O/summary.json || exit $?
cat $O/summary.json
