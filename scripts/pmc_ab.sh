#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the step launches of bench.py --config $CONFIG per A/B build ($VARIANTS: names
# under build/ab, or main), one counter per rocprofv3 pass; medians printed per variant.
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06/${TAG:-pmcab}
mkdir -p $O
for V in ${VARIANTS:-main}; do
  if [ "$V" = main ]; then L=$R/marl-delivery_amd/marl_gpu/libmdl.so; else L=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_step" -d $O/$V/$C -o run \
      --output-format csv -- python3 $R/bench.py --config ${CONFIG:-5} --cpu-seconds 0 --no-graph --graph-only --fused-k 0 \
      --no-floor --steps 40 --warmup 5 > $O/${V}_$C.log 2>&1
    rc=$?; echo "pmc $V $C rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/${V}_$C.log; exit $rc; }
    python3 - "$O/$V/$C" "$V" "$C" <<'PY'
import csv, glob, statistics, sys
vals = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if "k_step" in r["Kernel_Name"]]
print("PMC", sys.argv[2], sys.argv[3], "dispatches", len(vals), "median KB %.0f" % statistics.median(vals))
PY
  done
done
exit 0
