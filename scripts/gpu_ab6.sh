#!/bin/bash
# Round 6 A/B pass: 1. GPU tests of a candidate build ($CAND, under build/ab/) on its layout's test
# file ($TESTS); 2. bench.py config 5 per build variant ($VARIANTS) in the halves layout and main in
# the wave layout, interleaved ($REPS); 3. optional probes ($PROBES: binaries under scripts/exp).
set -u
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/r06/${TAG:-ab}
mkdir -p $O
if [ -n "${CAND:-}" ]; then
  if [ "$CAND" = main ]; then CL=$R/marl-delivery_amd/marl_gpu/libmdl.so; else CL=$R/marl-delivery_amd/build/ab/libmdl_$CAND.so; fi
  MDL_PROFILING=1 MDL_LIB_PATH=$CL timeout -k 10 600 \
    python -u -m pytest ${TESTS:-tests/test_gpu_step_halves.py} -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_$CAND.out 2>&1
  rc=$?; tail -3 $O/pytest_$CAND.out; [ $rc -ne 0 ] && { tail -40 $O/pytest_$CAND.out; exit $rc; }
fi
for p in ${PROBES:-}; do
  timeout -k 10 300 $R/scripts/exp/$p.bin > $O/$p.jsonl 2> $O/$p.err
  rc=$?; echo "probe $p rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/$p.err; exit $rc; }
  cat $O/$p.jsonl
done
for rep in $(seq 1 ${REPS:-2}); do
  for VL in ${VARIANTS:-main:wave}; do   # build:layout
    V=${VL%%:*}; L=${VL##*:}
    {
      if [ "$V" = main ]; then Lb=$R/marl-delivery_amd/marl_gpu/libmdl.so; else Lb=$R/marl-delivery_amd/build/ab/libmdl_$V.so; fi
      MDL_PROFILING=1 MDL_LIB_PATH=$Lb timeout -k 10 200 python3 $R/bench.py --config ${CONFIG:-5} --step-layout $L \
        --steps ${STEPS:-300} --warmup 30 --cpu-seconds 0 --fused-k 0 --no-floor --graph-only ${BENCH_EXTRA:-} \
        > $O/${V}_${L}_$rep.json 2> $O/${V}_${L}_$rep.err
      rc=$?; [ $rc -ne 0 ] && { echo "$V $L rc=$rc"; tail -20 $O/${V}_${L}_$rep.err; exit $rc; }
      python3 -c "
import json
d = json.loads(open('$O/${V}_${L}_$rep.json').read().strip().splitlines()[-1])
print('AB', '$V', '$L', $rep, 'us/step %.2f' % (d['ms_per_step'] * 1e3), d['roofline']['kernel'])" | tee -a $O/ab.txt
    }
  done
done
exit 0
