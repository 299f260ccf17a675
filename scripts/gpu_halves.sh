#!/bin/bash
# Round 6: the two-envs-per-wave config-5 step (k_step_halves).  1. its GPU tests; 2. bench.py
# config 5 per layout (wave / halves) over a batch-size sweep, interleaved; 3. SQ counters per wave of
# both layouts at the full 131,072 envs (eager launches, one PMC pass each).  Each step has its own
# time limit; the first failure ends the call.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06/${TAG:-halves}
mkdir -p $O
run() {   # name seconds cmd...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s "$@" > $O/$n.out 2> $O/$n.err
  local rc=$?; echo "$n rc=$rc"; tail -c 400 $O/$n.out; echo
  [ $rc -ne 0 ] && { tail -30 $O/$n.err; exit $rc; }
  return 0
}
if [ -z "${SKIP_TESTS:-}" ]; then
  run pytest_halves 600 python -u -m pytest ${TESTS:-tests/test_gpu_step_halves.py} -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
fi
for rep in 1 2; do
  for N in ${SIZES:-8192 16384 32768 65536 131072}; do
    for L in wave halves; do
      run c5_${N}_${L}_$rep 200 python bench.py --config 5 --total-envs $N --step-layout $L --steps 300 --warmup 30 --cpu-seconds 0 --fused-k 0 --graph-only
      python3 -c "
import json
d = json.loads(open('$O/c5_${N}_${L}_$rep.out').read().strip().splitlines()[-1])
print('SWEEP', $N, '$L', $rep, 'us/step %.2f' % (d['ms_per_step'] * 1e3), d['roofline']['kernel'])" | tee -a $O/sweep.txt
    done
  done
done
if [ -z "${SKIP_SQ:-}" ]; then
  SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  for L in wave halves; do
    timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "k_step" -d $O/sq_$L -o run --output-format csv -- \
      python3 bench.py --config 5 --step-layout $L --no-graph --graph-only --fused-k 0 --cpu-seconds 0 --no-floor --steps 100 --warmup 10 > $O/sq_$L.log 2>&1
    rc=$?; echo "sq_$L rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/sq_$L.log; exit $rc; }
  done
fi
exit 0
