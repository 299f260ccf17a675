#!/bin/bash
# rows-kernel variants: parity tests on each variant lib, then interleaved config 4 / 16,384-env timings.
set -u
R=$(pwd); O=$R/gpurun_out/abrows2; mkdir -p $O
export PYTHONUNBUFFERED=1
for V in ${VARIANTS:-sg pickall}; do
  MDL_PROFILING=1 MDL_LIB_PATH=$R/marl-delivery_amd/build/ab/libmdl_$V.so timeout -k 10 300 python3 -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step_rows.py > $O/tests_$V.log 2>&1
  rc=$?; echo "tests $V rc=$rc"; tail -1 $O/tests_$V.log; [ $rc -ne 0 ] && exit $rc
done
VARIANTS="main ${VARIANTS:-sg pickall}" ENVS=${ENVS:-16384} REPS=${REPS:-3} $R/scripts/exp/ab_rows.sh
