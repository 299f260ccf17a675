#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench.  Stops at the first crash /
# timeout (exit codes other than 0 = pass and 1 = test failures).
set -u
mkdir -p gpurun_out
STEPS=${STEPS:-1000}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 100 > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc
