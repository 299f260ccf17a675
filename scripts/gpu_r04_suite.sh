#!/bin/bash
# Round 4: the GPU suite (all gpu-marked tests), smoke, and the driver's default bench line.
set -u
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/r04/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r04/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04/bench_driver.json 2> gpurun_out/r04/bench_driver.err || exit $?
tail -1 gpurun_out/r04/bench_driver.json | cut -c1-400
if [ -x scripts/exp/expand_probe.bin ]; then
  timeout -k 10 120 scripts/exp/expand_probe.bin > gpurun_out/r04/expand_probe.jsonl 2>&1 || exit $?
  cat gpurun_out/r04/expand_probe.jsonl
fi
