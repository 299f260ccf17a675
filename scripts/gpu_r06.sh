#!/bin/bash
# Round 6 GPU pass: the GPU suite (new tests first), smoke, the driver's default bench line,
# the plain multi-rank command, config 3's line.  Each GPU step has its own time limit; the
# first failure ends the call.
set -u
O=gpurun_out/r06/${TAG:-pass}
mkdir -p $O
run() {   # name seconds cmd...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s "$@" > $O/$n.out 2> $O/$n.err
  local rc=$?; echo "$n rc=$rc"; tail -c 600 $O/$n.out; echo
  [ $rc -ne 0 ] && { tail -30 $O/$n.err; exit $rc; }
  return 0
}
if [ -n "${FIRST:-}" ]; then
  run pytest_first 900 python -u -m pytest $FIRST -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [ -z "${SKIP_SUITE:-}" ]; then
  run pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
fi
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_long 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 200
run bench_gpus2 300 python bench.py --gpus 2 --backend gloo --steps 40 --warmup 5 --cpu-seconds 2 --gather
run bench_c3 300 python bench.py --config 3 --steps 200 --warmup 20 --cpu-seconds 4
run bench_c4 300 python bench.py --config 4 --steps 200 --warmup 20 --cpu-seconds 2 --fused-k 0
run bench_c5 300 python bench.py --config 5 --steps 200 --warmup 20 --cpu-seconds 2 --fused-k 0
exit 0
