#!/bin/bash
# One GPU-box pass: parity tests, smoke, the driver's bench command (20 steps) and a
# long bench.  Each GPU step has its own time limit; the first crash / timeout ends it.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; echo "smoke rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err
rc=$?; echo "bench(20) rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > $OUT/bench_long.json 2> $OUT/bench_long.err
rc=$?; echo "bench(2000) rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 - <<EOF
import json
for f in ("bench_driver", "bench_long"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    print(f, "value %.3e" % d["value"], "wall us/step %.3f" % (d["ms_per_step"] * 1e3),
          "event us/step %.3f" % (d["gpu_event_ms_per_step"] * 1e3), "frac %.4f" % d["roofline"]["frac"])
EOF
