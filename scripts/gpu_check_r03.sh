#!/bin/bash
# One GPU-box pass for round-3 work: the GPU suite, then the dict-API / helper per-call costs,
# config 5 with chunked observations, and bench.py --config 4 / 5 at one rank.  Every GPU step
# has its own time limit; the first failure ends the script.
set -u
O=gpurun_out/${TAG:-r03}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/bench_configs.py --config 1 > $O/config1.json 2>&1 || exit $?
cat $O/config1.json
timeout -k 10 120 python scripts/exp/helper_cost.py > $O/helper_cost.txt 2>&1 || exit $?
cat $O/helper_cost.txt
if [ -z "${QUICK:-}" ]; then
timeout -k 10 300 python scripts/bench_configs.py --config 5 > $O/config5.json 2>&1 || exit $?
cat $O/config5.json
timeout -k 10 300 python bench.py --config 4 --steps 200 --warmup 20 --cpu-seconds 3 > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 300 python bench.py --config 5 --steps 200 --warmup 20 --cpu-seconds 3 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
python3 -c "
import json
for f in ('bench_c4', 'bench_c5'):
    d = json.loads(open('$O/%s.json' % f).read().strip().splitlines()[-1])
    print(f, 'value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'frac %.4f' % d['roofline']['frac'], d['config']['map_runs_rank0'])
"
fi
