mkdir -p gpurun_out/r03am
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_dist.py tests/test_gpu_api.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r03am/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03am/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03am/driver_$rep.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r03am/driver_$rep.json').read().strip().splitlines()[-1]); print('driver', $rep, 'value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'event %.2f' % (d['gpu_event_ms_per_step']*1e3), 'frac %.4f' % d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > gpurun_out/r03am/long.json 2>/dev/null || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r03am/long.json').read().strip().splitlines()[-1]); print('long value %.3e' % d['value'], 'us/step %.3f' % (d['ms_per_step']*1e3))"
