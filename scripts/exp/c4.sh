set -u
for m in map1.txt map2.txt; do
timeout -k 10 200 python bench.py --cpu-seconds 0 --fused-k 0 --graph-only --envs 8192 --map $m --steps 1000 --warmup 50 > gpurun_out/c4_$m.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/c4_$m.json').read().strip().splitlines()[-1]);print('$m 8192 envs', round(d['ms_per_step']*1e3,3), 'us/step')"
done
timeout -k 10 200 python scripts/bench_configs.py --config 4 > gpurun_out/c4_mixed.json 2>/dev/null || exit 1
tail -1 gpurun_out/c4_mixed.json
