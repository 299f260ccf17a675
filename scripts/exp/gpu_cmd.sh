mkdir -p gpurun_out/r03af
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03af/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r03af/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
MDL_LIB_PATH=$PWD/marl-delivery_amd/build/ab/libmdl_stamps.so timeout -k 10 120 python scripts/exp/stamps.py 1024 4096 > gpurun_out/r03af/stamps.json 2>&1 || exit $?
python3 -c "
import json; t=open('gpurun_out/r03af/stamps.json').read(); d=json.loads(t[t.index('{'):])
for E in d: print(E, d[E]['median_cycles'], d[E]['wave_total_median'])"
VARIANTS="noxcd main" REPS=3 bash scripts/exp/ab_bench.sh || exit $?
VARIANTS="noxcd main" REPS=2 CONFIG=5 STEPS=400 BENCH_EXTRA="--total-envs 16384" bash scripts/exp/ab_bench.sh || exit $?
