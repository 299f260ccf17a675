mkdir -p gpurun_out/r03as
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03as/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r03as/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="prev main" REPS=3 bash scripts/exp/ab_bench.sh || exit $?
VARIANTS="prev main" REPS=2 CONFIG=5 STEPS=400 BENCH_EXTRA="--total-envs 16384" bash scripts/exp/ab_bench.sh || exit $?
VARIANTS="prev main" REPS=2 CONFIG=4 STEPS=400 bash scripts/exp/ab_bench.sh || exit $?
CONFIG=3 VARIANTS="prev main" REPS=2 bash scripts/exp/ab_obs.sh || exit $?
for rep in 1 2; do for V in prev main; do
  if [ "$V" = main ]; then L=$PWD/marl-delivery_amd/marl_gpu/libmdl.so; else L=$PWD/marl-delivery_amd/build/ab/libmdl_$V.so; fi
  MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r03as/${V}_$rep.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r03as/${V}_$rep.json').read().strip().splitlines()[-1]); print('driver $V', $rep, 'value %.3e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3))"
done; done
