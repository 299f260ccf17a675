timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sw.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_sw.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="main nosw" REPS=3 CONFIG=3b bash scripts/exp/ab_obs.sh || exit $?
VARIANTS="main nosw" REPS=1 CONFIG=3 bash scripts/exp/ab_obs.sh || exit $?
MDL_LIB_PATH=$PWD/marl-delivery_amd/build/ab/libmdl_trk.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_step_obs.py tests/test_gpu_checkpoint.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_trk.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_trk.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="main trk" REPS=3 bash scripts/exp/ab_bench.sh || exit $?
MDL_LIB_PATH=$PWD/marl-delivery_amd/build/ab/libmdl_br.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_br.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_br.log; [ $rc -ne 0 ] && exit $rc
for V in main br; do
  if [ $V = main ]; then L=$PWD/marl-delivery_amd/marl_gpu/libmdl.so; else L=$PWD/marl-delivery_amd/build/ab/libmdl_$V.so; fi
  for C in 1024 4096; do
    MDL_LIB_PATH=$L MDL_OBS_CHUNK=$C timeout -k 10 300 python scripts/bench_configs.py --config 5 --steps 100 > gpurun_out/c5obs_${V}_$C.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/c5obs_${V}_$C.json').read().strip().splitlines()[-1])
print('$V chunk $C', 'obs chunk us %.1f' % d['obs_chunk_us'], 'TB/s %.2f' % (d['obs_chunk_roofline']['achieved_GBs']/1e3), 'step us %.2f' % d['step_us'])"
  done
done
