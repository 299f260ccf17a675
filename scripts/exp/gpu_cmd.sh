mkdir -p gpurun_out/r03an
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_rollout.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03an/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03an/pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="head nu2 main nu8" REPS=3 CONFIG=5 STEPS=400 BENCH_EXTRA="--total-envs 16384" bash scripts/exp/ab_bench.sh || exit $?
