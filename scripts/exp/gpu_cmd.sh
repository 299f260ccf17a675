mkdir -p gpurun_out/r03ai
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03ai/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/r03ai/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="soa main" REPS=3 bash scripts/exp/ab_bench.sh || exit $?
VARIANTS="soa main" REPS=2 CONFIG=5 STEPS=400 BENCH_EXTRA="--total-envs 16384" bash scripts/exp/ab_bench.sh || exit $?
CONFIG=3 VARIANTS="soa main" REPS=2 bash scripts/exp/ab_obs.sh || exit $?
