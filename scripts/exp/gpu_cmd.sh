mkdir -p gpurun_out/r03ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_rollout.py tests/test_gpu_api.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03ab/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r03ab/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/exp/vec_cost.py > gpurun_out/r03ab/vec_cost.txt 2>&1; rc=$?; cat gpurun_out/r03ab/vec_cost.txt; [ $rc -ne 0 ] && exit $rc
