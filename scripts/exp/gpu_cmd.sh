mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03v/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r03v/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 120 python scripts/bench_configs.py --config 1 > gpurun_out/r03v/config1_$i.json 2>/dev/null || exit $?; cat gpurun_out/r03v/config1_$i.json; done
timeout -k 10 120 python scripts/exp/helper_cost.py > gpurun_out/r03v/helper_cost.txt 2>&1; cat gpurun_out/r03v/helper_cost.txt
