mkdir -p gpurun_out/r03p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_altfeat.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03p/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r03p/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/exp/helper_cost.py > gpurun_out/r03p/helper_cost.txt 2>&1; rc=$?; cat gpurun_out/r03p/helper_cost.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p/prof -o helper -- python3 scripts/exp/helper_cost.py > gpurun_out/r03p/helper_prof.log 2>&1; rc=$?; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/r03p/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f"
