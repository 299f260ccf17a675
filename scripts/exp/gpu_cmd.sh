TAG=r03k bash scripts/gpu_round.sh > gpurun_out/r03k.log 2>&1; rc=$?; cat gpurun_out/r03k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/exp/helper_cost.py > gpurun_out/r03k/helper_cost.txt 2>&1; cat gpurun_out/r03k/helper_cost.txt
timeout -k 10 120 python scripts/bench_configs.py --config 1 > gpurun_out/r03k/config1.json 2>/dev/null; cat gpurun_out/r03k/config1.json
timeout -k 10 300 python scripts/bench_configs.py --config 3,3b,5 > gpurun_out/r03k/configs.jsonl 2>/dev/null; cut -c1-300 gpurun_out/r03k/configs.jsonl
MDL_LIB_PATH=$PWD/marl-delivery_amd/build/ab/libmdl_pick.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_rollout.py tests/test_gpu_checkpoint.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_pick.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pick.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="nopick pick" REPS=3 CONFIG=5 STEPS=400 BENCH_EXTRA="--total-envs 16384" bash scripts/exp/ab_bench.sh
