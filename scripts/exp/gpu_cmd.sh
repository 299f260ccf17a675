TAG=r03f bash scripts/gpu_check_r03.sh > gpurun_out/r03f.log 2>&1; rc=$?; cat gpurun_out/r03f.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_configs.py --config 3,3b > gpurun_out/r03f/config3.jsonl 2>/dev/null || exit $?
cat gpurun_out/r03f/config3.jsonl | cut -c1-600
TAG=r03f bash scripts/profile_r03.sh > gpurun_out/prof_r03f.log 2>&1; rc=$?; tail -40 gpurun_out/prof_r03f.log; exit $rc
