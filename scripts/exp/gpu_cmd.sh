TAG=r03d bash scripts/gpu_check_r03.sh > gpurun_out/r03d.log 2>&1; rc=$?; cat gpurun_out/r03d.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="main nowait notup" REPS=2 CONFIG=3b bash scripts/exp/ab_obs.sh || exit $?
timeout -k 10 120 build/graph_gaps > gpurun_out/graph_gaps.jsonl 2>&1; rc=$?; cat gpurun_out/graph_gaps.jsonl; exit $rc
