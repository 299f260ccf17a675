#!/bin/bash
# Same-box A/B of the fused step + observation launch shape: graph rollout (4096 envs) and config 3.
set -u
MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_B.so timeout -k 10 600 python -u -m pytest -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread tests/test_gpu_step_obs.py tests/test_gpu_rollout.py > gpurun_out/ab_so_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/ab_so_pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for V in A B; do
    L=marl-delivery_amd/build/ablate/libmdl_$V.so
    r=$(MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 300 python scripts/bench_configs.py --config rollout_graph 2>/dev/null | tail -1 | python3 -c "import json,sys; print('%.2f' % json.loads(sys.stdin.read())['us_per_env_step'])")
    c=$(MDL_PROFILING=1 MDL_LIB_PATH=$L timeout -k 10 300 python scripts/bench_configs.py --config 3 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f' % d['step_obs_fused_us'])")
    echo "$V $rep rollout_graph $r us/env-step | config3 step_obs $c us"
  done
done
