MDL_LIB_PATH=$PWD/marl-delivery_amd/build/ab/libmdl_sort5.so timeout -k 10 600 python -u -m pytest tests/test_gpu_step_obs.py tests/test_gpu_obs_small.py tests/test_gpu_parity.py tests/test_gpu_rollout.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sort5.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_sort5.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="main sort5" REPS=3 CONFIG=3b bash scripts/exp/ab_obs.sh || exit $?
VARIANTS="main sort5" REPS=2 CONFIG=3 bash scripts/exp/ab_obs.sh
