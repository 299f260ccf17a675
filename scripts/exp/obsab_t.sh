#!/bin/bash
# Observation-builder parity tests against build B, then the config 3 / 3b A/B.
set -u
mkdir -p gpurun_out/obsab
MDL_PROFILING=1 MDL_LIB_PATH=marl-delivery_amd/build/ablate/libmdl_B.so timeout -k 10 600 python -u -m pytest -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread tests/test_gpu_obs_small.py tests/test_gpu_step_obs.py tests/test_gpu_parity.py \
    tests/test_gpu_scale.py > gpurun_out/obsab/pytest_B.log 2>&1
rc=$?; tail -2 gpurun_out/obsab/pytest_B.log; [ $rc -ne 0 ] && exit $rc
bash scripts/exp/obsab.sh
