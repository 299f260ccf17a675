#!/bin/bash
# Parity of mdl_step_obs, then config 3 timing: step + build_obs (two launches) vs step_obs,
# and the config-2 A/B of the step kernel after the step_body refactor.
set -u
mkdir -p gpurun_out/so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/so/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/so/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/bench_configs.py --config 3 > gpurun_out/so/c3.json 2>gpurun_out/so/c3.err || exit 1
tail -1 gpurun_out/so/c3.json
timeout -k 10 200 python scripts/bench_configs.py --config 3b > gpurun_out/so/c3b.json 2>gpurun_out/so/c3b.err || exit 1
tail -1 gpurun_out/so/c3b.json
TESTS=0 bash scripts/exp/ab.sh
