mkdir -p gpurun_out/r03s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "helper or kat" > gpurun_out/r03s/pytest.log 2>&1; rc=$?; tail -30 gpurun_out/r03s/pytest.log; exit $rc
