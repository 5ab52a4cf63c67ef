#!/bin/bash
# One GPU pytest run (args = pytest selection), log under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 ${GPU_TEST_TIMEOUT:-900} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/gpu_pytest.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> gpurun_out/gpu_pytest.log; tail -5 gpurun_out/gpu_pytest.log; exit $s
