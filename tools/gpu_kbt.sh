#!/bin/bash
# kernel sweep + the split-f16 GPU tests (correctness of a kernel change), in one call
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hx.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kbt_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> gpurun_out/kbt_tests.log; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
timeout -k 10 600 python tools/kbench.py "$KB_SWEEP" > gpurun_out/kbench.log 2>&1
s=$?; echo "KB_EXIT $s" >> gpurun_out/kbench.log; exit $s
