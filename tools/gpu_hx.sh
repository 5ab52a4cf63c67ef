#!/bin/bash
# Split-f16 kernel bring-up: hx tests, all GPU tests, knob sweep.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hx.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hx_tests.log 2>&1
s=$?; echo "HX_EXIT $s" >> gpurun_out/hx_tests.log; [ $s -eq 0 ] || exit $s
if [ -z "$SKIP_ALL" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> gpurun_out/gpu_tests.log; [ $s -eq 0 ] || exit $s
fi
if [ -n "$KB_SWEEP" ]; then
timeout -k 10 600 python tools/kbench.py "$KB_SWEEP" > gpurun_out/kbench.log 2>&1
s=$?; echo "KB_EXIT $s" >> gpurun_out/kbench.log; [ $s -eq 0 ] || exit $s
fi
exit 0
