#!/bin/bash
# hxt ring-aligned loads: GPU tests with hxt forced on (bit identity with hxs across chunkings) and
# with the defaults, then hxt vs hxs bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04n; mkdir -p $O
GAR_HXT=1 timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_layouts.py > $O/tests_hxt.log 2>&1
s=$?; echo "PYTEST_HXT_EXIT $s"; tail -2 $O/tests_hxt.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_HXT=1 GAR_HXT=0" bash tools/gpu_ab.sh || exit 1
