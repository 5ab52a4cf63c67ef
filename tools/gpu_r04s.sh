#!/bin/bash
# hxt A/B: uniform mirror decision (libgar_um.so) vs default; group-size sweep on the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04s; mkdir -p $O
U=$R/go-audio-resampler_amd/libgar_um.so
GAR_LIB_PATH=$U timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_um.log 2>&1
s=$?; echo "PYTEST_UM_EXIT $s"; tail -2 $O/tests_um.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_LIB_PATH=$U - GAR_LIB_PATH=$U -" bash tools/gpu_ab.sh || exit 1
NO_TESTS=1 WORKLOADS="cfg2 ns256" ABS="GAR_HXS_G=4 GAR_HXS_G=3" bash tools/gpu_ab.sh || exit 1
