#!/bin/bash
# hxt A/B: loud test on the packed f16 hi halves (libgar_pk.so) vs default; tests on the variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04t; mkdir -p $O
U=$R/go-audio-resampler_amd/libgar_pk.so
GAR_LIB_PATH=$U timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_pk.log 2>&1
s=$?; echo "PYTEST_PK_EXIT $s"; tail -2 $O/tests_pk.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_LIB_PATH=$U - GAR_LIB_PATH=$U -" bash tools/gpu_ab.sh || exit 1
