#!/bin/bash
# Loud bound 16 -> 16 - 2^-8: the new regression test against the previous library (expected to fail),
# then every GPU test and the default bench line on the fixed library.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04q; mkdir -p $O
GAR_LIB_PATH=$R/go-audio-resampler_amd/libgar_old16.so timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py -k just_below_16 > $O/old_lib_test.log 2>&1
echo "OLD_LIB_TEST_EXIT $?"; tail -3 $O/old_lib_test.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -2 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="-" bash tools/gpu_ab.sh || exit 1
