set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 120 ./tools/ubench/mfma_store > $O/mfma_store.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03b_gpu_tests.log 2>&1; s=$?; echo "PYTEST_EXIT $s" >> $O/r03b_gpu_tests.log; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
TAG=r03b bash tools/gpu_cabi.sh
