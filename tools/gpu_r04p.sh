#!/bin/bash
# New defaults (hxt_kernel for every stereo / 16-channel-row f32 plan): all GPU tests, then cfg3 roles A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04p; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -2 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg3" ABS="GAR_HXT_ROLES=0 -" bash tools/gpu_ab.sh || exit 1
NO_TESTS=1 WORKLOADS="cfg2 ns256" ABS="- GAR_HXT=0" bash tools/gpu_ab.sh || exit 1
