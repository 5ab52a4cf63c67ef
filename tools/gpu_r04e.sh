#!/bin/bash
# GPU tests, then the short-call numbers (C-ABI) and a kernel trace of the stereo stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r04e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_layouts.py tests/test_gpu_pcm.py} > $O/tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -3 $O/tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 240 ./tools/cabi_stream 4096 60 2 > $O/cabi_stereo.txt 2>&1 || exit 1
timeout -k 10 240 ./tools/cabi_stream 4096 10 256 > $O/cabi_256.txt 2>&1 || exit 1
cat $O/cabi_stereo.txt $O/cabi_256.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/cprof -o run -- $R/tools/cabi_stream 4096 10 2 > $O/cprof.log 2>&1 || exit 1
cd $R && python3 tools/prof_db.py $(find $O/cprof -name "*.db")
