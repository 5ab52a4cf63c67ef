#!/bin/bash
# GPU tests; short-call numbers (C-ABI); cfg5 per-kind attribution (GAR_BG_DBG: 2 no stores,
# 16 no B / window loads, 32 no A loads, 64 no history keep).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r04h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_layouts.py tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_pcm.py} > $O/tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -3 $O/tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 240 ./tools/cabi_stream 4096 30 2 > $O/cabi.txt 2>&1 || exit 1
timeout -k 10 240 ./tools/cabi_stream 4096 10 256 >> $O/cabi.txt 2>&1 || exit 1
cat $O/cabi.txt
L=$O/cfg5_attr.txt
for v in 0 2 16 32 64 114; do
  echo "== GAR_BG_DBG=$v" >> $L
  GAR_BG_DBG=$v P_N=300 timeout -k 10 90 python tools/cfg5_probe.py >> $L 2>&1 || exit 1
done
grep -v amdgpu.ids $L
