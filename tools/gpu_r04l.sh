#!/bin/bash
# hxt (inlined slow paths, opaque loader indices) and hxs (opaque loader indices) vs the previous hxs:
# GPU tests with hxt forced on and with the defaults, bench A/B, hxt dev attribution.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04l; mkdir -p $O
GAR_HXT=1 timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_hxt.log 2>&1
s=$?; echo "PYTEST_HXT_EXIT $s"; tail -2 $O/tests_hxt.log; [ $s -eq 0 ] || exit $s
timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_layouts.py > $O/tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -2 $O/tests.log; [ $s -eq 0 ] || exit $s
B=$R/go-audio-resampler_amd/libgar_base.so
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_HXT=1 GAR_HXT=0 GAR_HXT=0,GAR_LIB_PATH=$B" bash tools/gpu_ab.sh || exit 1
D=$R/go-audio-resampler_amd/libgar_dev.so
cfgs=""
for dbg in 0 19 127; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"1\",\"GAR_HXS_DBG\":\"$dbg\"},"; done
cfgs="[${cfgs%,}]"
KB_CH=2 KB_SECONDS=600 timeout -k 10 300 python tools/kbench.py "$cfgs" > $O/attr.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/attr.jsonl'):
    d=json.loads(l); print(d['cfg'].get('GAR_HXT'), d['cfg'].get('GAR_HXS_DBG'), d.get('ms'), d.get('err','')[-120:])"
