#!/bin/bash
# hxt with inlined slow paths: tests with hxt forced on (NS 9 plans too), hxt vs hxs bench lines,
# dev attribution (nothing / full).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04k; mkdir -p $O
GAR_HXT=1 timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_hxt.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -2 $O/tests_hxt.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_HXT=1 GAR_HXT=0" bash tools/gpu_ab.sh || exit 1
D=$R/go-audio-resampler_amd/libgar_dev.so
cfgs=""
for dbg in 0 19 127; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"1\",\"GAR_HXS_DBG\":\"$dbg\"},"; done
cfgs="[${cfgs%,}]"
KB_CH=2 KB_SECONDS=600 timeout -k 10 300 python tools/kbench.py "$cfgs" > $O/attr.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/attr.jsonl'):
    d=json.loads(l); print(d['cfg'].get('GAR_HXT'), d['cfg'].get('GAR_HXS_DBG'), d.get('ms'), d.get('err','')[-120:])"
