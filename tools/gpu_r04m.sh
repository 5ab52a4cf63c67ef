#!/bin/bash
# hxt role timing (dev build, GAR_HXS_PROF): cfg2 full / MFMA+LDS+counters / skeleton.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04m; mkdir -p $O
D=$R/go-audio-resampler_amd/libgar_dev.so
cfgs=""
for dbg in 0 19 127; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"1\",\"GAR_HXS_PROF\":\"1\",\"GAR_HXS_DBG\":\"$dbg\"},"; done
cfgs="[${cfgs%,}]"
KB_CH=2 KB_SECONDS=600 timeout -k 10 300 python tools/kbench.py "$cfgs" > $O/attr.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/attr.jsonl'):
    d=json.loads(l); print(d['cfg'].get('GAR_HXS_DBG'), d.get('ms'), d.get('err','')[-200:])
    for p in d.get('prof', []): print('   ', p[:220])"
