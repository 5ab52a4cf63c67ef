#!/bin/bash
# hxt sync vs LDS attribution (dev build, cfg2): DBG 1 no steady loads, 2 no stores, 4 no MFMA,
# 8 no B reads, 16 no conversion, 32 compute waves never wait, 64 loaders never wait (wrong output).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/attr5; mkdir -p $O
D=$R/go-audio-resampler_amd/libgar_dev.so
cfgs=""
for dbg in 0 96 19 115 23 119 31 127; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"1\",\"GAR_HXS_DBG\":\"$dbg\"},"; done
for dbg in 0 147; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"0\",\"GAR_HXS_DBG\":\"$dbg\"},"; done
cfgs="[${cfgs%,}]"
KB_CH=2 KB_SECONDS=600 timeout -k 10 300 python tools/kbench.py "$cfgs" > $O/cfg2.jsonl 2>&1 || exit 1
python3 -c "
import json
for l in open('$O/cfg2.jsonl'):
    d=json.loads(l); print(d['cfg'].get('GAR_HXT'), d['cfg'].get('GAR_HXS_DBG'), d.get('ms'), d.get('err','')[-120:])"
