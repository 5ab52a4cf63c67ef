#!/bin/bash
# hxt attribution on the dev build: DBG modes (1 no steady loads, 2 no stores, 4 no MFMA, 16 no conversion).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/attr; mkdir -p $O
D=$R/go-audio-resampler_amd/libgar_dev.so
EXTRA=${EXTRA:-'"GAR_HXT":"1"'}
cfgs=""
for dbg in 0 4 2 16 17 6 19 23; do cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",$EXTRA,\"GAR_HXS_DBG\":\"$dbg\"},"; done
cfgs="[${cfgs%,}]"
for wl in ${WLS:-"KB_CH=2,KB_SECONDS=600" "KB_CH=256,KB_SECONDS=10,KB_IN=48000,KB_OUT=44100,KB_Q=4"}; do
  tag=$(echo $wl | tr '=,' '__')
  env $(echo $wl | tr ',' ' ') timeout -k 10 300 python tools/kbench.py "$cfgs" > $O/$tag.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l); print('$wl'[:14], d['cfg'].get('GAR_HXS_DBG'), d.get('ms'), d.get('err','')[-120:])"
done
