#!/bin/bash
# Attribution of the streaming kernel on one workload (dev build libgar_dev.so: -DGAR_HXS_DEV=1):
# kernel ms per launch (HIP events) with parts of the work switched off (GAR_HXS_DBG bits: 1 no load
# issue, 2 no stores, 4 no MFMA, 8 no B reads, 16 no steady conversion, 32 compute never waits,
# 64 loaders never waits) for each roles setting.  Output values are wrong in every mode but 0.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-attr}; mkdir -p $O
D=$R/go-audio-resampler_amd/${LIB:-libgar_dev.so}
cfgs=""
for roles in ${ROLES_LIST:-0 1}; do
  for dbg in ${DBG_LIST:-0 16 1 17 2 4 12 19 32 64}; do
    cfgs="$cfgs{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT_ROLES\":\"$roles\",\"GAR_HXS_DBG\":\"$dbg\"${EXTRA:+,$EXTRA}},"
  done
done
cfgs="[${cfgs%,}]"
KB_CH=${KB_CH:-2} KB_SECONDS=${KB_SECONDS:-600} KB_IN=${KB_IN:-44100} KB_OUT=${KB_OUT:-48000} KB_Q=${KB_Q:-3} \
  timeout -k 10 ${ATTR_TIMEOUT:-500} python tools/kbench.py "$cfgs" > $O/attr.jsonl 2>&1 || { tail -5 $O/attr.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/attr.jsonl'):
    d=json.loads(l); c=d['cfg']; print('roles', c.get('GAR_HXT_ROLES'), 'dbg', c.get('GAR_HXS_DBG'), 'ms', d.get('ms'), d.get('err','')[-200:])
    for p in d.get('prof', []): print('    ', p[:260])"
exit 0
