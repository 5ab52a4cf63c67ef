#!/bin/bash
# cfg5 chunk probes: bg_rb_kernel B-fetch paths (GAR_BG_DBG 128: branch-free gathers for every
# column, 256: branchy srcRead for every column, 16: no B loads)
O=$GRAFT_REPO_ROOT/gpurun_out; L=$O/cfg5_reuse.log; : > $L
for v in "GAR_BG_DBG=0" "GAR_BG_DBG=128" "GAR_BG_DBG=256" "GAR_BG_DBG=16"; do
  echo "== $v" >> $L
  env $v P_N=300 timeout -k 10 60 python tools/cfg5_probe.py 2>&1 | grep "kind\|no-profile" >> $L || exit 1
done
