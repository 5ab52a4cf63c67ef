#!/bin/bash
O=$GRAFT_REPO_ROOT/gpurun_out; L=$O/cfg5_dbg.log; : > $L
for v in 0 2 16 32 48 64 114; do
  echo "== GAR_BG_DBG=$v" >> $L
  GAR_BG_DBG=$v P_N=300 timeout -k 10 60 python tools/cfg5_probe.py 2>&1 | grep "kind\|no-profile" >> $L || exit 1
done
