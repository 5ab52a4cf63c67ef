#!/bin/bash
# Attribution runs of the streaming kernel (dev build libgar_dev.so, GAR_HXS_DBG modes: 1 no steady loads,
# 2 no stores, 4 no MFMA, 8 no B reads, 16 no conversion; outputs wrong by design): kernel ms per launch
# of workload $WL for each mode in $MODES (DBGVAR: the knob, default GAR_HXS_DBG; GAR_BG_DBG for the f64 kernels: 2 no stores,
# 16 no B loads, 32 no A loads, 64 no history keep).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-dbg}; mkdir -p $O; cd $R
for m in ${MODES:-0 16}; do
  env ${DBGVAR:-GAR_HXS_DBG}=$m GAR_LIB_PATH=$R/go-audio-resampler_amd/${LIB:-libgar_dev.so} timeout -k 10 300 python3 bench.py --workload ${WL:-ns256} \
    --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-pmc --no-streaming --check-seconds 0 --secondary none > $O/run.json 2> $O/run.err || { tail -20 $O/run.err; exit 1; }
  python3 - "$O/run.json" "$m" <<'PY' | tee -a $O/modes.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print("mode", sys.argv[2], d["config"]["workload"], "kernel_ms", r.get("kernel_ms_per_launch"), r.get("kernel_ms_min_median_max"))
PY
done
