#!/bin/bash
# A/B of bench workloads across library builds on one box: LIBS="a.so b.so", WL=primary, SEC=secondaries,
# ROUNDS interleaved rounds; one JSON summary line per run under gpurun_out/$TAG/ab.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-ab}; mkdir -p $O; cd $R
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS}; do
    GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 300 python3 bench.py --workload ${WL:-cfg2} --steps ${STEPS:-10} --warmup 3 \
      --no-cpu-baseline --no-pmc --no-streaming --check-seconds 0 --secondary ${SEC:-none} > $O/run.json 2> $O/run.err || { tail -20 $O/run.err; exit 1; }
    python3 - "$O/run.json" "$lib" "$r" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2], "round", sys.argv[3]]
for k, o in [(d["config"]["workload"], d)] + list((d.get("secondary") or {}).items()):
    r = o.get("roofline") or {}
    out += [k, o["value"], r.get("kernel_ms_per_launch"), r.get("kernel_ms_min_median_max")]
print(*out)
PY
  done
done
