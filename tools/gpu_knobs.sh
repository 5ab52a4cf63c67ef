#!/bin/bash
# Runtime-knob sweep of one workload (WL) on one box: each entry of KNOBS ("NAME=V,NAME2=V2" or "default")
# runs bench.py once per round; kernel ms per launch avg [min, median, max] to gpurun_out/$TAG/knobs.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${TAG:-knobs}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for k in $KNOBS; do
    e=""; [ "$k" = default ] || e="${k//,/ }"
    env $e timeout -k 10 200 python3 bench.py --workload ${WL:-ns256} --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline --no-pmc \
      --no-streaming --check-seconds 0 --secondary ${SEC:-none} > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
    python3 - "$O/run.json" "$k" "$r" <<'PY' | tee -a $O/knobs.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2], "round", sys.argv[3]]
for key, o in [(d["config"]["workload"], d)] + list((d.get("secondary") or {}).items()):
    r = o.get("roofline") or {}
    out += [key[:12], round(o["value"]), r.get("kernel_ms_per_launch"), r.get("kernel_ms_min_median_max")]
print(*out)
PY
  done
done
