#!/bin/bash
# r06f: final round-6 run -- all -m gpu tests + smoke, the driver's bench command, rocprof kernel stats,
# PMC (cfg2, ns256), then cfg3 on one-wave-per-row-block roles (GAR_HXT_ROLES=0, which lets it take
# 32-channel blocks) against its default, two interleaved rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=r06f PMC_WL="cfg2 ns256" bash tools/gpu_run.sh || exit $?
O=gpurun_out/r06f_cfg3roles; mkdir -p $O
for r in 1 2; do
  for roles in default 0; do
    if [ $roles = default ]; then e=""; else e="GAR_HXT_ROLES=0"; fi
    env $e timeout -k 10 200 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline --no-pmc --no-streaming \
      --check-seconds 2 --secondary none > $O/run.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/run.json').read().strip().splitlines()[-1]); r=d['roofline']; print('roles', '$roles', 'round', $r, d['value'], r.get('kernel_ms_per_launch'), r.get('kernel_ms_min_median_max'), 'rms', d.get('rms_vs_oracle'))" | tee -a $O/ab.txt
  done
done
