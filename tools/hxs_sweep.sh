#!/bin/bash
# Attribution sweep of the streaming kernel: env settings per line of $1 (or defaults).
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 100 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --check-seconds 0 > gpurun_out/sw.log 2>&1 || { echo "FAIL $1"; tail -3 gpurun_out/sw.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
}
for cfg in "${@:-GAR_HXS_DBG=0}"; do run "$cfg" || exit 1; done
