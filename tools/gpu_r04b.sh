#!/bin/bash
# One GPU call: hxt vs hxs A/B (cfg2 ns256 cfg3), cfg5 small-launch kernels (GAR_BG_RT 0 rb / 1 rt / 2 rc)
# with the f64 parity tests, then hxt attribution on the dev build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04b; mkdir -p $O
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_HXT=1 GAR_HXT=1,GAR_HXT_ROLES=0 GAR_HXT=0" bash tools/gpu_ab.sh || exit 1
for rt in 1 2; do
  GAR_BG_RT=$rt timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "f64 or cfg5 or chunking or multistage or fixture" > $O/tests_rt$rt.log 2>&1
  s=$?; echo "rt=$rt PYTEST_EXIT $s"; tail -2 $O/tests_rt$rt.log; [ $s -eq 0 ] || exit $s
done
for rt in 0 1 2; do
  GAR_BG_RT=$rt GAR_BG_TRACE=1 timeout -k 10 200 python bench.py --workload cfg5 --no-cpu-baseline --no-pmc --no-streaming > $O/cfg5_rt$rt.json 2> $O/cfg5_rt$rt.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/cfg5_rt$rt.json').read().strip().splitlines()[-1]); r=d['roofline']; print('rt=$rt cfg5', round(d['value']), d['ms_per_step'], r.get('kernel_ms_by_kind'), 'rms', d.get('rms_vs_oracle'))"
done
bash tools/gpu_attr4.sh
