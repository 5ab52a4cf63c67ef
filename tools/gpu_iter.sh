#!/bin/bash
# Kernel iteration in one GPU call: selected GPU tests (TESTS, default the split-f16 + parity files), then
# short bench lines (WORKLOADS, default cfg2 ns256) without CPU baseline / PMC.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/it
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    ${TESTS:-tests/test_gpu_hx.py tests/test_gpu_parity.py} > $O/tests.log 2>&1
  s=$?; echo "PYTEST_EXIT $s" >> $O/tests.log; tail -3 $O/tests.log; [ $s -eq 0 ] || exit $s
fi
for w in ${WORKLOADS:-cfg2 ns256}; do
  GAR_HX_TRACE=${TRACE:-} timeout -k 10 200 python $R/bench.py --workload $w --no-cpu-baseline --no-pmc --no-streaming ${BENCH_ARGS:-} > $O/bench_$w.json 2> $O/bench_$w.err
  s=$?; [ $s -eq 0 ] || { echo "bench $w failed $s"; tail -5 $O/bench_$w.err; exit $s; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$w', round(d['value']), d['ms_per_step'], 'kernel_ms', r.get('kernel_ms_per_launch'), 'frac', round(r['frac'],3), 'rms', d.get('rms_vs_oracle'))"
done
exit 0
