#!/bin/bash
# One GPU call: selected GPU tests, then bench lines for WORKLOADS under each env setting in ABS
# (space-separated NAME=VALUE[,NAME=VALUE] groups; "-" = defaults).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-abb}
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    ${TESTS:-tests/test_gpu_hx.py tests/test_gpu_parity.py} > $O/tests.log 2>&1
  s=$?; echo "PYTEST_EXIT $s" >> $O/tests.log; tail -3 $O/tests.log; [ $s -eq 0 ] || exit $s
fi
for ab in ${ABS:--}; do
  envs=""; [ "$ab" != "-" ] && envs=$(echo $ab | tr ',' ' ')
  for w in ${WORKLOADS:-cfg2 ns256 cfg3}; do
    tag=$(echo "${ab}_$w" | tr '=,/' '__-')
    env $envs GAR_HX_TRACE=${TRACE:-} timeout -k 10 200 python $R/bench.py --workload $w --no-cpu-baseline --no-pmc --no-streaming ${BENCH_ARGS:-} > $O/b_$tag.json 2> $O/b_$tag.err
    s=$?; [ $s -eq 0 ] || { echo "bench $ab $w failed $s"; tail -5 $O/b_$tag.err; exit $s; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$ab', '$w', round(d['value']), d['ms_per_step'], 'kernel_ms', r.get('kernel_ms_per_launch'), 'frac', round(r['frac'],3), 'rms', d.get('rms_vs_oracle'))"
  done
done
exit 0
