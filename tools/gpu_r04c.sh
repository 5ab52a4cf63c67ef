#!/bin/bash
# One GPU call: GPU tests (new small-launch fast loads, bg_rt for the decimator), hxt roles A/B,
# cfg5 and the streaming (4096-frame) numbers with the defaults.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04c; mkdir -p $O
timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hx.py tests/test_gpu_parity.py tests/test_gpu_layouts.py tests/test_gpu_fullsize.py tests/test_gpu_pcm.py > $O/tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -2 $O/tests.log; [ $s -eq 0 ] || exit $s
NO_TESTS=1 WORKLOADS="cfg2 ns256 cfg3" ABS="GAR_HXT=1,GAR_HXT_ROLES=0 GAR_HXT=0 -" TRACE=1 bash tools/gpu_ab.sh || exit 1
timeout -k 10 200 python bench.py --workload cfg5 --no-cpu-baseline --no-pmc --no-streaming > $O/cfg5.json 2> $O/cfg5.err || exit 1
python3 -c "import json; d=json.loads(open('$O/cfg5.json').read().strip().splitlines()[-1]); r=d['roofline']; print('cfg5', round(d['value']), d['ms_per_step'], r.get('kernel_ms_by_kind'), 'rms', d.get('rms_vs_oracle'))"
timeout -k 10 300 python bench.py --workload cfg2 --no-cpu-baseline --no-pmc --secondary none > $O/cfg2s.json 2> $O/cfg2s.err || exit 1
python3 -c "import json; d=json.loads(open('$O/cfg2s.json').read().strip().splitlines()[-1]); print('streaming', json.dumps(d.get('streaming'))[:600])"
