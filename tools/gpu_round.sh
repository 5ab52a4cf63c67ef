#!/bin/bash
# One GPU call: GPU tests, smoke, bench, kernel sweep. Stops at the first fault/abort/timeout.
mkdir -p gpurun_out
ok() { local s=$1; [ "$s" -eq 0 ] || [ "$s" -eq 1 ]; }
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> gpurun_out/gpu_tests.log; ok $s || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
s=$?; echo "SMOKE_EXIT $s" >> gpurun_out/smoke.log; ok $s || exit $s
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
s=$?; echo "BENCH_EXIT $s" >> gpurun_out/bench.log; ok $s || exit $s
if [ -n "$DO_PMC" ]; then
  bash tools/pmc.sh; s=$?; echo "PMC_EXIT $s" > gpurun_out/pmc_exit.log; [ $s -eq 0 ] || exit $s
fi
if [ -n "$KB_SWEEP" ]; then
  timeout -k 10 600 python tools/kbench.py "$KB_SWEEP" > gpurun_out/kbench.log 2>&1
  s=$?; echo "KB_EXIT $s" >> gpurun_out/kbench.log
fi
exit 0
